"""Diagnostics: per-workgroup timeline of ONE fused mat-vec of the GPT-2 decode step
(GGML_MI355X_STAMP_MV = its index: 4 per layer in the order c_attn, c_proj, c_fc, mlp c_proj;
48 = lm_head). s_memrealtime (100 MHz) stamps: start, activations quantized (after the LDS
barrier), end. Usage: python scripts/gpt2_stamps.py INDEX [steps]"""
import ctypes as C
import os
import sys

idx = int(sys.argv[1]) if len(sys.argv) > 1 else 2
os.environ["GGML_MI355X_STAMPS"] = "1"
os.environ["GGML_MI355X_STAMP_MV"] = str(idx)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ggml-gfx906_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpt2 as G  # noqa: E402
import mi355x_qmm as M  # noqa: E402

torch.cuda.set_device(0)
hp = G.make_hparams(M.Q4_0)
st = G.Stage(hp)
st.fill_synthetic(1234)
c = G.Context(st, 1)
s = torch.cuda.Stream()
L = M.lib()
L.ggml_mi355x_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
# GGML_MI355X_GPT2_BLOCK unset (two-launch layers): the only fused mat-vec of a step is lm_head
block = os.environ.get("GGML_MI355X_GPT2_BLOCK", "1") != "0"
N = 50257 if block or idx >= 48 else [2304, 768, 3072, 768][idx % 4]
nwg = 256 if N == 50257 else min(2048, (N + 31) // 32)   # lm_head: resident-size grid (mmvq_fused.hip)
buf = np.zeros(4 * 65536 + 4 * 8 * nwg, np.uint64)
res = []
wres = []
with torch.cuda.stream(s):
    z = torch.zeros(1, dtype=torch.int32, device="cuda")
    c.set_pos(z.data_ptr(), s.cuda_stream)
    c.set_tokens((z + 40).data_ptr(), s.cuda_stream)
    for step in range(int(sys.argv[2]) if len(sys.argv) > 2 else 40):
        c.decode(s.cuda_stream, True)
        torch.cuda.synchronize()
        if step < 4:
            continue
        L.ggml_mi355x_debug_stamps(buf.ctypes.data, buf.size)
        t = buf[:8 * nwg].reshape(nwg, 8).astype(np.int64)
        wv = buf[4 * 65536:].reshape(nwg, 8, 4).astype(np.int64)
        t0 = t[:, 0].min()
        wres.append(((wv[:, :, 0] - t[:, 0:1]) * 10, (wv[:, :, 1] - t[:, 0:1]) * 10, (wv[:, :, 2] - t[:, 0:1]) * 10))
        res.append(((t[:, 0] - t0) * 10, (t[:, 1] - t[:, 0]) * 10, (t[:, 2] - t[:, 1]) * 10, (t[:, 2].max() - t0) * 10, (t[:, 6] - t[:, 0]) * 10))
st_off = np.concatenate([r[0] for r in res])
pro = np.concatenate([r[1] for r in res])
body = np.concatenate([r[2] for r in res])
span = np.array([r[3] for r in res])
print(f"mat-vec #{idx}: N={N} workgroups={nwg}")
print(f"  span first start -> last end (ns): median {np.median(span):.0f}  min {span.min():.0f}")
print(f"  WG start offset (ns): median {np.median(st_off):.0f}  p90 {np.percentile(st_off, 90):.0f}  max {st_off.max():.0f}")
xin = np.concatenate([r[4] for r in res])
print(f"  start -> activations arrived (ns): median {np.median(xin):.0f}  p90 {np.percentile(xin, 90):.0f}")
print(f"  start -> activations in LDS (ns): median {np.median(pro):.0f}  p90 {np.percentile(pro, 90):.0f}")
print(f"  LDS ready -> end (ns): median {np.median(body):.0f}  p90 {np.percentile(body, 90):.0f}")
ws = np.concatenate([w[0].ravel() for w in wres])
wx = np.concatenate([w[1].ravel() for w in wres])
wq = np.concatenate([w[2].ravel() for w in wres])
wmax = np.concatenate([w[2].max(1) for w in wres])
print(f"  per wave, rel. to its WG's wave-0 start (ns): start median {np.median(ws):.0f} max {ws.max():.0f};"
      f" x arrived median {np.median(wx):.0f} p90 {np.percentile(wx, 90):.0f};"
      f" at barrier median {np.median(wq):.0f}; last wave of the WG at barrier median {np.median(wmax):.0f}")
