"""Diagnostics: phase timeline of the two-launch GPT-2 layer (gpt2_block.hip) from its
s_memrealtime stamps (GGML_MI355X_STAMPS=1; 100 MHz). Per layer kind, the median over steps and
workgroups of each phase's offset from the workgroup's start, the kernel span (first start ->
last end) and the gap between one kernel's last end and the next kernel's first start.
Usage: python scripts/block_stamps.py [steps] [pos0]"""
import ctypes as C
import os
import sys

os.environ["GGML_MI355X_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ggml-gfx906_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpt2 as G  # noqa: E402
import mi355x_qmm as M  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 24
pos0 = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.cuda.set_device(0)
hp = G.make_hparams(M.Q4_0)
st = G.Stage(hp)
st.fill_synthetic(1234)
c = G.Context(st, 1)
s = torch.cuda.Stream()
L = M.lib()
L.ggml_mi355x_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
NL = hp["n_layer"]
NWG = [hp["n_head"], 4 * hp["n_embd"] // 256]
NPH = [7, 6]
buf = np.zeros(2 * NL * 64 * 16, np.uint64)
ph = {0: [], 1: []}
spans = {0: [], 1: []}
gaps = []
clk = []
extra = []
extra1 = []
with torch.cuda.stream(s):
    z = torch.full((1,), pos0, dtype=torch.int32, device="cuda")
    c.set_pos(z.data_ptr(), s.cuda_stream)
    c.set_tokens((z * 0 + 40).data_ptr(), s.cuda_stream)
    for step in range(steps):
        c.decode(s.cuda_stream, True)
        torch.cuda.synchronize()
        if step < 4:
            continue
        L.ggml_mi355x_debug_stamps(buf.ctypes.data, buf.size)
        t = buf.reshape(NL, 2, 64, 16).astype(np.int64)
        prev_end = None
        for layer in range(NL):
            for k in (0, 1):
                w = t[layer, k, :NWG[k], :NPH[k]]
                if k == 0:
                    extra.append((t[layer, 0, :NWG[0]][:, [8, 9, 11]] - t[layer, 0, :NWG[0], 0:1]) * 10)
                else:
                    extra1.append((t[layer, 1, :NWG[1]][:, [8, 9, 11]] - t[layer, 1, :NWG[1], 0:1]) * 10)
                start = w[:, 0:1]
                ph[k].append((w - start) * 10)
                spans[k].append((w[:, NPH[k] - 1].max() - w[:, 0].min()) * 10)
                if prev_end is not None:
                    gaps.append((w[:, 0].min() - prev_end) * 10)
                prev_end = w[:, NPH[k] - 1].max()
                if k == 1:
                    mt = t[layer, 1, :NWG[1], 7] - t[layer, 1, :NWG[1], 6]
                    rt = t[layer, 1, :NWG[1], 5] - t[layer, 1, :NWG[1], 0]
                    clk.append(np.median(mt / np.maximum(rt, 1)) * 100.0)
names = {0: ["start", "x arrived", "LN+quant", "qkv done", "attn loop done", "merged+quant", "end"],
         1: ["start", "x arrived", "LN+quant", "fc done", "h quantized", "end"]}
print(f"pos {pos0}..{pos0 + steps}: n_embd {hp['n_embd']}, heads {hp['n_head']}")
for k, nm in ((0, "attn block"), (1, "mlp block")):
    a = np.concatenate(ph[k])
    med = np.median(a, axis=0)
    p90 = np.percentile(a, 90, axis=0)
    print(f"{nm}: span median {np.median(spans[k]):.0f} ns")
    for i, n in enumerate(names[k]):
        print(f"   {n:16s} +{med[i]:7.0f} ns (p90 {p90[i]:7.0f})")
print(f"kernel gaps (last end -> next first start): median {np.median(gaps):.0f} ns, p90 {np.percentile(gaps, 90):.0f}")
print(f"in-kernel shader clock (mlp block, s_memtime / s_memrealtime): median {np.median(clk):.0f} MHz")
ex = np.median(np.concatenate(extra), axis=0)
print(f"attn block: loads issued +{ex[0]:.0f} ns, wave 0's first residual row landed +{ex[1]:.0f} ns, "
      f"its last q/k/v weights landed +{ex[2]:.0f} ns")
ex = np.median(np.concatenate(extra1), axis=0)
print(f"mlp block: loads issued +{ex[0]:.0f} ns, wave 0's fc weights landed +{ex[1]:.0f} ns, fc computed (wave 0) +{ex[2]:.0f} ns")
