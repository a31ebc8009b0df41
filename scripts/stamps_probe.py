#!/usr/bin/env python3
"""scripts/stamps_probe.py — diagnostic: where does a mat-vec launch spend its time?

Runs one HBM-cold GEMV config with GGML_MI355X_STAMPS=1 and prints, over workgroups, the
s_memrealtime (100 MHz) offsets of: start, activations quantized into LDS (after the barrier),
dot products done (weights consumed), end — relative to the first workgroup's start.
  python scripts/stamps_probe.py [type] [K] [N] [M]
"""
import ctypes as C
import os
import sys

os.environ["GGML_MI355X_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import mi355x_qmm as M  # noqa: E402

tname = sys.argv[1] if len(sys.argv) > 1 else "q4_0"
t = {v: k for k, v in M.NAMES.items()}[tname]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
Mc = int(sys.argv[4]) if len(sys.argv) > 4 else 1
BATCH = int(sys.argv[5]) if len(sys.argv) > 5 else 1

L = M.lib()
L.ggml_mi355x_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
g = bench.MatVecSet(torch, t, K, N, Mc, BATCH, 64 if BATCH == 1 else 2)
g.launch(0)
torch.cuda.synchronize()
rpw = int(os.environ.get("GGML_MI355X_RPW", "0")) or (2 if N * BATCH >= 4096 and tname != "q6_K" else 1)
rows_per_wg = 8 * rpw
nwg = min((N + rows_per_wg - 1) // rows_per_wg, max(1, (1024 + BATCH - 1) // BATCH))
buf = np.zeros(4 * 65536 + nwg * 8 * 4, np.uint64)   # workgroup stamps, then per-wave stamps
wa, wq, wd = [], [], []
spans, xs, ds, es, starts, clk = [], [], [], [], [], []
for i in range(16):
    for j in range(63 if BATCH == 1 else 3):   # measure a launch inside a back-to-back run
        g.launch(i + j)
    torch.cuda.synchronize()
    L.ggml_mi355x_debug_stamps(buf.ctypes.data, buf.size)
    s = buf[:8 * nwg].reshape(nwg, 8).astype(np.int64)
    w = buf[4 * 65536:].reshape(nwg, 8, 4).astype(np.int64)   # per wave: start, x arrived, x quantized
    wa.append(np.median((w[:, :, 1] - w[:, :, 0]) * 10))
    wq.append(np.median((w[:, :, 2] - w[:, :, 1]) * 10))
    wd.append(np.median((w[:, :, 3] - w[:, :, 2]) * 10))
    clk.append(np.median((s[:, 5] - s[:, 4]) / np.maximum(1, (s[:, 3] - s[:, 0]) * 10)))
    t0 = s[:, 0].min()
    spans.append((s[:, 3].max() - t0) * 10)
    starts.append(np.percentile((s[:, 0] - t0) * 10, [50, 100]))
    xs.append(np.median((s[:, 1] - s[:, 0]) * 10))
    ds.append(np.median((s[:, 2] - s[:, 1]) * 10))
    es.append(np.median((s[:, 3] - s[:, 2]) * 10))
print(f"{tname} K={K} N={N} M={Mc} batch={BATCH}: workgroups(x)={nwg}")
print(f"  kernel span (first start -> last end) ns: median {np.median(spans):.0f}  min {np.min(spans):.0f}")
print(f"  start offsets ns (median, max over WGs): {np.median(starts, axis=0)}")
print(f"  shader clock during the workgroup (memtime/realtime): {np.median(clk):.2f} GHz")
print(f"  per-WG median ns: start->x_ready {np.median(xs):.0f}  x_ready->end {np.median(ds):.0f}")
print(f"  per-wave median ns: start->activations in registers {np.median(wa):.0f}  ->quantized {np.median(wq):.0f}"
      f"  ->dots stored {np.median(wd):.0f}")
