#!/usr/bin/env python3
"""scripts/solo_stamps.py — diagnostic: per-wave phase stamps of one single-wave mat-vec launch
(csrc/mmvq_solo.hip) inside a back-to-back run of single-matrix launches (64 rotated copies):
start offsets, activations in registers, quantized, end (s_memrealtime, 100 MHz).
  python scripts/solo_stamps.py [type] [K] [N]"""
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

tname = sys.argv[1] if len(sys.argv) > 1 else "q4_K"
t = {v: k for k, v in M.NAMES.items()}[tname]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
R = 4 if tname == "q6_K" else 8
L = M.lib()
L.ggml_mi355x_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
g = bench.MatVecSet(torch, t, K, N, 1, 1, 64)
g.launch(0)
torch.cuda.synchronize()
nw = (N + R - 1) // R
buf = np.zeros(8 * nw, np.uint64)
rows = []
for i in range(16):
    for j in range(63):
        g.launch(i + j)
    torch.cuda.synchronize()
    L.ggml_mi355x_debug_stamps(buf.ctypes.data, buf.size)
    s = buf.reshape(nw, 8).astype(np.int64)
    t0 = s[:, 0].min()
    rows.append([(s[:, 3].max() - t0) * 10, np.median((s[:, 0] - t0) * 10), np.max((s[:, 0] - t0) * 10),
                 np.median((s[:, 1] - s[:, 0]) * 10), np.median((s[:, 2] - s[:, 1]) * 10), np.median((s[:, 3] - s[:, 2]) * 10),
                 np.median((s[:, 3] - s[:, 0]) * 10), np.median((s[:, 5] - s[:, 4]) / np.maximum(1, (s[:, 3] - s[:, 0]) * 10))])
r = np.median(np.array(rows), axis=0)
print(f"{tname} K={K} N={N} M=1: {nw} single-wave workgroups of {R} rows")
print(f"  kernel span (first start -> last end) ns: {r[0]:.0f};  start offsets median {r[1]:.0f}, max {r[2]:.0f}")
print(f"  per wave median ns: start->activations in registers {r[3]:.0f}  ->quantized {r[4]:.0f}  ->end {r[5]:.0f}"
      f"  (lifetime {r[6]:.0f}, shader clock {r[7]:.2f} GHz)")
