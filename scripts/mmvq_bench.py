"""Mat-vec timing probe: per-launch device time of one MUL_MAT over `batch` stacked matrices
(events around back-to-back launches, 2 rotated copies of the stack -> HBM-cold).
Usage: python scripts/mmvq_bench.py [type:K:N:M:batch ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

M = bench.M
TYPES = {"q4_0": M.Q4_0, "q8_0": M.Q8_0, "q4_K": M.Q4_K, "q5_K": M.Q5_K, "q6_K": M.Q6_K}
shapes = sys.argv[1:] or ["q4_0:4096:4096:1:64", "q4_K:4096:4096:1:64", "q6_K:4096:11008:1:24", "q8_0:4096:4096:1:64"]
M.build()
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("GGML_MI355X_"))
for sh in shapes:
    tn, K, N, Mc, b = sh.split(":")
    s = bench.MatVecSet(torch, TYPES[tn], int(K), int(N), int(Mc), int(b), 2)
    s.launch(0)
    torch.cuda.synchronize()
    us = min(s.launch_us(20) for _ in range(3))
    print(f"{tag:30s} {sh:24s} {us:9.2f} us  {s.bytes / us / 1e3:8.1f} GB/s  {s.bytes / us / 1e3 / 80:5.1f}% of 8 TB/s", flush=True)
    del s
    torch.cuda.empty_cache()
