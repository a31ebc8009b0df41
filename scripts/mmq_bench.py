"""Mat-mat (MMQ) timing probe: mean device time of one MUL_MAT (activation conversion + tile
kernel) for the shapes given, HBM-cold (24 rotated weight copies). Tile shape via
GGML_MI355X_MMQ_TILE. Usage: python scripts/mmq_bench.py [type:K:N:M ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

M = bench.M
TYPES = {"q4_0": M.Q4_0, "q8_0": M.Q8_0, "q4_K": M.Q4_K, "q5_K": M.Q5_K, "q6_K": M.Q6_K}
shapes = sys.argv[1:] or ["q8_0:4096:4096:512", "q4_K:4096:4096:512", "q4_0:4096:4096:512",
                          "q6_K:4096:11008:512", "q4_K:4096:4096:128", "q8_0:4096:4096:2048"]
M.build()
tile = os.environ.get("GGML_MI355X_MMQ_TILE", "auto")
if os.environ.get("MMQ_REPACKED") == "1":
    tile = "repacked"
elif os.environ.get("GGML_MI355X_MMQ_REPACK_MIN"):
    tile = "rp_call"
for sh in shapes:
    tn, K, N, Mc = sh.split(":")
    s = bench.MatVecSet(torch, TYPES[tn], int(K), int(N), int(Mc), 1, 24, repacked=os.environ.get("MMQ_REPACKED") == "1")
    s.launch(0)
    torch.cuda.synchronize()
    ev_us = s.launch_us(24)
    us = s.graph_period_us(24)   # back-to-back launches in one hipGraph: no host gaps
    print(f"tile={tile:8s} {sh:22s} {us:9.2f} us  {s.flops / us / 1e6:8.1f} TFLOP/s  "
          f"{s.bytes / us / 1e3:8.1f} GB/s  (events {ev_us:.2f} us)", flush=True)
    del s
    torch.cuda.empty_cache()
