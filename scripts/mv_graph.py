"""hipGraph period of back-to-back mat-vec calls (n launches captured in one graph): the
launch-bound form a decode graph and the reference perf harness run. Two weight regimes: 'warm'
(2 rotated copies: resident in the 256 MB Infinity Cache, as test-backend-ops perf reuses one
tensor) and 'cold' (enough rotated copies to exceed it, as a model's decode pass).
usage: python scripts/mv_graph.py [--cold|--warm|--both] type:K:N:M ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

M = bench.M
TYPES = {"q4_0": M.Q4_0, "q8_0": M.Q8_0, "q4_K": M.Q4_K, "q5_K": M.Q5_K, "q6_K": M.Q6_K}
M.build()
args = sys.argv[1:]
mode = "both"
if args and args[0].startswith("--"):
    mode = args.pop(0)[2:]
tag = " ".join(f"{k}={os.path.basename(v) if k == 'GGML_MI355X_LIB' else v}" for k, v in os.environ.items()
               if k.startswith("GGML_MI355X_")) or "default"
for sh in args:
    tn, K, N, Mc = sh.split(":")
    t, K, N, Mc = TYPES[tn], int(K), int(N), int(Mc)
    res = []
    for regime in (("warm", "cold") if mode == "both" else (mode,)):
        one = M.row_size(t, K) * N
        copies = 2 if regime == "warm" else max(2, (320 << 20) // one + 1)
        s = bench.MatVecSet(torch, t, K, N, Mc, 1, copies)
        us = min(s.graph_period_us(max(32, copies)) for _ in range(3))
        res.append(f"{regime} {us:8.2f} us {s.bytes / us / 1e3:7.1f} GB/s")
        del s
        torch.cuda.empty_cache()
    print(f"{tag:32s} {sh:20s} " + "  ".join(res), flush=True)
