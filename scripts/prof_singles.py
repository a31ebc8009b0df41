"""Single-matrix launches for rocprofv3 --kernel-trace --stats: each BASELINE mat-vec config
as ONE MUL_MAT per launch, cold (64 rotated weight copies, > 256 MB Infinity Cache) and hot
(one copy, re-read from the Infinity Cache). The kernel trace then gives the true per-launch
kernel duration that hipGraph periods and events cannot separate from the launch boundary.
Usage: python scripts/prof_singles.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

M = bench.M
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 128
only = sys.argv[2] if len(sys.argv) > 2 else None   # e.g. "q4_0:4096:64" = type:N:copies
M.build()
torch.cuda.set_device(0)
for name, t, K, N in (("q4_0", M.Q4_0, 4096, 4096), ("q4_K", M.Q4_K, 4096, 4096), ("q4_K", M.Q4_K, 4096, 11008),
                      ("q5_K", M.Q5_K, 4096, 11008), ("q6_K", M.Q6_K, 4096, 11008)):
    for copies in (64, 1):
        if only and only != f"{name}:{N}:{copies}":
            continue
        s = bench.MatVecSet(torch, t, K, N, 1, 1, copies)
        s.launch(0)
        torch.cuda.synchronize()
        us = s.launch_us(reps)
        print(f"{name} K={K} N={N} copies={copies}: events {us:.3f} us/launch, "
              f"{s.bytes / us / 1e3:.1f} GB/s", flush=True)
        del s
        torch.cuda.empty_cache()
