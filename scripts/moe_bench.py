"""MUL_MAT_ID timing probe: E experts [K, N] of one type, U experts per token, T tokens;
hipGraph period of back-to-back calls. GGML_MI355X_MMQ_ID_MIN selects the path (pairs at which
the grouped MFMA path takes over; a huge value forces one mat-vec per pair).
Usage: python scripts/moe_bench.py type:K:N:E:U:T ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

M = bench.M
TYPES = {"q4_0": M.Q4_0, "q8_0": M.Q8_0, "q4_K": M.Q4_K, "q5_K": M.Q5_K, "q6_K": M.Q6_K}
M.build()
tag = os.environ.get("GGML_MI355X_MMQ_ID_MIN", "default") + "/" + os.environ.get("GGML_MI355X_MMQ", "i8")
for sh in sys.argv[1:] or ["q4_K:4096:11008:8:2:512", "q4_0:4096:4096:64:8:256"]:
    tn, K, N, E, U, T = sh.split(":")
    t, K, N, E, U, T = TYPES[tn], int(K), int(N), int(E), int(U), int(T)
    w = torch.from_numpy(np.tile(bench.synthetic_weights(t, N, K, 7).reshape(-1), E)).cuda()
    x = torch.rand((T, U, K), device="cuda") * 2 - 1
    rng = np.random.default_rng(1)
    ids = torch.from_numpy(np.stack([rng.permutation(E)[:U] for _ in range(T)]).astype(np.int32)).cuda()
    y = torch.empty((T, U, N), device="cuda")
    A = M.tensor(t, w.data_ptr(), [K, N, E, 1], M.contiguous_nb(t, [K, N, E]))
    B = M.tensor(M.F32, x.data_ptr(), [K, U, T, 1], M.contiguous_nb(M.F32, [K, U, T]))
    I = M.tensor(M.I32, ids.data_ptr(), [U, T, 1, 1], M.contiguous_nb(M.I32, [U, T]))
    D = M.tensor(M.F32, y.data_ptr(), [N, U, T, 1], M.contiguous_nb(M.F32, [N, U, T]))
    s = torch.cuda.Stream()
    M.mul_mat_id(A, B, I, D, s)     # eager first: the stream's scratch grows outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(4):
            M.mul_mat_id(A, B, I, D, s)
    g.replay()
    torch.cuda.synchronize()
    a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a_.record()
    for _ in range(5):
        g.replay()
    b_.record()
    torch.cuda.synchronize()
    us = a_.elapsed_time(b_) * 1e3 / 20
    flops = 2.0 * K * N * U * T
    print(f"min_pairs={tag:10s} {sh:28s} {us:10.1f} us  {flops / us / 1e6:8.1f} TFLOP/s", flush=True)
