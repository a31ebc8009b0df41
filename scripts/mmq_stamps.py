"""MMQ phase breakdown (diagnostic build, GGML_MI355X_STAMPS=1): per-wave s_memtime cycles per
K-step spent issuing loads, in MFMAs, decoding weights, waiting for the DMA, at the barrier.
Usage: python scripts/mmq_stamps.py type:K:N:M"""
import ctypes as C
import os
import sys

os.environ["GGML_MI355X_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

M = bench.M
TYPES = {"q4_0": M.Q4_0, "q8_0": M.Q8_0, "q4_K": M.Q4_K, "q5_K": M.Q5_K, "q6_K": M.Q6_K}
for sh in sys.argv[1:] or ["q4_K:4096:4096:128", "q8_0:4096:4096:512"]:
    tn, K, N, Mc = sh.split(":")
    s = bench.MatVecSet(torch, TYPES[tn], int(K), int(N), int(Mc), 1, 8)
    L = M.lib()
    L.ggml_mi355x_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
    for i in range(8):
        s.launch(i)
    torch.cuda.synchronize()
    buf = np.zeros(8 * 65536, np.uint64)
    L.ggml_mi355x_debug_stamps(buf.ctypes.data, buf.size)
    st = buf.reshape(-1, 8).astype(np.int64)
    st = st[st[:, 7] > 0]
    n = st[:, 7].astype(np.float64)
    tot = (st[:, 6] - st[:, 0]) / n
    names = ["issue loads", "mfma", "decode+ds_write", "wait dma", "barrier"]
    if os.environ.get("GGML_MI355X_MMQ_TILE", "").startswith(("wave", "wl")):   # register-decode kernels
        names = ["top (ds_read issue)", "mfma+loads+decode", "wait dma", "barrier", "-"]
    print(f"{sh}: {len(st)} waves, nsteps={int(n[0])}, cycles per step (median over waves):")
    for i, nm in enumerate(names):
        print(f"   {nm:16s} {np.median(st[:, 1 + i] / n):8.1f}")
    print(f"   {'total':16s} {np.median(tot):8.1f}")
    del s
    torch.cuda.empty_cache()
