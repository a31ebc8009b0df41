"""int8 MFMA mat-mat debugging probe: one-hot activations make dst[t][r] = w[r][t] (dequantized),
so index-mapping errors show up as permutations. Usage: python scripts/mmq8_debug.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ggml-gfx906_amd")):
    sys.path.insert(0, p)
os.environ["GGML_MI355X_MMQ"] = "i8"
import torch  # noqa: E402

import golden_cases as G  # noqa: E402
import qref  # noqa: E402
from test_gpu_parity import run_mul_mat  # noqa: E402
import mi355x_qmm as M  # noqa: E402

M.build()
np.set_printoptions(linewidth=200, precision=3, suppress=True)
for t in (qref.Q8_0, qref.Q4_0, qref.Q4_K):
    N, Mc, K = 64, 64, 256
    w = qref.quantize(t, qref.fill_uniform(N * K, 5), n_per_row=K)
    wd = qref.dequantize(t, w, N * K).reshape(N, K)
    x = np.zeros((Mc, K), np.float32)
    for i in range(Mc):
        x[i, (3 * i) % K] = 1.0
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x.ravel(), [K, Mc, 1, 1], qref.contiguous_nb(qref.F32, [K, Mc, 1, 1]))
    got = run_mul_mat(M, a, b, [N, Mc, 1, 1]).reshape(Mc, N)
    want = (x @ wd.T)
    print(qref.NAMES[t], "nmse", qref.nmse(got.ravel(), want.ravel()))
    print("got[0:6,0:8]\n", got[0:6, 0:8], "\nwant\n", want[0:6, 0:8])
    bad = np.abs(got - want) > 1e-3 * (np.abs(want) + 1e-3)
    blk = np.array([((3 * i) % K) // 32 for i in range(Mc)])
    print("bad count", bad.sum(), "of", bad.size)
    for bb in range(8):
        rows = bad[blk == bb]
        print(f"  block {bb}: tokens {np.nonzero(blk == bb)[0][:3].tolist()}.. bad per row-octet",
              [int(rows[:, 8 * o:8 * o + 8].sum()) for o in range(8)])
    print("bad rows per token", bad.sum(axis=1).tolist())
    if t in (qref.Q8_0, qref.Q4_0):
        bs = 34 if t == qref.Q8_0 else 18
        d = np.frombuffer(w.tobytes(), np.uint8).reshape(N, 8, bs)[:, :, :2].copy().view(np.float16)[:, :, 0].astype(np.float32)
        for (ti, ri) in ((12, 0), (12, 5), (23, 2), (33, 40)):
            b = ((3 * ti) % K) // 32
            ratio = got[ti, ri] / want[ti, ri]
            print(f"tok {ti} row {ri} blk {b}: ratio {ratio:.4f}; d ratios", (d[ri] / d[ri, b]).round(4).tolist())
    # where does want[t][r] show up in got?
    for (ti, ri) in ((0, 0), (1, 0), (0, 1), (5, 3), (33, 40)):
        v = want[ti, ri]
        hits = np.argwhere(np.abs(got - v) < 1e-3 * max(1e-6, abs(v)))
        print(f"want[{ti},{ri}]={v:.4f} found at", hits[:6].tolist())
