"""Diagnostic: run one int8 mat-mat shape many times and map every element that disagrees with
the oracle to its MFMA output position (32x32 tile: register r, lane l), to tell a hazard on
particular result registers from a layout fault.  python tests/diag/mmq8_positions.py [type N M K reps]"""
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ggml-gfx906_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import golden_cases as G  # noqa: E402
import mi355x_qmm as M  # noqa: E402
import qref  # noqa: E402
from test_gpu_parity import dev_bytes  # noqa: E402

tn = sys.argv[1] if len(sys.argv) > 1 else "q4_0"
N, M_, K, reps = (int(a) for a in (sys.argv[2:6] if len(sys.argv) > 5 else (512, 200, 4096, 40)))
t = {"q8_0": qref.Q8_0, "q4_0": qref.Q4_0, "q4_K": qref.Q4_K, "q5_K": qref.Q5_K, "q6_K": qref.Q6_K}[tn]
M.build()
w = qref.quantize(t, qref.fill_uniform(N * K, 1), n_per_row=K)
x = qref.fill_uniform(M_ * K, 2)
a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
want = G.oracle_mul_mat(a, b, [N, M_, 1, 1]).reshape(M_, N)
da, db = dev_bytes(w), dev_bytes(x)
A = M.tensor(t, da.data_ptr(), a.ne, a.nb)
B = M.tensor(qref.F32, db.data_ptr(), b.ne, b.nb)
out = torch.empty(M_ * N, dtype=torch.float32, device="cuda")
D = M.tensor(qref.F32, out.data_ptr(), [N, M_, 1, 1], qref.contiguous_nb(qref.F32, [N, M_, 1, 1]))
scale = np.sqrt(np.mean(want ** 2))
regs, lanes, toks, rows, nbad_runs = Counter(), Counter(), Counter(), Counter(), 0
for rep in range(reps):
    out.fill_(float("nan"))
    M.mul_mat(A, B, D)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(M_, N)
    bad = np.argwhere(~(np.abs(got - want) <= 0.05 * scale))
    if len(bad):
        nbad_runs += 1
        print(f"rep {rep}: {len(bad)} bad, e.g. tok {bad[0][0]} row {bad[0][1]} got {got[tuple(bad[0])]:.4g} want {want[tuple(bad[0])]:.4g}", flush=True)
    for tok, row in bad:
        tl, rl = tok % 32, row % 32
        r = (tl // 8) * 4 + tl % 4            # D[tok][row]: register of the 32x32 output
        lane = rl + 32 * ((tl // 4) % 2)
        regs[r] += 1
        lanes[lane] += 1
        toks[tok % 64] += 1
        rows[row % 128] += 1
print(f"{tn} N={N} M={M_} K={K}: {nbad_runs}/{reps} runs wrong")
print("by register:", dict(sorted(regs.items())))
print("by lane:", dict(sorted(lanes.items())))
print("by token % 64:", dict(sorted(toks.items())))
print("by row % 128:", dict(sorted(rows.items())))
