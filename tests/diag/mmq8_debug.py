"""Diagnostic: int8 mat-mat (GGML_MI355X_MMQ=i8) vs the oracle on small shapes, per type, with
the error split by token / row so a layout fault shows its pattern."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ggml-gfx906_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
os.environ["GGML_MI355X_MMQ"] = "i8"
import torch  # noqa: E402,F401

import golden_cases as G  # noqa: E402
import mi355x_qmm as M  # noqa: E402
import qref  # noqa: E402
import test_gpu_parity as T  # noqa: E402

M.build()
shapes = [tuple(map(int, a.split('x'))) for a in os.environ.get('SHAPES', '64x64x256 128x64x512 256x128x1024 200x100x1536').split()]
for t in [qref.TYPE_BY_NAME[n] for n in os.environ.get('TYPES', 'q8_0 q4_0 q4_K q5_K q6_K').split()] if hasattr(qref, 'TYPE_BY_NAME') else [{'q8_0': qref.Q8_0, 'q4_0': qref.Q4_0, 'q4_K': qref.Q4_K, 'q5_K': qref.Q5_K, 'q6_K': qref.Q6_K}[n] for n in os.environ.get('TYPES', 'q8_0 q4_0 q4_K q5_K q6_K').split()]:
    for N, M_, K in shapes:
        w = qref.quantize(t, qref.fill_uniform(N * K, 1), n_per_row=K)
        x = qref.fill_uniform(M_ * K, 2)
        a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
        b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
        got = T.run_mul_mat(M, a, b, [N, M_, 1, 1]).reshape(M_, N)
        want = G.oracle_mul_mat(a, b, [N, M_, 1, 1]).reshape(M_, N)
        err = qref.nmse(got, want)
        print(f"{qref.NAMES[t]:5s} N={N} M={M_} K={K} nmse {err:.3e}", flush=True)
        if err > float(os.environ.get('SHOW', '1e-3')):
            tok_err = np.sqrt(((got - want) ** 2).mean(1) / (want ** 2).mean())
            row_err = np.sqrt(((got - want) ** 2).mean(0) / (want ** 2).mean())
            print("  got[0,:6] ", got[0, :6])
            print("  want[0,:6]", want[0, :6])
            print("  per-token rel err (first 16):", np.round(tok_err[:16], 3))
            print("  per-row rel err (first 40):", np.round(row_err[:40], 3))
            ratio = np.median(got / np.where(want == 0, 1, want))
            print("  median got/want", ratio)
            e = np.abs(got - want)
            for f in np.argsort(e.ravel())[::-1][:12]:
                tk, rw = divmod(int(f), N)
                print(f"  worst tok {tk} row {rw}: got {got[tk, rw]:.4f} want {want[tk, rw]:.4f}")
