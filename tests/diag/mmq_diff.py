"""Test-side diagnostic (imports the oracle as the checker). Error map of one golden MUL_MAT record on the current mat-mat tile (GGML_MI355X_MMQ_TILE):
per-token and per-row error against the threaded oracle, to localize a tile bug.
Usage: python tests/diag/mmq_diff.py record_name"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "ggml-gfx906_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_cases as G  # noqa: E402
import test_gpu_parity as T  # noqa: E402
import mi355x_qmm as M  # noqa: E402

M.build()
for name in sys.argv[1:]:
    r = [x for x in G.manifest() if x.get("name") == name][0]
    a, b, out_ne = G.mul_mat_operands(r)
    got = T.run_mul_mat(M, a, b, out_ne).reshape(-1, out_ne[0])
    reps = [T.run_mul_mat(M, a, b, out_ne).reshape(-1, out_ne[0]) for _ in range(4)]
    print("  run-to-run max |diff|:", [float(np.abs(x - got).max()) for x in reps])
    want = G.oracle_mul_mat(a, b, out_ne, threads=16).reshape(-1, out_ne[0])
    err = (got - want) ** 2
    den = (want ** 2).mean()
    tok = err.mean(1) / den
    row = err.mean(0) / den
    print(name, "shape (tokens, rows)", got.shape, "nmse", err.mean() / den)
    print("  worst tokens", np.argsort(tok)[-8:], np.sort(tok)[-8:])
    print("  worst rows  ", np.argsort(row)[-8:], np.sort(row)[-8:])
    print("  token nmse by tile of 32:", [f"{tok[i:i + 32].mean():.1e}" for i in range(0, len(tok), 32)])
    print("  row nmse by 32:", [f"{row[i:i + 32].mean():.1e}" for i in range(0, len(row), 32)])
