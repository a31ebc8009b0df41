"""GPU parity of the single-wave mat-vec (csrc/mmvq_solo.hip, GGML_MI355X_SOLO): one column, one
matrix, K <= 4096 with K % 64 == 0. Each lane quantizes its own slot of the column in registers
with the arithmetic of the 8-wave kernel (mmvq_impl.h xblock_store), so against that kernel
(SOLO=0, same activation blocks, same block dots) only the order of the cross-lane row sum can
differ: NMSE <= 1e-10; against the CPU oracle the reference's MUL_MAT bar 5e-4
(tests/test-backend-ops.cpp:3106-3108). Rows per wave 2 / 4 / 8, ragged N, K from one slot to the
full 64 slots, all five types (Q6_K's slots interleave four half-blocks: the amax exchange with
lane ^ 1)."""
import numpy as np
import pytest

import golden_cases as G
import qref
from test_gpu_parity import mm, run_mul_mat  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

TYPES = [qref.Q4_0, qref.Q8_0, qref.Q4_K, qref.Q5_K, qref.Q6_K]


def operands(t, N, K, seed):
    w = qref.quantize(t, qref.fill_uniform(N * K, seed), n_per_row=K)
    x = qref.fill_uniform(K, seed + 1)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, 1, 1, 1], qref.contiguous_nb(qref.F32, [K, 1, 1, 1]))
    return a, b, [N, 1, 1, 1]


@pytest.mark.parametrize("rows", [1, 2, 8])
@pytest.mark.parametrize("K", [64, 256, 768, 2048, 4096])
@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
def test_solo_vs_kernel_and_oracle(mm, t, K, rows):
    if qref.BLCK[t] == 256 and K % 256:
        K = 256 * max(1, K // 256)
    a, b, out_ne = operands(t, 301, K, 7 + K)
    with mm.knobs(GGML_MI355X_SOLO=rows):
        got = run_mul_mat(mm, a, b, out_ne)
    with mm.knobs(GGML_MI355X_SOLO=0):
        ref = run_mul_mat(mm, a, b, out_ne)
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, ref) <= 1e-10
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne)) <= 5e-4


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
def test_solo_north_star_shape_repeatable(mm, t):
    """the 4096 x 4096 single launch: against the 8-wave kernel and bitwise repeatable"""
    a, b, out_ne = operands(t, 4096, 4096, 3)
    with mm.knobs(GGML_MI355X_SOLO=1):
        g1 = run_mul_mat(mm, a, b, out_ne)
        g2 = run_mul_mat(mm, a, b, out_ne)
    with mm.knobs(GGML_MI355X_SOLO=0):
        ref = run_mul_mat(mm, a, b, out_ne)
    assert np.array_equal(g1.view(np.uint32), g2.view(np.uint32))
    assert qref.nmse(g1, ref) <= 1e-10
