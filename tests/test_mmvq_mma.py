"""GPU parity of the int8-MFMA mat-vec for 1..8 src1 columns (csrc/mmvq_mma.hip).

The path quantizes every src1 column per 32-block exactly as the VALU mat-vec kernels do
(d = amax/127, round-to-nearest-even: mmvq_impl.h xblock_store) and sums the integer block dots
in int32 on v_mfma_i32_16x16x32_i8, so against the VALU path (GGML_MI355X_MMA=0, the same
activation bytes) only the fp32 order of the per-block scale sums differs: NMSE <= 1e-10. Against
the CPU oracle (ggml-cpu's vec_dot on its own src1 quantization) the reference's MUL_MAT bar
5e-4 (tests/test-backend-ops.cpp:3106-3108) applies, as for every mat-vec case. (Its default
forms are also pinned by golden records from the reference itself, tests/golden mm_166..mm_172,
replayed by test_gpu_parity.py.)

Covered: all five types (Q6_K: two scales per 32-block, one MFMA chain per half); 1..8 columns (4- and 8-token
forms); ragged rows (N % 16 != 0); Q4_0 / Q8_0 K that ends inside a 128-step (K % 128 = 32, 64,
96), K-quants at odd super-block counts; the reference's perf shapes (K = 14336, bs 2..8);
broadcast batch slices (ne12 = 2 * ne02); every per-wave step run (K = 4096 .. 28672) with one and
two K parts; one or two row tiles per workgroup; paired and unpaired steps; bitwise repeatability.
"""
import numpy as np
import pytest

import golden_cases as G
import qref
from test_gpu_parity import mm, run_mul_mat  # noqa: F401  (fixture)

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

TYPES = [qref.Q4_0, qref.Q8_0, qref.Q4_K, qref.Q5_K, qref.Q6_K]


def operands(t, N, M_, K, seed, ne2=(1, 1)):
    """src0 [K, N, ne02] and src1 [K, M, ne12] (ne12 = 2 * ne02: broadcast)"""
    ne02, ne12 = ne2
    w = qref.quantize(t, qref.fill_uniform(N * K * ne02, seed), n_per_row=K)
    x = qref.fill_uniform(M_ * K * ne12, seed + 1)
    a = G.Operand(t, w, [K, N, ne02, 1], qref.contiguous_nb(t, [K, N, ne02, 1]))
    b = G.Operand(qref.F32, x, [K, M_, ne12, 1], qref.contiguous_nb(qref.F32, [K, M_, ne12, 1]))
    return a, b, [N, M_, ne12, 1]


def run_with(mm, a, b, out_ne, env):
    with mm.knobs(**env):
        return run_mul_mat(mm, a, b, out_ne)


def check(mm, t, N, M_, K, seed=3, ne2=(1, 1), oracle=True):
    a, b, out_ne = operands(t, N, M_, K, seed, ne2)
    env = {"GGML_MI355X_MMA": 2}
    got = run_with(mm, a, b, out_ne, env)
    assert np.all(np.isfinite(got))
    valu = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 0})
    e_valu = qref.nmse(got, valu)
    assert e_valu <= 1e-10, f"{qref.NAMES[t]} N={N} M={M_} K={K}: nmse vs the VALU mat-vec {e_valu:.3e}"
    if oracle:
        e = qref.nmse(got, G.oracle_mul_mat(a, b, out_ne, threads=16))
        assert e <= 5e-4, f"{qref.NAMES[t]} N={N} M={M_} K={K}: nmse vs oracle {e:.3e}"
    return got


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("M_", [2, 3, 5, 8])
def test_mma_columns(mm, t, M_):
    K = 512 if qref.BLCK[t] == 256 else 448   # (Q4_0 / Q8_0: 3.5 steps of 128)
    check(mm, t, 200, M_, K)


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q8_0], ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("K", [32, 64, 96, 160, 4160])
def test_mma_partial_step(mm, t, K):
    """the last 128-step holds 1..3 live blocks: activation codes past K are zero; the weight
    loads of the blocks past K read whatever follows the row (the next row, here), and the
    kernel zeroes those blocks' weight scales"""
    check(mm, t, 37, 4, K)


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q8_0], ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("K", [160, 4160])
def test_mma_partial_step_padded_rows(mm, t, K):
    """a strided view whose row padding (nb01 > row bytes) holds f16 infinities where
    the blocks past K would have their scale d: those blocks must not turn 0 * d into NaN"""
    N, M_ = 40, 4
    rowb = K // 32 * qref.TSIZE[t]
    pad = 4 * qref.TSIZE[t]
    w = qref.quantize(t, qref.fill_uniform(N * K, 5), n_per_row=K).view(np.uint8).reshape(N, rowb)
    buf = np.tile(np.array([0x00, 0x7C], np.uint8), N * (rowb + pad) // 2 + 1)[:N * (rowb + pad)].reshape(N, rowb + pad)
    buf[:, :rowb] = w
    nb = [qref.TSIZE[t], rowb + pad, (rowb + pad) * N, (rowb + pad) * N]
    a = G.Operand(t, buf.ravel(), [K, N, 1, 1], nb)
    x = qref.fill_uniform(M_ * K, 6)
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    out_ne = [N, M_, 1, 1]
    got = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 1})
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne)) <= 5e-4


@pytest.mark.parametrize("t,M_,K", [(qref.Q4_0, 5, 25600), (qref.Q4_K, 3, 49408), (qref.Q4_K, 3, 55296), (qref.Q4_K, 3, 55552),
                                    (qref.Q4_0, 8, 25600), (qref.Q8_0, 8, 14336), (qref.Q5_K, 5, 14336)])
def test_mma_rule_shapes_past_the_image(mm, t, M_, K):
    """at the edges of the LDS image (paired runs rounded up to even, 14 steps
    at 4 tokens; since round 6 the image is what the instantiation's static arrays leave, so the
    one-part plans of K = 14336 at 8 tokens and the two-part run of Q4_K K = 55296 fit while
    K = 55552 does not) the plan and the launcher agree: the MFMA kernel where it fits, the VALU
    kernels elsewhere, never a failed launch (tests/test_dispatch_plan.py pins the choices)"""
    a, b, out_ne = operands(t, 64, M_, K, 21)
    got = run_mul_mat(mm, a, b, out_ne)
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne, threads=16)) <= 5e-4


@pytest.mark.parametrize("t", [qref.Q4_K, qref.Q5_K, qref.Q6_K], ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("K", [256, 768, 2304])
def test_mma_kquant_k(mm, t, K):
    """odd super-block counts (the steps are half super-blocks: odd step pairs per wave)"""
    check(mm, t, 48, 6, K)


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("M_", [2, 8])
def test_mma_reference_perf_shape(mm, t, M_):
    """test-backend-ops perf's mat-vec shape, K = 14336, N = 4096, against the VALU path (the
    oracle at this size takes minutes; the smaller cases above hold the oracle check)"""
    a, b, out_ne = operands(t, 4096, M_, 14336, 7)
    got = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 2})
    valu = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 0})
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, valu) <= 1e-10


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
def test_mma_broadcast_slices(mm, t):
    check(mm, t, 64, 3, 256 if qref.BLCK[t] == 256 else 128, ne2=(2, 4))


@pytest.mark.parametrize("K", [4096, 4352, 8192, 14336, 28672])
@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q4_K], ids=lambda t: qref.NAMES[t])
def test_mma_wave_steps(mm, t, K):
    """each K picks another straight-line run per wave over the 16 waves of a workgroup, and from
    32 steps the K halves add into the zeroed dst (K = 4352: 34 steps, parts of 18 and 16); run
    twice: the waves meet in LDS in wave order and two halves add the same either way round, so
    the result repeats bit for bit"""
    a, b, out_ne = operands(t, 100, 5, K, 5)
    g1 = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 2})
    g2 = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 2})
    assert np.array_equal(g1.view(np.uint32), g2.view(np.uint32)), "result not repeatable"
    valu = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 0})
    assert qref.nmse(g1, valu) <= 1e-10


@pytest.mark.parametrize("layout", [(1, 1), (1, 2), (2, 1)], ids=lambda l: f"kh{l[0]}rt{l[1]}")
@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
def test_mma_layouts(mm, t, layout):
    """one K part and/or one 16-row tile per workgroup (GGML_MI355X_MMA_KH / _RT) against the
    VALU path, unpaired steps (Q4_0 / Q8_0 at this K would pair by default); ragged rows
    (N % 32 = 20)"""
    kh, rt = layout
    a, b, out_ne = operands(t, 180, 6, 8192, 11)
    got = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 2, "GGML_MI355X_MMA_KH": kh, "GGML_MI355X_MMA_RT": rt,
                                      "GGML_MI355X_MMA_PAIR": 0})
    valu = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 0})
    assert qref.nmse(got, valu) <= 1e-10


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
def test_mma_one_column(mm, t):
    """GGML_MI355X_MMA=1 takes single columns too (lanes past the live column repeat it)"""
    a, b, out_ne = operands(t, 100, 1, 2048, 9)
    got = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 1})
    valu = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 0})
    assert qref.nmse(got, valu) <= 1e-10


@pytest.mark.parametrize("K", [4096, 4160, 14336, 28672])
@pytest.mark.parametrize("M_", [3, 8])
@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q8_0], ids=lambda t: qref.NAMES[t])
def test_mma_paired_steps(mm, t, M_, K):
    """paired steps (GGML_MI355X_MMA_PAIR=1): a lane loads two adjacent blocks and permlane swaps
    hand each lane its block of both steps; K = 4160 ends inside a double step (the pair's second
    step past K meets zero columns); ragged rows; run twice for bitwise repeatability"""
    a, b, out_ne = operands(t, 200, M_, K, 13)
    env = {"GGML_MI355X_MMA": 1, "GGML_MI355X_MMA_PAIR": 1}
    g1 = run_with(mm, a, b, out_ne, env)
    g2 = run_with(mm, a, b, out_ne, env)
    assert np.array_equal(g1.view(np.uint32), g2.view(np.uint32)), "result not repeatable"
    valu = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 0})
    assert qref.nmse(g1, valu) <= 1e-10


@pytest.mark.parametrize("rt", [1, 2])
@pytest.mark.parametrize("K", [4096, 4352, 14336, 28672])
@pytest.mark.parametrize("M_", [3, 8])
@pytest.mark.parametrize("t", [qref.Q4_K, qref.Q5_K], ids=lambda t: qref.NAMES[t])
def test_mma_kquant_paired_steps(mm, t, M_, K, rt):
    """Q4_K / Q5_K paired steps (GGML_MI355X_MMA_PAIR=1): both halves of a super-block per wave,
    the qs bytes of 16 rows loaded 8 rows x 128 B per instruction and handed to the MFMA lanes by
    ds_bpermute, header (and Q5_K's qh piece) once per super-block; K = 4352 has an odd
    super-block count; ragged rows (N = 200); one and two row tiles (Q5_K: one); run twice for
    bitwise repeatability"""
    a, b, out_ne = operands(t, 200, M_, K, 19)
    env = {"GGML_MI355X_MMA": 1, "GGML_MI355X_MMA_PAIR": 1, "GGML_MI355X_MMA_RT": rt}
    g1 = run_with(mm, a, b, out_ne, env)
    g2 = run_with(mm, a, b, out_ne, env)
    assert np.array_equal(g1.view(np.uint32), g2.view(np.uint32)), "result not repeatable"
    valu = run_with(mm, a, b, out_ne, {"GGML_MI355X_MMA": 0})
    assert qref.nmse(g1, valu) <= 1e-10
