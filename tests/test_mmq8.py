"""GPU parity of the int8 MFMA mat-mat path (csrc/mmq8.hip) against the CPU oracle.

The path is forced with GGML_MI355X_MMQ=i8 (read on every call). Its activations are quantized
exactly like the CPU backend's Q8_K blocks (quantize_row_q8_K_ref, reference
src/ggml-quants.c:2555-2591) and its block dot products are exact int32 sums, so:
  * Q4_K / Q5_K / Q6_K: the oracle (ggml_vec_dot_q4_K_q8_K / _q5_K_ / _q6_K_ semantics on the
    same Q8_K blocks) differs only by the fp32 order of the per-block scale accumulation:
    NMSE <= 1e-9;
  * Q4_0 / Q8_0: the CPU quantizes activations per 32 (Q8_0 blocks), this path per 256:
    NMSE <= 5e-4 (the reference's MUL_MAT bar, test-backend-ops.cpp:3106-3108), and against the
    exact float64 product of the bit-exact dequantized weights within the activation rounding.
"""
import os

import numpy as np
import pytest

import golden_cases as G
import qref
from test_gpu_parity import mm, run_mul_mat  # noqa: F401  (fixture)

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

TYPES = [qref.Q4_0, qref.Q8_0, qref.Q4_K, qref.Q5_K, qref.Q6_K]
TIGHT = {qref.Q4_K: 1e-9, qref.Q5_K: 1e-9, qref.Q6_K: 1e-9, qref.Q4_0: 5e-4, qref.Q8_0: 5e-4}


@pytest.fixture(autouse=True)
def force_i8():
    old = os.environ.get("GGML_MI355X_MMQ")
    os.environ["GGML_MI355X_MMQ"] = "i8"
    yield
    if old is None:
        del os.environ["GGML_MI355X_MMQ"]
    else:
        os.environ["GGML_MI355X_MMQ"] = old


def exact(t, w, N, K, x, M_):
    wd = qref.dequantize(t, w, N * K).reshape(N, K).astype(np.float64)
    return (x.reshape(M_, K).astype(np.float64) @ wd.T).astype(np.float64).ravel()


def case(mm, t, N, M_, K, seed=1, ksplit=None, tt=None):
    if ksplit is not None:
        os.environ["GGML_MI355X_MMQ8_KSPLIT"] = str(ksplit)
    if tt is not None:
        os.environ["GGML_MI355X_MMQ8_TT"] = str(tt)
    try:
        w = qref.quantize(t, qref.fill_uniform(N * K, seed), n_per_row=K)
        x = qref.fill_uniform(M_ * K, seed + 1)
        a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
        b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
        got = run_mul_mat(mm, a, b, [N, M_, 1, 1])
    finally:
        os.environ.pop("GGML_MI355X_MMQ8_KSPLIT", None)
        os.environ.pop("GGML_MI355X_MMQ8_TT", None)
    assert np.all(np.isfinite(got))
    want = G.oracle_mul_mat(a, b, [N, M_, 1, 1])
    err = qref.nmse(got, want)
    assert err <= TIGHT[t], f"{qref.NAMES[t]} N={N} M={M_} K={K}: nmse vs oracle {err:.3e}"
    ex = exact(t, w, N, K, x, M_)
    err_x = float(np.sum((got - ex) ** 2) / np.sum(ex ** 2))
    assert err_x <= 2e-4, f"{qref.NAMES[t]} N={N} M={M_} K={K}: nmse vs exact {err_x:.3e}"
    return err


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("shape", [(64, 64, 256), (100, 37, 512), (256, 130, 1280), (33, 9, 768), (512, 200, 4096),
                                   (300, 129, 2048), (128, 512, 1024)],
                         ids=lambda s: "x".join(map(str, s)))
def test_mmq8_shapes(mm, t, shape):
    N, M_, K = shape
    case(mm, t, N, M_, K)


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("ksplit", [1, 2, 3])
def test_mmq8_ksplit(mm, t, ksplit):
    """split-K over workgroups (fixed-order reduce), with a super-block count the splits do not
    divide evenly"""
    case(mm, t, 192, 96, 256 * 5, seed=7, ksplit=ksplit)


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("tt", [64, 128])
def test_mmq8_token_tiles(mm, t, tt):
    """both workgroup shapes (128 rows x 64 tokens with two K-groups, 128 x 128 with whole
    super-blocks per wave), with ragged rows and tokens"""
    case(mm, t, 200, 300, 768, seed=11, tt=tt)


@pytest.mark.parametrize("t,big", [(qref.Q8_0, 7.0e4), (qref.Q4_K, 2.0e3), (qref.Q4_0, 1.0e5), (qref.Q6_K, 3.0e3),
                                   (qref.Q5_K, 2.0e3)])
@pytest.mark.parametrize("M_", [16, 200, 512])
def test_mmq8_huge_scales(mm, t, big, M_):
    """block scales far beyond what quantized weights hold (|w| in the thousands),
    at token counts that run the full 128 x 64 tiles: the int8 path converts every scale to f32,
    so there is no f16 range to overflow"""
    K, N = 512, 160
    f = qref.fill_uniform(N * K, 77).reshape(N, K)
    f[5::7] *= big
    w = qref.quantize(t, f.reshape(-1), n_per_row=K)
    x = qref.fill_uniform(M_ * K, 78)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    got = run_mul_mat(mm, a, b, [N, M_, 1, 1])
    want = G.oracle_mul_mat(a, b, [N, M_, 1, 1])
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, want) <= TIGHT[t]
    keep = np.ones(N, bool)
    keep[5::7] = False
    assert qref.nmse(got.reshape(M_, N)[:, keep], want.reshape(M_, N)[:, keep]) <= TIGHT[t]


@pytest.mark.parametrize("K", [256, 768])
def test_mmq8_q6_k_odd_rows(mm, K):
    """Q6_K rows of an odd number of super-blocks are 2-byte aligned every other row
    (210-byte super-blocks): the staging realigns each lane's windows"""
    case(mm, qref.Q6_K, 131, 70, K, seed=9)


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q4_K, qref.Q6_K], ids=lambda t: qref.NAMES[t])
def test_mmq8_broadcast_and_strided_rows(mm, t):
    """weights [K,N,2,1] broadcast over activations [K,M,4,3] with padded rows (nb11 > 4K)"""
    K, N, M_ = 512, 96, 40
    w = qref.quantize(t, qref.fill_uniform(N * K * 2, 31), n_per_row=K)
    pad = 24
    xs = qref.fill_uniform((K + pad) * M_ * 12, 32)
    a = G.Operand(t, w, [K, N, 2, 1], qref.contiguous_nb(t, [K, N, 2, 1]))
    nb1 = 4 * (K + pad)
    b = G.Operand(qref.F32, xs, [K, M_, 4, 3], [4, nb1, nb1 * M_, nb1 * M_ * 4])
    out_ne = [N, M_, 4, 3]
    got = run_mul_mat(mm, a, b, out_ne)
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne)) <= TIGHT[t]


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
def test_mmq8_activation_range(mm, t):
    """per-256 int8 blocks with an f32 scale: no under/overflow from 1e-6 to 1e7, outlier tokens"""
    K, N, M_ = 512, 64, 33
    w = qref.quantize(t, qref.fill_uniform(N * K, 41), n_per_row=K)
    for scale in (1e-6, 3e4, 1e7):
        x = (qref.fill_uniform(M_ * K, 42) * np.float32(scale)).astype(np.float32)
        x[5 * K + 7] *= 50.0
        x[9 * K:10 * K] = 0.0     # an all-zero token: d = 0, q = 0
        a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
        b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
        got = run_mul_mat(mm, a, b, [N, M_, 1, 1])
        ex = exact(t, w, N, K, x, M_)
        err = float(np.sum((got - ex) ** 2) / np.sum(ex ** 2))
        assert np.all(np.isfinite(got)) and err <= 2e-4, f"scale {scale}: {err:.3e}"
        assert np.all(got[9 * N:10 * N] == 0.0)


def test_mmq8_q8_0_config3(mm):
    """BASELINE configs[3]: Q8_0 4096 x 4096 x 512, every element against the threaded oracle"""
    t, N, M_, K = qref.Q8_0, 4096, 512, 4096
    w = qref.quantize(t, qref.fill_uniform(N * K, 3), n_per_row=K)
    x = qref.fill_uniform(M_ * K, 4)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    got = run_mul_mat(mm, a, b, [N, M_, 1, 1])
    want = G.oracle_mul_mat(a, b, [N, M_, 1, 1], threads=16)
    assert qref.nmse(got, want) <= 5e-4
