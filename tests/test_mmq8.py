"""GPU parity of the int8 MFMA mat-mat path (csrc/mmq8.hip) against the CPU oracle.

Every case with more than 8 tokens runs the int8 tile (the only mat-mat path); the fixture
force_i8 runs it on the weights in place and on a per-call repacked copy. Its activations are quantized
exactly like the CPU backend's Q8_K blocks (quantize_row_q8_K_ref, reference
src/ggml-quants.c:2555-2591) and its block dot products are exact int32 sums, so:
  * Q4_K / Q5_K / Q6_K: the oracle (ggml_vec_dot_q4_K_q8_K / _q5_K_ / _q6_K_ semantics on the
    same Q8_K blocks) differs only by the fp32 order of the per-block scale accumulation:
    NMSE <= 1e-9;
  * Q4_0 / Q8_0: the CPU quantizes activations per 32 (Q8_0 blocks), this path per 256:
    NMSE <= 5e-4 (the reference's MUL_MAT bar, test-backend-ops.cpp:3106-3108), and against the
    exact float64 product of the bit-exact dequantized weights within the activation rounding.
"""
import numpy as np
import pytest

import golden_cases as G
import qref
from test_gpu_parity import mm, run_mul_mat  # noqa: F401  (fixture)

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

TYPES = [qref.Q4_0, qref.Q8_0, qref.Q4_K, qref.Q5_K, qref.Q6_K]
TIGHT = {qref.Q4_K: 1e-9, qref.Q5_K: 1e-9, qref.Q6_K: 1e-9, qref.Q4_0: 5e-4, qref.Q8_0: 5e-4}


@pytest.fixture(autouse=True, params=["inplace", "repack"])
def force_i8(request, mm):
    """every case runs twice: on the in-place int8 tile (mmq8_kernel) and on the tile over a
    per-call repacked copy of the weights (repack_kernel + mmq8r_kernel, GGML_MI355X_MMQ_REPACK_MIN)"""
    with mm.knobs(GGML_MI355X_MMQ_REPACK_MIN=9 if request.param == "repack" else None):
        yield request.param


def exact(t, w, N, K, x, M_):
    wd = qref.dequantize(t, w, N * K).reshape(N, K).astype(np.float64)
    return (x.reshape(M_, K).astype(np.float64) @ wd.T).astype(np.float64).ravel()


def case(mm, t, N, M_, K, seed=1, ksplit=None, tt=None, sk=None, ret_got=False):
    w = qref.quantize(t, qref.fill_uniform(N * K, seed), n_per_row=K)
    x = qref.fill_uniform(M_ * K, seed + 1)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    with mm.knobs(GGML_MI355X_MMQ8_KSPLIT=ksplit, GGML_MI355X_MMQ8_TT=tt, GGML_MI355X_MMQ8_SK=sk):
        got = run_mul_mat(mm, a, b, [N, M_, 1, 1])
    assert np.all(np.isfinite(got))
    want = G.oracle_mul_mat(a, b, [N, M_, 1, 1])
    err = qref.nmse(got, want)
    assert err <= TIGHT[t], f"{qref.NAMES[t]} N={N} M={M_} K={K}: nmse vs oracle {err:.3e}"
    ex = exact(t, w, N, K, x, M_)
    err_x = float(np.sum((got - ex) ** 2) / np.sum(ex ** 2))
    assert err_x <= 2e-4, f"{qref.NAMES[t]} N={N} M={M_} K={K}: nmse vs exact {err_x:.3e}"
    return got if ret_got else err


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


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q8_0], ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("shape", [(64, 16, 32), (37, 9, 96), (200, 129, 288), (130, 200, 96 * 11), (128, 512, 4096 + 96),
                                   (256, 300, 2048 - 32)],
                         ids=lambda s: "x".join(map(str, s)))
def test_mmq8_partial_superblock(mm, t, shape):
    """K not a multiple of 256: the last super-block is partial; its missing
    32-blocks carry zero activation codes and a zero weight scale. Rows of an odd number of
    blocks (K = 32, 96, ...) are 2-byte aligned every other row."""
    N, M_, K = shape
    case(mm, t, N, M_, K, seed=13)


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q8_0], ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("ksplit", [2, 3])
def test_mmq8_partial_superblock_ksplit(mm, t, ksplit):
    """split-K whose last split ends in the partial super-block"""
    case(mm, t, 192, 96, 256 * 4 + 160, seed=17, ksplit=ksplit)


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q8_0, qref.Q6_K], ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("K", [256, 96 * 5], ids=lambda k: f"k{k}")
def test_mmq8_matrix_at_2_mod_4(mm, t, K):
    """the weight matrix itself starts at 2 mod 4 (a view at an odd block offset): the buffer is
    based at its dword floor and every window realigned from its own offset"""
    if qref.BLCK[t] == 256 and K % 256:
        pytest.skip("K-quants: K is a multiple of 256")
    from test_gpu_parity import check_guard, guarded_out
    N, M_ = 150, 70
    w = qref.quantize(t, qref.fill_uniform(N * K, 19), n_per_row=K)
    x = qref.fill_uniform(M_ * K, 20)
    raw = np.zeros(w.nbytes + 2, np.uint8)
    raw[2:] = w.view(np.uint8)
    dw = torch.from_numpy(raw).cuda()
    dx = torch.from_numpy(x.copy()).cuda()
    nel = N * M_
    dout = guarded_out(nel)
    A = mm.tensor(t, dw.data_ptr() + 2, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    B = mm.tensor(qref.F32, dx.data_ptr(), [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    D = mm.tensor(qref.F32, dout.data_ptr() + 4 * 1024, [N, M_, 1, 1], qref.contiguous_nb(qref.F32, [N, M_, 1, 1]))
    mm.mul_mat(A, B, D)
    torch.cuda.synchronize()
    got = check_guard(dout, nel)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, G.oracle_mul_mat(a, b, [N, M_, 1, 1])) <= TIGHT[t]


@pytest.mark.parametrize("t,big", [(qref.Q8_0, 7.0e4), (qref.Q4_0, 1.0e5)])
@pytest.mark.parametrize("M_", [200, 512])
@pytest.mark.parametrize("K", [96, 96 * 7])
def test_mmq8_huge_scales_ragged_k(mm, t, big, M_, K):
    """block scales far past the f16 tile's range (d > 511) with K = 96 k, the
    shapes that used to fall to the f16 LDS-staged tiles; now on the exact int8 tile"""
    N = 160
    f = qref.fill_uniform(N * K, 79).reshape(N, K)
    f[5::7] *= big
    w = qref.quantize(t, f.reshape(-1), n_per_row=K)
    x = qref.fill_uniform(M_ * K, 80)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    got = run_mul_mat(mm, a, b, [N, M_, 1, 1])
    want = G.oracle_mul_mat(a, b, [N, M_, 1, 1])
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, want) <= TIGHT[t]
    keep = np.ones(N, bool)
    keep[5::7] = False
    assert qref.nmse(got.reshape(M_, N)[:, keep], want.reshape(M_, N)[:, keep]) <= TIGHT[t]


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


# ------------------------------------------------------------------------------------------
# MUL_MAT_ID on the int8 tile (>= 64 (slot, token) pairs; mmq8_id_launch): experts grouped on
# the device, activation columns gathered per 64-pair tile, rows scattered to dst[slot][token]
# ------------------------------------------------------------------------------------------
def run_mul_mat_id(mm, t, w, x, ids, K, N, E, b_ne1):
    from test_gpu_parity import check_guard, dev_bytes, guarded_out
    U, T = ids.shape[1], ids.shape[0]
    a = G.Operand(t, w, [K, N, E, 1], qref.contiguous_nb(t, [K, N, E, 1]))
    b = G.Operand(qref.F32, x, [K, b_ne1, T, 1], qref.contiguous_nb(qref.F32, [K, b_ne1, T, 1]))
    iop = G.Operand(qref.I32, ids, [U, T, 1, 1], [4, 4 * U, 4 * U * T, 4 * U * T])
    out_ne = [N, U, T, 1]
    da, db, di = dev_bytes(w), dev_bytes(x), dev_bytes(ids)
    nel = int(np.prod(out_ne))
    dout = guarded_out(nel)
    A = mm.tensor(t, da.data_ptr(), a.ne, a.nb)
    B = mm.tensor(qref.F32, db.data_ptr(), b.ne, b.nb)
    I = mm.tensor(qref.I32, di.data_ptr(), iop.ne, iop.nb)
    D = mm.tensor(qref.F32, dout.data_ptr() + 4 * 1024, out_ne, qref.contiguous_nb(qref.F32, out_ne))
    mm.mul_mat_id(A, B, I, D)
    torch.cuda.synchronize()
    return check_guard(dout, nel), G.oracle_mul_mat_id(a, b, iop, out_ne)


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("case_", ["skewed", "empty_experts", "one_expert", "b_shared"])
def test_mmq8_mul_mat_id(mm, t, case_):
    """expert counts that are not multiples of the 64-pair tile, a hot expert, experts with no
    pair (their tiles do not exist), all pairs on one expert, src1 shared by the slots"""
    K, N, E, U, T = 512, 200, 8, 2, 150
    rng = np.random.default_rng(61)
    ids = np.stack([rng.permutation(E)[:U] for _ in range(T)]).astype(np.int32)
    if case_ == "skewed":
        ids[: T // 2, 0] = 3
        ids[: T // 2, 1] = np.where(ids[: T // 2, 1] == 3, 5, ids[: T // 2, 1])
    elif case_ == "empty_experts":
        ids = np.stack([rng.choice([1, 4, 6], U, replace=False) for _ in range(T)]).astype(np.int32)
    elif case_ == "one_expert":
        U = 1
        ids = np.full((T, 1), 7, np.int32)
    b_ne1 = 1 if case_ == "b_shared" else U
    w = qref.quantize(t, qref.fill_uniform(N * K * E, 62), n_per_row=K)
    x = qref.fill_uniform(K * b_ne1 * T, 63)
    got, want = run_mul_mat_id(mm, t, w, x, ids, K, N, E, b_ne1)
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, want) <= TIGHT[t]


@pytest.mark.parametrize("t,big", [(qref.Q8_0, 7.0e4), (qref.Q4_K, 2.0e3), (qref.Q6_K, 3.0e3)])
def test_mmq8_mul_mat_id_huge_scales(mm, t, big):
    """scales far beyond real weights on the grouped path: exact int32 block sums, f32 scales"""
    K, N, E, U, T = 512, 96, 4, 2, 100
    f = qref.fill_uniform(N * K * E, 71).reshape(N * E, K)
    f[3::5] *= big
    w = qref.quantize(t, f.reshape(-1), n_per_row=K)
    x = qref.fill_uniform(K * U * T, 72)
    ids = np.stack([np.random.default_rng(73 + i).permutation(E)[:U] for i in range(T)]).astype(np.int32)
    got, want = run_mul_mat_id(mm, t, w, x, ids, K, N, E, U)
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, want) <= TIGHT[t]


@pytest.mark.parametrize("t", [qref.Q8_0, qref.Q4_K], ids=lambda t: qref.NAMES[t])
def test_mmq8_two_halves_bitwise_repeatable(mm, t):
    """the 2-way split-K adds both K-halves into the zeroed dst with float atomics: with exactly
    two addends the sum is order-independent, so repeated calls agree bit for bit (N = 1024,
    M = 512, K = 1024: 64 tiles of 128 x 64, four super-blocks, two K-halves)"""
    N, M_, K = 1024, 512, 1024
    w = qref.quantize(t, qref.fill_uniform(N * K, 91), n_per_row=K)
    x = qref.fill_uniform(M_ * K, 92)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    outs = [run_mul_mat(mm, a, b, [N, M_, 1, 1]) for _ in range(3)]
    assert all(np.array_equal(outs[0].view(np.uint32), o.view(np.uint32)) for o in outs[1:])
    assert qref.nmse(outs[0], G.oracle_mul_mat(a, b, [N, M_, 1, 1])) <= TIGHT[t]


@pytest.mark.parametrize("t", [qref.Q8_0, qref.Q4_0], ids=lambda t: qref.NAMES[t])
def test_mmq8_config3_repeat_bitwise(mm, t):
    """the magic-constant tiles (Q8_0 / Q4_0) at BASELINE configs[3] size, 48 calls back to back:
    every call bit-identical to the first. The fault this guards against (the
    packed-f32 fault: the compiler reused the MFMA C-input registers 7 wait states after the last
    MFMA that read them) showed as a few wrong (register, lane) positions varying run to run."""
    from test_gpu_parity import dev_bytes
    N, M_, K = 4096, 512, 4096
    w = qref.quantize(t, qref.fill_uniform(N * K, 5), n_per_row=K)
    x = qref.fill_uniform(M_ * K, 6)
    da, db = dev_bytes(w), dev_bytes(x)
    A = mm.tensor(t, da.data_ptr(), [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    B = mm.tensor(qref.F32, db.data_ptr(), [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    outs = [torch.empty(M_ * N, dtype=torch.float32, device="cuda") for _ in range(2)]
    Ds = [mm.tensor(qref.F32, o.data_ptr(), [N, M_, 1, 1], qref.contiguous_nb(qref.F32, [N, M_, 1, 1])) for o in outs]
    mm.mul_mat(A, B, Ds[0])
    bad = 0
    for _ in range(48):
        outs[1].fill_(float("nan"))
        mm.mul_mat(A, B, Ds[1])
        bad += int((outs[0].view(torch.int32) != outs[1].view(torch.int32)).sum().item())
    assert bad == 0, f"{bad} elements differ from the first call over 48 calls"
    assert torch.isfinite(outs[0]).all()
