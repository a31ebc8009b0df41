"""GPU parity: the MI355X kernels (through the C ABI of libggml-hip-mi355x.so) vs the oracle.

Every case replays a golden record (tests/golden/manifest.json, produced by the reference's
own ggml-cpu) on byte-identical inputs and checks, like test-backend-ops does
(tests/test-backend-ops.cpp:1173-1213 of the reference):
  * NMSE <= 5e-4 against the reference CPU output (the MUL_MAT / MUL_MAT_ID bar, :3106-3108),
  * and against the CPU oracle recomputed here on the same bytes,
  * no NaN/Inf, and 1024-float sentinels on both sides of dst left untouched.
Dequantization must be bit-exact with the reference's dequantize_row_*.
"""
import numpy as np
import pytest

import golden_cases as G
import qref

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

SENT = 1024
SENT_VAL = np.float32(-8675309.0)


@pytest.fixture(scope="module")
def mm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import mi355x_qmm as M
    M.build()
    assert M.device_count() >= 1, "no gfx950 device visible"
    return M


def dev_bytes(buf: np.ndarray):
    t = torch.from_numpy(np.ascontiguousarray(buf).view(np.uint8).copy()).cuda()
    return t


def guarded_out(nel: int):
    host = np.full(nel + 2 * SENT, SENT_VAL, np.float32)
    return torch.from_numpy(host).cuda()


def check_guard(out_dev, nel: int) -> np.ndarray:
    host = out_dev.cpu().numpy()
    assert np.all(host[:SENT] == SENT_VAL), "write before dst"
    assert np.all(host[SENT + nel:] == SENT_VAL), "write after dst"
    return host[SENT:SENT + nel]


def run_mul_mat(M, a: G.Operand, b: G.Operand, out_ne):
    da, db = dev_bytes(a.buf), dev_bytes(b.buf)
    nel = int(np.prod(out_ne))
    dout = guarded_out(nel)
    A = M.tensor(a.type, da.data_ptr(), a.ne, a.nb)
    B = M.tensor(qref.F32, db.data_ptr(), b.ne, b.nb)
    D = M.tensor(qref.F32, dout.data_ptr() + 4 * SENT, out_ne, qref.contiguous_nb(qref.F32, out_ne))
    M.mul_mat(A, B, D)
    torch.cuda.synchronize()
    return check_guard(dout, nel)


MM = [r for r in G.manifest() if r["kind"] == "mul_mat"]
MMID = [r for r in G.manifest() if r["kind"] == "mul_mat_id"]


@pytest.mark.parametrize("r", MM, ids=lambda r: r["name"])
def test_mul_mat_vs_reference(mm, r):
    a, b, out_ne = G.mul_mat_operands(r)
    got = run_mul_mat(mm, a, b, out_ne)
    want = G.load_bin(r["name"] + ".out.f32", np.float32)
    assert np.all(np.isfinite(got))
    if "sample_cols" in r:
        # big case (Q8_0 4096x4096x512): the reference output of a strided column sample that
        # touches every 128-column tile, and every column's (sum, sum of squares) in f64
        cols = got.reshape(-1, out_ne[0])
        e_ref = qref.nmse(cols[r["sample_cols"]], want.reshape(len(r["sample_cols"]), -1))
        cs = G.load_bin(r["colsums"], np.float64).reshape(-1, 2)
        c64 = cols.astype(np.float64)
        norm = np.sqrt(cs[:, 1])
        # independent per-element errors at the sample's NMSE give a column-sum error with
        # std sqrt(nmse) * norm; allow 6 sigma (a wrong or missing tile is off by ~norm)
        tol = 6 * np.sqrt(max(e_ref, 1e-6)) * norm
        assert np.all(np.abs(c64.sum(1) - cs[:, 0]) <= tol), "column sums"
        assert np.all(np.abs((c64 ** 2).sum(1) / cs[:, 1] - 1) <= 1e-3), "column sums of squares"
    else:
        assert got.size == want.size
        e_ref = qref.nmse(got, want)
    assert e_ref <= 5e-4, f"nmse vs reference CPU {e_ref:.3e}"
    # every output element against the oracle recomputed on the same bytes (threaded for the
    # BASELINE-size cases)
    e_orc = qref.nmse(got, G.oracle_mul_mat(a, b, out_ne, threads=16))
    assert e_orc <= 5e-4, f"nmse vs oracle {e_orc:.3e}"


@pytest.mark.parametrize("r", MMID, ids=lambda r: r["name"])
def test_mul_mat_id_vs_reference(mm, r):
    a, b, ids, out_ne = G.mul_mat_id_operands(r)
    da, db, di = dev_bytes(a.buf), dev_bytes(b.buf), dev_bytes(ids.buf)
    nel = int(np.prod(out_ne))
    dout = guarded_out(nel)
    A = mm.tensor(a.type, da.data_ptr(), a.ne, a.nb)
    B = mm.tensor(qref.F32, db.data_ptr(), b.ne, b.nb)
    I = mm.tensor(qref.I32, di.data_ptr(), ids.ne, ids.nb)
    D = mm.tensor(qref.F32, dout.data_ptr() + 4 * SENT, out_ne, qref.contiguous_nb(qref.F32, out_ne))
    mm.mul_mat_id(A, B, I, D)
    torch.cuda.synchronize()
    got = check_guard(dout, nel)
    want = G.load_bin(r["name"] + ".out.f32", np.float32)
    assert qref.nmse(got, want) <= 5e-4
    assert qref.nmse(got, G.oracle_mul_mat_id(a, b, ids, out_ne)) <= 5e-4


QUANT = [r for r in G.manifest() if r["kind"] == "quant"]


@pytest.mark.parametrize("r", QUANT, ids=lambda r: r["name"])
def test_dequantize_bit_exact(mm, r):
    q = G.load_bin(r["name"] + ".q", np.uint8)
    want = G.load_bin(r["name"] + ".deq.f32", np.float32)
    dq = dev_bytes(q)
    out = torch.empty(r["n"], dtype=torch.float32, device="cuda")
    mm.dequantize(r["type_id"], dq.data_ptr(), out.data_ptr(), r["n"])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("t", qref.HOT_TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("n", [0, 1, 3, 8, 9, 17])
def test_edge_shapes(mm, t, n):
    """empty batch, ragged columns and ragged K (K % 64 == 32 for the 32-block types)."""
    K = 32 * 3 if qref.BLCK[t] == 32 else 512
    N = 37
    w = qref.quantize(t, qref.fill_uniform(N * K, 11), n_per_row=K)
    x = qref.fill_uniform(max(n, 1) * K, 12)[: n * K]
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x if n else np.zeros(1, np.float32), [K, n, 1, 1], qref.contiguous_nb(qref.F32, [K, n, 1, 1]))
    out_ne = [N, n, 1, 1]
    got = run_mul_mat(mm, a, b, out_ne)
    if n:
        want = G.oracle_mul_mat(a, b, out_ne)
        assert qref.nmse(got, want) <= 5e-4


def test_rejects_bad_shapes(mm):
    t = qref.Q4_K
    w = torch.zeros(144 * 4, dtype=torch.uint8, device="cuda")
    x = torch.zeros(256 * 2, dtype=torch.float32, device="cuda")
    d = torch.zeros(8, dtype=torch.float32, device="cuda")
    A = mm.tensor(t, w.data_ptr(), [256, 4, 1, 1], qref.contiguous_nb(t, [256, 4]))
    B = mm.tensor(qref.F32, x.data_ptr(), [128, 4, 1, 1], qref.contiguous_nb(qref.F32, [128, 4]))   # K mismatch
    D = mm.tensor(qref.F32, d.data_ptr(), [4, 2, 1, 1], qref.contiguous_nb(qref.F32, [4, 2]))
    with pytest.raises(mm.Mi355xError):
        mm.mul_mat(A, B, D)


# ------------------------------------------------------------------------------------------
# mat-mat (ne11 > 8) path: the int8 MFMA tile (every K), K % 256 != 0 included
# ------------------------------------------------------------------------------------------
MMQ_SHAPES = [  # (N, M, K-multiplier) around the tile edges
    (37, 9, 1), (64, 127, 2), (65, 128, 1), (200, 129, 2), (128, 300, 3),
]


@pytest.mark.parametrize("t", qref.HOT_TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("shape", MMQ_SHAPES, ids=lambda s: f"n{s[0]}_m{s[1]}_k{s[2]}")
def test_mmq_tile_edges(mm, t, shape):
    N, M_, km = shape
    # 32-block types: K % 64 == 32 for odd multipliers (a partial last super-block on the int8
    # tile), K % 256 == 0 for even ones; K-quants: any multiple of 256
    K = (96 if qref.BLCK[t] == 32 and km % 2 else 256) * km
    w = qref.quantize(t, qref.fill_uniform(N * K, 21), n_per_row=K)
    x = qref.fill_uniform(M_ * K, 22)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    out_ne = [N, M_, 1, 1]
    got = run_mul_mat(mm, a, b, out_ne)
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne)) <= 5e-4


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q6_K], ids=lambda t: qref.NAMES[t])
def test_mmq_broadcast_and_strided_rows(mm, t):
    """weights [K,N,2,1] broadcast over activations [K,M,4,3] whose rows are padded (nb11 > 4K)."""
    K, N, M_ = 512, 96, 40
    w = qref.quantize(t, qref.fill_uniform(N * K * 2, 31), n_per_row=K)
    pad = 24
    xs = qref.fill_uniform((K + pad) * M_ * 12, 32)
    a = G.Operand(t, w, [K, N, 2, 1], qref.contiguous_nb(t, [K, N, 2, 1]))
    nb1 = 4 * (K + pad)
    b = G.Operand(qref.F32, xs, [K, M_, 4, 3], [4, nb1, nb1 * M_, nb1 * M_ * 4])
    out_ne = [N, M_, 4, 3]
    got = run_mul_mat(mm, a, b, out_ne)
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne)) <= 5e-4


@pytest.mark.parametrize("scale", [1e-6, 3e4, 1e7])
def test_mmq_activation_range(mm, scale):
    """activations far outside the f16 range: the int8 tile's Q8_K blocks of 256 carry an f32
    scale, so nothing under/overflows; the bar (NMSE <= 2e-4) is the int8 rounding of the
    activations (the per-256 block of the outlier token is coarse).

    Checked against the exact product (bit-exact dequantized weights x activations in float64):
    at these magnitudes the reference's own Q8_0 activation blocks underflow / overflow their fp16
    scale (d = amax/127 stored as fp16), so ggml-cpu is not a usable oracle here.
    """
    bar = 2e-4
    t, K, N, M_ = qref.Q8_0, 256, 64, 33
    w = qref.quantize(t, qref.fill_uniform(N * K, 41), n_per_row=K)
    x = (qref.fill_uniform(M_ * K, 42) * np.float32(scale)).astype(np.float32)
    x[5 * K + 7] *= 50.0          # one outlier token
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x, [K, M_, 1, 1], qref.contiguous_nb(qref.F32, [K, M_, 1, 1]))
    out_ne = [N, M_, 1, 1]
    got = run_mul_mat(mm, a, b, out_ne)
    assert np.all(np.isfinite(got))
    wf = qref.dequantize(t, w, N * K).reshape(N, K).astype(np.float64)
    exact = (x.reshape(M_, K).astype(np.float64) @ wf.T).reshape(-1)
    assert qref.nmse(got.astype(np.float64), exact) <= bar


# ------------------------------------------------------------------------------------------
# MUL_MAT_ID, grouped MFMA path (>= 64 (slot, token) pairs): experts sorted on the device
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("t", qref.HOT_TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("bcast", [False, True], ids=["b_per_slot", "b_shared"])
def test_mul_mat_id_grouped(mm, t, bcast):
    """the grouped int8 tile (experts sorted on the device by moe_prep)"""
    K = 512 if qref.BLCK[t] == 256 else 96 * 3
    N, E, U, T = 300, 8, 2, 200
    w = qref.quantize(t, qref.fill_uniform(N * K * E, 51), n_per_row=K)
    b_ne1 = 1 if bcast else U
    x = qref.fill_uniform(K * b_ne1 * T, 52)
    rng = np.random.default_rng(53)
    ids = np.stack([rng.permutation(E)[:U] for _ in range(T)]).astype(np.int32)   # [T][U]
    ids[: T // 2, 0] = 3                                                           # a hot expert
    ids[: T // 2, 1] = np.where(ids[: T // 2, 1] == 3, 5, ids[: T // 2, 1])
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
    D = mm.tensor(qref.F32, dout.data_ptr() + 4 * SENT, out_ne, qref.contiguous_nb(qref.F32, out_ne))
    mm.mul_mat_id(A, B, I, D)
    torch.cuda.synchronize()
    got = check_guard(dout, nel)
    want = G.oracle_mul_mat_id(a, b, iop, out_ne)
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, want) <= 5e-4
