"""GPU parity for the §8(f) device conversions: GET_ROWS of quantized rows (bit-exact with
dequantize_row_*) and f32 -> Q4_0 / Q8_0 quantization (bit-exact with quantize_row_*_ref),
through the C ABI (ggml_mi355x_get_rows / ggml_mi355x_quantize)."""
import numpy as np
import pytest

import golden_cases as G
import qref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import mi355x_qmm as M
    M.build()
    assert M.device_count() >= 1
    return M


def dev(buf: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(buf).view(np.uint8).copy()).cuda()


@pytest.mark.parametrize("t", [qref.F32] + list(qref.HOT_TYPES), ids=lambda t: "f32" if t == qref.F32 else qref.NAMES[t])
@pytest.mark.parametrize("b,view", [(1, False), (7, False), (1, True), (7, True)])
def test_get_rows_bit_exact(mm, t, b, view):
    """test-backend-ops' GET_ROWS grid (tests/test-backend-ops.cpp:1951-2004, 5308-5320):
    in [256, 5, b], rows [4, b] (or a [2, b] view of them)."""
    n, m, r = 256, 5, 4
    src = G.weights_bytes(t, [n, m, b, 1], 77 + b)
    rng = np.random.default_rng(b)
    rows = rng.integers(0, m, size=(b, r), dtype=np.int32)
    rr = r // 2 if view else r
    ds, di = dev(src), dev(rows)
    out = torch.full((b, rr, n), -1.0, dtype=torch.float32, device="cuda")
    A = mm.tensor(t, ds.data_ptr(), [n, m, b, 1], qref.contiguous_nb(t, [n, m, b, 1]))
    R = mm.tensor(qref.I32, di.data_ptr(), [rr, b, 1, 1], [4, 4 * r, 4 * r * b, 4 * r * b])
    D = mm.tensor(qref.F32, out.data_ptr(), [n, rr, b, 1], qref.contiguous_nb(qref.F32, [n, rr, b, 1]))
    mm.get_rows(A, R, D)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    rowbytes = qref.row_size(t, n) if t != qref.F32 else 4 * n
    for i2 in range(b):
        for i1 in range(rr):
            row = src[(i2 * m + rows[i2, i1]) * rowbytes:(i2 * m + rows[i2, i1] + 1) * rowbytes]
            want = row.view(np.float32) if t == qref.F32 else qref.dequantize(t, row, n)
            np.testing.assert_array_equal(got[i2, i1].view(np.uint32), want.view(np.uint32))


QUANT_REF = [r for r in G.manifest() if r["kind"] == "quant" and r["imatrix"] == 0 and r["type_id"] in (qref.Q4_0, qref.Q8_0)]


@pytest.mark.parametrize("r", QUANT_REF, ids=lambda r: r["name"])
def test_quantize_matches_reference_fixture(mm, r):
    x = G.load_bin(r["input"], np.float32)[: r["n"]]
    want = G.load_bin(r["name"] + ".q", np.uint8)
    t, n = r["type_id"], r["n"]
    got = quantize_dev(mm, t, x.reshape(1, n))
    np.testing.assert_array_equal(got, want)


def quantize_dev(mm, t, x2d: np.ndarray) -> np.ndarray:
    rows, n = x2d.shape
    dx = torch.from_numpy(np.ascontiguousarray(x2d, np.float32)).cuda()
    nbytes = qref.row_size(t, n) * rows
    dq = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    S = mm.tensor(qref.F32, dx.data_ptr(), [n, rows, 1, 1], qref.contiguous_nb(qref.F32, [n, rows, 1, 1]))
    Q = mm.tensor(t, dq.data_ptr(), [n, rows, 1, 1], qref.contiguous_nb(t, [n, rows, 1, 1]))
    mm.quantize(S, Q)
    torch.cuda.synchronize()
    return dq.cpu().numpy()


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q8_0], ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("scale", [1e-7, 1.0, 3e4])
def test_quantize_random_vs_oracle(mm, t, scale):
    rows, n = 37, 512
    x = (qref.fill_uniform(rows * n, 91) * np.float32(scale)).reshape(rows, n)
    x[0, :32] = 0.0                            # all-zero block: d = 0, id = 0
    x[1, :32] = np.float32(scale)               # all-equal block
    x[2, 5], x[2, 9] = -np.float32(scale) * 2, np.float32(scale) * 2   # |max| tie: first one wins
    x[3, :32] = np.arange(32, dtype=np.float32) - 16.0                  # exact .5 products in q4_0
    got = quantize_dev(mm, t, x)
    want = qref.quantize(t, x.reshape(-1), n_per_row=n)
    np.testing.assert_array_equal(got, want)


def test_quantize_strided_rows(mm):
    """CPY by rows from a permuted f32 source (test-backend-ops 'cpy by rows', :5589)."""
    t = qref.Q8_0
    ne = [256, 2, 3, 4]
    x = qref.fill_uniform(int(np.prod(ne)), 5).reshape(ne[::-1])        # [4][3][2][256]
    dx = torch.from_numpy(x.copy()).cuda()
    # logical view with dims 1 and 2 swapped: ne = [256, 3, 2, 4]
    nb = qref.contiguous_nb(qref.F32, ne)
    lne, lnb = [256, 3, 2, 4], [nb[0], nb[2], nb[1], nb[3]]
    dq = torch.zeros(qref.row_size(t, 256) * 24, dtype=torch.uint8, device="cuda")
    S = mm.tensor(qref.F32, dx.data_ptr(), lne, lnb)
    Q = mm.tensor(t, dq.data_ptr(), lne, qref.contiguous_nb(t, lne))
    mm.quantize(S, Q)
    torch.cuda.synchronize()
    want = qref.quantize(t, np.ascontiguousarray(x.transpose(0, 2, 1, 3)).reshape(-1), n_per_row=256)
    np.testing.assert_array_equal(dq.cpu().numpy(), want)


def test_rejects_unsupported(mm):
    x = torch.zeros(64, dtype=torch.float32, device="cuda")
    q = torch.zeros(144, dtype=torch.uint8, device="cuda")
    S = mm.tensor(qref.F32, x.data_ptr(), [64, 1, 1, 1], qref.contiguous_nb(qref.F32, [64, 1]))
    Q = mm.tensor(qref.Q4_K, q.data_ptr(), [64, 1, 1, 1], [144, 144, 144, 144])
    with pytest.raises(mm.Mi355xError):
        mm.quantize(S, Q)            # K-quant device quantization is not implemented
