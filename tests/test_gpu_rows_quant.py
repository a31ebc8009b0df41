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


# ---- GGML_OP_CPY out of a quantized tensor (cpy_q_f32, reference src/ggml-cuda/cpy.cu:94;
# ggml-cpu dup_q src/ggml-cpu/ops.cpp:1105-1154, dup_bytes :956-1103) ----------------------

def _logical_rows(src: np.ndarray, t: int, ne, nb) -> list:
    """the quantized rows of a 4-d view in row-major logical order (bytes of each row)"""
    rb = qref.row_size(t, ne[0])
    out = []
    for i3 in range(ne[3]):
        for i2 in range(ne[2]):
            for i1 in range(ne[1]):
                o = i1 * nb[1] + i2 * nb[2] + i3 * nb[3]
                out.append(src[o:o + rb])
    return out


def _permuted_view(t, ne):
    """a [ne0, ne2, ne1, ne3] view of a contiguous [ne0, ne1, ne2, ne3] tensor (dims 1, 2 swapped)"""
    nb = qref.contiguous_nb(t, ne)
    return [ne[0], ne[2], ne[1], ne[3]], [nb[0], nb[2], nb[1], nb[3]]


@pytest.mark.parametrize("t", list(qref.HOT_TYPES), ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("layout", ["contig", "permuted", "reshaped_dst", "padded_dst"])
def test_cpy_q_to_f32_bit_exact(mm, t, layout):
    """CPY Q* -> f32 (test-backend-ops test_cpy, tests/test-backend-ops.cpp:5560-5600, with the
    src permutes it runs): every element the bit-exact dequantize_row_* value at dup_q's place."""
    blck = qref.BLCK[t]
    ne = [2 * blck, 3, 2, 2]
    src = G.weights_bytes(t, ne, 4242 + t)
    if layout == "permuted":
        lne, lnb = _permuted_view(t, ne)
    else:
        lne, lnb = ne, qref.contiguous_nb(t, ne)
    rows = _logical_rows(src, t, lne, lnb)
    want = np.concatenate([qref.dequantize(t, r, lne[0]) for r in rows])
    nel = int(np.prod(lne))
    ds = dev(src)
    if layout == "padded_dst":        # dst rows hold whole blocks, 64 floats of padding after each
        pad = 64
        out = torch.full((nel // lne[0], lne[0] + pad), -7.0, dtype=torch.float32, device="cuda")
        dne = [lne[0], lne[1], lne[2], lne[3]]
        row = 4 * (lne[0] + pad)
        dnb = [4, row, row * lne[1], row * lne[1] * lne[2]]
    else:
        out = torch.full((nel,), -7.0, dtype=torch.float32, device="cuda")
        dne = [nel // 4, 2, 2, 1] if layout == "reshaped_dst" else lne   # contiguous: any shape
        dnb = qref.contiguous_nb(qref.F32, dne)
    S = mm.tensor(t, ds.data_ptr(), lne, lnb)
    D = mm.tensor(qref.F32, out.data_ptr(), dne, dnb)
    mm.cpy(S, D)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    if layout == "padded_dst":
        assert (got[:, lne[0]:] == -7.0).all(), "padding written"
        got = got[:, :lne[0]]
    np.testing.assert_array_equal(got.reshape(-1).view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("t", list(qref.HOT_TYPES), ids=lambda t: qref.NAMES[t])
def test_cpy_q_same_type_blocks(mm, t):
    """CPY of a permuted quantized view into a contiguous tensor of the same type: the blocks in
    logical order, byte for byte (dup_bytes)."""
    blck = qref.BLCK[t]
    ne = [3 * blck, 2, 3, 1]
    src = G.weights_bytes(t, ne, 99 + t)
    lne, lnb = _permuted_view(t, ne)
    want = np.concatenate(_logical_rows(src, t, lne, lnb))
    ds = dev(src)
    out = torch.zeros(want.size, dtype=torch.uint8, device="cuda")
    mm.cpy(mm.tensor(t, ds.data_ptr(), lne, lnb), mm.tensor(t, out.data_ptr(), lne, qref.contiguous_nb(t, lne)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_cpy_q_rejects(mm):
    t = qref.Q4_0
    q = torch.zeros(18 * 4, dtype=torch.uint8, device="cuda")
    f = torch.zeros(128, dtype=torch.float32, device="cuda")
    S = mm.tensor(t, q.data_ptr(), [64, 2], qref.contiguous_nb(t, [64, 2]))
    with pytest.raises(mm.Mi355xError):     # element counts differ
        mm.cpy(S, mm.tensor(qref.F32, f.data_ptr(), [64, 1], qref.contiguous_nb(qref.F32, [64, 1])))
    with pytest.raises(mm.Mi355xError):     # dst rows of 16 floats split blocks and dst is not contiguous
        mm.cpy(S, mm.tensor(qref.F32, f.data_ptr(), [16, 8, 1, 1], [4, 128, 1024, 1024]))
    with pytest.raises(mm.Mi355xError):     # Q4_0 -> Q8_0 is not a copy this path does
        mm.cpy(S, mm.tensor(qref.Q8_0, q.data_ptr(), [64, 2], qref.contiguous_nb(qref.Q8_0, [64, 2])))


@pytest.mark.parametrize("t", [qref.F32, qref.Q4_0], ids=["f32", "q4_0"])
def test_get_rows_out_of_range_raises(mm, t):
    """an index outside [0, ne01) is the reference's GGML_ASSERT (ops.cpp:5157): the device error
    word is raised and that row is not written; in-range rows are still right"""
    n, m = 64, 5
    src = G.weights_bytes(t, [n, m, 1, 1], 7)
    rows = np.array([1, m, -1, 3], dtype=np.int32)
    ds, di = dev(src), dev(rows)
    out = torch.full((4, n), -3.0, dtype=torch.float32, device="cuda")
    assert mm.device_error() in (0, 1)      # clear anything a previous test left
    A = mm.tensor(t, ds.data_ptr(), [n, m], qref.contiguous_nb(t, [n, m]) if t != qref.F32 else [4, 4 * n, 4 * n * m, 4 * n * m])
    R = mm.tensor(qref.I32, di.data_ptr(), [4, 1, 1, 1], [4, 16, 16, 16])
    D = mm.tensor(qref.F32, out.data_ptr(), [n, 4], qref.contiguous_nb(qref.F32, [n, 4]))
    mm.get_rows(A, R, D)
    torch.cuda.synchronize()
    assert mm.device_error() == 1
    assert mm.device_error() == 0          # reading clears it
    got = out.cpu().numpy()
    assert (got[1] == -3.0).all() and (got[2] == -3.0).all()
    rb = qref.row_size(t, n) if t != qref.F32 else 4 * n
    for k, r in ((0, 1), (3, 3)):
        row = src[r * rb:(r + 1) * rb]
        want = row.view(np.float32) if t == qref.F32 else qref.dequantize(t, row, n)
        np.testing.assert_array_equal(got[k].view(np.uint32), want.view(np.uint32))
