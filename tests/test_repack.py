"""The repacked weight layout for the int8 mat-mat tile (csrc/mmq8.hip
repack_kernel + mmq8r_kernel) through the explicit C API: ggml_mi355x_repack_size /
ggml_mi355x_repack / ggml_mi355x_mul_mat_repacked.

Parity bar as tests/test_mmq8.py: the same Q8_K-style activation blocks and exact int32 block
sums, so against the CPU oracle NMSE <= 1e-9 for the K-quants and the reference's 5e-4 for
Q4_0 / Q8_0 (activations blocked per 256 here, per 32 on the CPU). The repacked copy made once
and the per-call repack (GGML_MI355X_MMQ_REPACK_MIN) run the same kernel on the same bytes, so
they agree bit for bit."""

import numpy as np
import pytest

import golden_cases as G
import qref
from test_gpu_parity import check_guard, dev_bytes, guarded_out, mm, SENT  # noqa: F401

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

TYPES = [qref.Q4_0, qref.Q8_0, qref.Q4_K, qref.Q5_K, qref.Q6_K]
TIGHT = {qref.Q4_K: 1e-9, qref.Q5_K: 1e-9, qref.Q6_K: 1e-9, qref.Q4_0: 5e-4, qref.Q8_0: 5e-4}


def run_repacked(M, a: G.Operand, b: G.Operand, out_ne):
    da, db = dev_bytes(a.buf), dev_bytes(b.buf)
    A = M.tensor(a.type, da.data_ptr() + a.offset, a.ne, a.nb)
    nbytes = M.repack_size(A)
    rp = torch.full((nbytes,), 0x5A, dtype=torch.uint8, device="cuda")   # garbage: every byte must be written
    M.repack(A, rp.data_ptr(), nbytes)
    nel = int(np.prod(out_ne))
    dout = guarded_out(nel)
    B = M.tensor(qref.F32, db.data_ptr() + b.offset, b.ne, b.nb)
    D = M.tensor(qref.F32, dout.data_ptr() + 4 * SENT, out_ne, qref.contiguous_nb(qref.F32, out_ne))
    M.mul_mat_repacked(A, rp.data_ptr(), B, D)
    torch.cuda.synchronize()
    return check_guard(dout, nel)


def operands(t, N, M_, K, ne2=(1, 1), bcast=(1, 1), seed=5):
    a_ne = [K, N, ne2[0], ne2[1]]
    b_ne = [K, M_, ne2[0] * bcast[0], ne2[1] * bcast[1]]
    w = qref.quantize(t, qref.fill_uniform(int(np.prod(a_ne)), seed), n_per_row=K)
    x = qref.fill_uniform(int(np.prod(b_ne)), seed + 1)
    a = G.Operand(t, w, a_ne, qref.contiguous_nb(t, a_ne))
    b = G.Operand(qref.F32, x, b_ne, qref.contiguous_nb(qref.F32, b_ne))
    return a, b, [N, M_, b_ne[2], b_ne[3]]


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("shape", [(128, 64, 256), (100, 37, 512), (33, 9, 768), (256, 130, 1280), (300, 512, 2048)],
                         ids=lambda s: "x".join(map(str, s)))
def test_repacked_matches_oracle(mm, t, shape):
    N, M_, K = shape
    a, b, out_ne = operands(t, N, M_, K)
    got = run_repacked(mm, a, b, out_ne)
    assert np.all(np.isfinite(got))
    err = qref.nmse(got, G.oracle_mul_mat(a, b, out_ne))
    assert err <= TIGHT[t], f"{qref.NAMES[t]} {shape}: nmse {err:.3e}"


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q8_0], ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("K", [32, 96, 96 * 11, 4096 + 96])
def test_repacked_partial_superblock(mm, t, K):
    """K not a multiple of 256: the repacked rows are padded with zero codes and zero scales"""
    a, b, out_ne = operands(t, 130, 70, K)
    got = run_repacked(mm, a, b, out_ne)
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne)) <= TIGHT[t]


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q4_K, qref.Q6_K], ids=lambda t: qref.NAMES[t])
def test_repacked_batched_broadcast(mm, t):
    """3-d / 4-d weights: every matrix repacked; src1 broadcast over dims 2 and 3 (r2 = 2, r3 = 3)"""
    a, b, out_ne = operands(t, 96, 40, 512, ne2=(2, 1), bcast=(2, 3))
    got = run_repacked(mm, a, b, out_ne)
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne)) <= TIGHT[t]


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
def test_repacked_equals_per_call_repack(mm, t):
    """the copy made once and the per-call repack of mul_mat run the same kernel on the same
    bytes: bit-identical results"""
    from test_gpu_parity import run_mul_mat
    a, b, out_ne = operands(t, 256, 200, 1024, seed=11)
    once = run_repacked(mm, a, b, out_ne)
    with mm.knobs(GGML_MI355X_MMQ_REPACK_MIN=9):
        per_call = run_mul_mat(mm, a, b, out_ne)
    np.testing.assert_array_equal(once.view(np.uint32), per_call.view(np.uint32))


@pytest.mark.parametrize("t", [qref.Q4_0, qref.Q4_K], ids=lambda t: qref.NAMES[t])
def test_repacked_wide_calls_use_src0(mm, t):
    """once the in-place tile runs 128-token tiles (>= 256 of them) it reads src0 itself, the
    repacked copy being slower there (profiles/r04_mmq_m_sweep.txt): bit-identical to mul_mat"""
    from test_gpu_parity import run_mul_mat
    a, b, out_ne = operands(t, 4096, 1032, 256, seed=13)
    np.testing.assert_array_equal(run_repacked(mm, a, b, out_ne).view(np.uint32),
                                  run_mul_mat(mm, a, b, out_ne).view(np.uint32))


def test_repacked_decode_shapes_use_src0(mm):
    """ne11 <= 8 runs the mat-vec on src0 itself; the repacked copy is not read"""
    t = qref.Q4_K
    a, b, out_ne = operands(t, 64, 4, 512)
    got = run_repacked(mm, a, b, out_ne)
    assert qref.nmse(got, G.oracle_mul_mat(a, b, out_ne)) <= 5e-4


def test_repack_rejects(mm):
    x = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    F = mm.tensor(qref.F32, x.data_ptr(), [64, 4, 1, 1], qref.contiguous_nb(qref.F32, [64, 4]))
    with pytest.raises(mm.Mi355xError):
        mm.repack_size(F)                                          # f32 is not a quantized type
    A = mm.tensor(qref.Q4_0, x.data_ptr(), [64, 4, 1, 1], qref.contiguous_nb(qref.Q4_0, [64, 4]))
    n = mm.repack_size(A)
    with pytest.raises(mm.Mi355xError):
        mm.repack(A, x.data_ptr(), n - 1)                          # destination too small
