"""Huge block scales on the mat-mat path: the int8 tile (csrc/mmq8.hip, every K and 2-byte-aligned
layout) converts every scale to f32, so it is exact at any M, including the K = 96 k shapes
(tests/test_mmq8.py covers M = 200 and 512 for all five types). (The f16 tiles that overflowed
past d > 511 were removed in round 5.) Checked against the CPU oracle on rows mixing ordinary and
huge scales."""

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
    return M


@pytest.fixture(params=["inplace", "repack"])
def path(request, mm):
    """the int8 tile on the weights in place, and on a per-call repacked copy"""
    with mm.knobs(GGML_MI355X_MMQ_REPACK_MIN=9 if request.param == "repack" else None):
        yield request.param


@pytest.mark.parametrize("t,big", [(qref.Q8_0, 7.0e4), (qref.Q4_K, 2.0e3), (qref.Q4_0, 1.0e5)])
@pytest.mark.parametrize("M,K", [(16, 512), (40, 512), (200, 96 * 3), (512, 96 * 5)])
def test_huge_scales_match_oracle(mm, path, t, big, M, K):
    if qref.BLCK[t] == 256 and K % 256:
        K = 768
    N = 160
    f = qref.fill_uniform(N * K, 77).reshape(N, K)
    f[5::7] *= big                      # every 7th row: block scales >= 1.0
    w = qref.quantize(t, f.reshape(-1), n_per_row=K)
    x = qref.fill_uniform(M * K, 78)
    a = G.Operand(t, w, [K, N, 1, 1], qref.contiguous_nb(t, [K, N, 1, 1]))
    b = G.Operand(qref.F32, x.view(np.uint8).copy(), [K, M, 1, 1], qref.contiguous_nb(qref.F32, [K, M, 1, 1]))
    import test_gpu_parity as T
    got = T.run_mul_mat(mm, a, b, [N, M, 1, 1])
    want = G.oracle_mul_mat(a, b, [N, M, 1, 1])
    assert np.all(np.isfinite(got))
    assert qref.nmse(got, want) <= 5e-4
    # the ordinary rows stay as accurate as without the huge ones
    keep = np.ones(N, bool)
    keep[5::7] = False
    g2, w2 = got.reshape(M, N)[:, keep], want.reshape(M, N)[:, keep]
    assert qref.nmse(g2, w2) <= 5e-4
