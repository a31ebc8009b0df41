"""GPU parity of the int8 tile's stream-K form (csrc/mmq8.hip, mmq8_kernel<..., SK>): the in-place
tile only (the repacked tile has no stream-K form), so these cases sit outside test_mmq8.py's
in-place / repacked parametrization."""
import numpy as np
import pytest

import qref
from test_gpu_parity import mm  # noqa: F401  (fixture)
from test_mmq8 import TYPES, case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("t", TYPES, ids=lambda t: qref.NAMES[t])
@pytest.mark.parametrize("shape", [(4224, 1024, 768, None), (8192, 640, 512, None), (4160, 1152, 1024, None),
                                   (8320, 520, 256, None), (4224, 1024, 768, 64)],
                         ids=lambda s: "x".join(map(str, s[:3])) + (f"_tt{s[3]}" if s[3] else ""))
def test_mmq8_stream_k(mm, t, shape):
    """stream-K (GGML_MI355X_MMQ8_SK=1): more 128-row tiles than the 256 workgroups, so the
    (tile, super-block) units split unevenly and tiles are finished by a second workgroup through
    the write-through partial + counter hand-off; against the oracle, bit-identical on a second
    run (two operands per tile: the order of arrival does not change the sum) and within the
    fp32 scale-sum order of the plain tiles (SK=0)"""
    N, M_, K, tt = shape
    if qref.BLCK[t] == 256 and K % 256:
        K = 768
    g1 = case(mm, t, N, M_, K, seed=13, sk=1, tt=tt, ret_got=True)
    g2 = case(mm, t, N, M_, K, seed=13, sk=1, tt=tt, ret_got=True)
    assert np.array_equal(g1.view(np.uint32), g2.view(np.uint32)), "stream-K result not repeatable"
    g0 = case(mm, t, N, M_, K, seed=13, sk=0, tt=tt, ret_got=True)
    assert qref.nmse(g1, g0) <= 1e-9
