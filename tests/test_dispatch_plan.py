"""CPU: which kernels MUL_MAT dispatches to, pinned for the benchmark shapes (BASELINE.json configs
and the bench's headline) and for test-backend-ops' perf shapes (reference
tests/test-backend-ops.cpp:6195-6202: every type, K = 14336, N = 4096, bs 1..8 and 512).

ggml_mi355x_mul_mat_plan runs the same routing code as ggml_mi355x_mul_mat (dispatch.cpp
mul_mat_route) but launches nothing, so this needs no GPU. A change to a dispatch rule or a launch
plan must show up here as a reviewed diff of PLANS. Also: supports_op for MUL_MAT_ID agrees with
what mul_mat_id accepts (whole-K activations in LDS cap K), and every knob goes
through the settings snapshot (ggml_mi355x_reload_settings)."""
import pytest

import mi355x_qmm as M

F32 = M.F32
TYPES = {"q4_0": M.Q4_0, "q8_0": M.Q8_0, "q4_K": M.Q4_K, "q5_K": M.Q5_K, "q6_K": M.Q6_K}


@pytest.fixture(scope="module")
def lib():
    M.build()
    L = M.lib()
    M.reload_settings()
    return L


def plan(t, K, N, cols, mats=1, repacked=False, addr=0x100000):
    a = M.tensor(t, addr, [K, N, mats, 1], M.contiguous_nb(t, [K, N, mats, 1]))
    b = M.tensor(F32, addr, [K, cols, mats, 1], M.contiguous_nb(F32, [K, cols, mats, 1]))
    return M.mul_mat_plan(a, b, repacked)


# (name, type, K, N, columns, matrices per call) -> plan text
PLANS = {
    # BASELINE configs[1] and the north-star shape: one matrix per launch, M = 1 (graph periods
    # put the 8-wave kernel ahead of the single-wave one at 4096 rows, mmvq_solo.hip)
    ("q4_0", 4096, 4096, 1, 1): "mmvq nc=1 lpr=64 rpw=2 grid=256x1x1",
    ("q4_K", 4096, 4096, 1, 1): "mmvq nc=1 lpr=64 rpw=2 grid=256x1x1",
    ("q8_0", 4096, 4096, 1, 1): "mmvq-solo rows=8 grid=512",
    # bench.py headline: 64 stacked matrices per MUL_MAT
    ("q4_0", 4096, 4096, 1, 64): "mmvq nc=1 lpr=64 rpw=2 grid=64x64x1",
    ("q4_K", 4096, 4096, 1, 64): "mmvq nc=1 lpr=64 rpw=2 grid=64x64x1",
    # BASELINE configs[2]: 4096 x 11008 k-quants, M = 1
    ("q4_K", 4096, 11008, 1, 1): "mmvq-solo rows=8 grid=1376",
    ("q5_K", 4096, 11008, 1, 1): "mmvq-solo rows=8 grid=1376",
    ("q6_K", 4096, 11008, 1, 1): "mmvq-solo rows=4 grid=2752",
    # below 4096 rows the 8-wave kernel (two rows per wave from 4096 rows on)
    ("q4_K", 4096, 2048, 1, 1): "mmvq nc=1 lpr=64 rpw=1 grid=256x1x1",
    # BASELINE configs[3]: the int8 MFMA tile
    ("q8_0", 4096, 4096, 512, 1): "mmq8 tile=128x64 tiles=256 ksplit=1",
}
# test-backend-ops perf (tests/test-backend-ops.cpp:6195-6202): K = 14336, N = 4096, (type, bs)
PERF = {
    ("q4_0", 1): "ring nc=1 rpw=1 cols=1",
    ("q4_0", 2): "ring nc=2 rpw=2 cols=2",
    ("q4_0", 3): "mma tok=4 kh=1 rt=1 paired run=8 cols=3",
    ("q4_0", 4): "mma tok=4 kh=1 rt=1 paired run=8 cols=4",
    ("q4_0", 5): "mma tok=8 kh=1 rt=1 paired run=8 cols=5",
    ("q4_0", 8): "mma tok=8 kh=1 rt=1 paired run=8 cols=8",
    ("q4_0", 512): "mmq8 tile=128x64 tiles=256 ksplit=1",
    ("q8_0", 1): "ring nc=1 rpw=1 cols=1",
    ("q8_0", 2): "ring nc=2 rpw=2 cols=2",
    ("q8_0", 3): "mma tok=4 kh=1 rt=1 paired run=8 cols=3",
    ("q8_0", 4): "mma tok=4 kh=1 rt=1 paired run=8 cols=4",
    ("q8_0", 5): "mma tok=8 kh=1 rt=1 paired run=8 cols=5",
    ("q8_0", 8): "mma tok=8 kh=1 rt=1 paired run=8 cols=8",
    ("q8_0", 512): "mmq8 tile=128x64 tiles=256 ksplit=1",
    ("q4_K", 1): "ring nc=1 rpw=2 cols=1",
    ("q4_K", 2): "ring nc=2 rpw=2 cols=2",
    ("q4_K", 3): "mma tok=4 kh=1 rt=1 paired run=8 cols=3",
    ("q4_K", 4): "mma tok=4 kh=1 rt=1 paired run=8 cols=4",
    ("q4_K", 5): "mma tok=8 kh=1 rt=1 run=7 cols=5",
    ("q4_K", 8): "mma tok=8 kh=1 rt=1 run=7 cols=8",
    ("q4_K", 512): "mmq8 tile=128x64 tiles=256 ksplit=1",
    ("q5_K", 1): "ring nc=1 rpw=2 cols=1",
    ("q5_K", 2): "ring nc=2 rpw=2 cols=2",
    ("q5_K", 3): "mma tok=4 kh=1 rt=1 paired run=8 cols=3",
    ("q5_K", 4): "mma tok=4 kh=1 rt=1 paired run=8 cols=4",
    ("q5_K", 5): "mma tok=8 kh=1 rt=1 paired run=8 cols=5",
    ("q5_K", 8): "mma tok=8 kh=1 rt=1 paired run=8 cols=8",
    ("q5_K", 512): "mmq8 tile=128x64 tiles=256 ksplit=1",
    ("q6_K", 1): "ring nc=1 rpw=1 cols=1",
    ("q6_K", 2): "ring nc=2 rpw=1 cols=2",
    ("q6_K", 3): "mma tok=4 kh=1 rt=1 run=7 cols=3",
    ("q6_K", 4): "mma tok=4 kh=1 rt=1 run=7 cols=4",
    ("q6_K", 5): "mma tok=8 kh=1 rt=1 run=7 cols=5",
    ("q6_K", 8): "mma tok=8 kh=1 rt=1 run=7 cols=8",
    ("q6_K", 512): "mmq8 tile=128x64 tiles=256 ksplit=1",
}


# the MFMA mat-vec rule's branches (dispatch.cpp use_mma, mmvq_mma.hip mma_plan; round-6 graph
# sweep profiles/r06_mma_plan_sweep.txt): (name, K, N, columns) -> plan text
MMA_RULE = {
    ("q4_0", 4096, 4096, 4): "mmvq nc=4 lpr=64 rpw=2 grid=256x1x1",           # small: VALU up to 4
    ("q4_0", 4096, 4096, 5): "mma tok=8 kh=1 rt=1 paired run=2 cols=5",       # one K part, one tile
    ("q4_0", 8192, 8192, 3): "mma tok=4 kh=1 rt=2 paired run=4 cols=3",       # two tiles at N, K >= 8192
    ("q4_0", 4096, 14336, 8): "mma tok=8 kh=1 rt=2 paired run=2 cols=8",      # two tiles at N >= 12288
    ("q8_0", 11008, 4096, 3): "mma tok=4 kh=1 rt=1 run=6 cols=3",             # unpaired, one tile
    ("q8_0", 8192, 4096, 4): "ring-pre nc=4 rpw=1 cols=4",                    # K < 11008: from 5
    ("q8_0", 8192, 4096, 5): "mma tok=8 kh=1 rt=1 run=4 cols=5",
    ("q4_K", 4096, 14336, 8): "mma tok=8 kh=1 rt=2 run=2 cols=8",
    ("q4_K", 14336, 4096, 8): "mma tok=8 kh=1 rt=1 run=7 cols=8",             # one tile: one part fits
    ("q4_K", 24576, 4096, 8): "mma tok=8 kh=2 rt=2 run=6 cols=8",             # image past LDS: two parts
    ("q4_K", 28672, 4096, 8): "ring-pre nc=8 rpw=1 cols=8",                   # no part size fits: VALU
    ("q4_K", 28672, 4096, 3): "mma tok=4 kh=1 rt=1 paired run=14 cols=3",     # 1..4 columns from K = 12288: pairs
    ("q4_K", 11008, 4096, 3): "mma tok=4 kh=1 rt=1 run=6 cols=3",
    ("q5_K", 4096, 4096, 5): "mma tok=8 kh=1 rt=1 paired run=2 cols=5",       # pairs: one part (S < 64)
    ("q5_K", 8192, 4096, 5): "mma tok=8 kh=1 rt=1 paired run=4 cols=5",
    ("q5_K", 14336, 4096, 3): "mma tok=4 kh=1 rt=1 paired run=8 cols=3",
    ("q5_K", 14336, 4096, 5): "mma tok=8 kh=1 rt=1 paired run=8 cols=5",
    ("q5_K", 28672, 4096, 3): "mma tok=4 kh=1 rt=1 paired run=14 cols=3",     # paired: from 3 at any K
    ("q5_K", 28672, 4096, 5): "ring-pre nc=8 rpw=1 cols=5",                   # two parts: unpaired, VALU to 7
    ("q5_K", 11008, 4096, 3): "mma tok=4 kh=1 rt=1 run=6 cols=3",             # rows off 128-B lines: unpaired
    # Q6_K (round 6, profiles/r06_q6k_mma.txt)
    ("q6_K", 4096, 4096, 3): "mmvq nc=3 lpr=64 rpw=1 grid=512x1x1",           # K < 8192: from 5
    ("q6_K", 4096, 4096, 5): "mma tok=8 kh=2 rt=1 run=1 cols=5",              # small: two parts
    ("q6_K", 11008, 4096, 5): "ring-pre nc=8 rpw=1 cols=5",                   # 8192 <= K < 12288, N < 8192: 8
    ("q6_K", 11008, 4096, 8): "mma tok=8 kh=1 rt=1 run=6 cols=8",
    ("q6_K", 8192, 8192, 3): "mma tok=4 kh=1 rt=1 run=4 cols=3",              # N >= 8192: from 3
    ("q6_K", 28672, 4096, 3): "mma tok=4 kh=1 rt=1 run=14 cols=3",
    ("q6_K", 28672, 4096, 8): "mma tok=8 kh=2 rt=1 run=7 cols=8",             # image past LDS: two parts
}


def test_mma_rule(lib):
    for (name, K, N, cols), want in MMA_RULE.items():
        got = plan(TYPES[name], K, N, cols)
        assert got == want, f"{name} K={K} N={N} cols={cols}: {got!r}"


def test_baseline_shapes(lib):
    for (name, K, N, cols, mats), want in PLANS.items():
        got = plan(TYPES[name], K, N, cols, mats)
        assert got == want, f"{name} K={K} N={N} cols={cols} mats={mats}: {got!r}"


def test_reference_perf_shapes(lib):
    for (name, bs), want in PERF.items():
        got = plan(TYPES[name], 14336, 4096, bs)
        assert got == want, f"{name} bs={bs}: {got!r}"


def test_mul_mat_id_support_matches_compute(lib):
    """the backend claimed MUL_MAT_ID at any K <= 2^24, but mul_mat_id keeps
    a column's whole K in LDS; supports_op must decline what compute would refuse"""
    for K, ok in ((4096, True), (14336, True), (65536, True), (131072, False)):
        t = M.Q4_0
        a = M.tensor(t, 0x1000, [K, 64, 8, 1], M.contiguous_nb(t, [K, 64, 8, 1]))
        b = M.tensor(F32, 0x1000, [K, 2, 4, 1], M.contiguous_nb(F32, [K, 2, 4, 1]))
        ids = M.tensor(M.I32, 0x1000, [2, 4, 1, 1], [4, 8, 32, 32])
        assert M.supports_mul_mat_id(a, b, ids) == ok, K


def test_settings_reload(lib):
    """a knob changes the plan only after reload_settings (no getenv on the call path)"""
    import os
    base = plan(M.Q4_0, 14336, 4096, 8)
    assert base.startswith("mma"), base
    os.environ["GGML_MI355X_MMA"] = "0"
    try:
        assert plan(M.Q4_0, 14336, 4096, 8) == base          # not re-read per call
        M.reload_settings()
        assert not plan(M.Q4_0, 14336, 4096, 8).startswith("mma")
    finally:
        os.environ.pop("GGML_MI355X_MMA", None)
        M.reload_settings()
    assert plan(M.Q4_0, 14336, 4096, 8) == base
    with M.knobs(GGML_MI355X_MMQ8_SK=1, GGML_MI355X_MMQ8_TT=128):
        assert "tile=128x128" in plan(M.Q8_0, 4096, 4096, 512)
    assert plan(M.Q8_0, 4096, 4096, 512) == PLANS[("q8_0", 4096, 4096, 512, 1)]


def test_mma_refused_shapes_take_valu(lib):
    """paired Q4_0 at K = 25600 with 5..8 columns and Q4_K past K = 55296 with 3
    columns would need an MFMA run longer than the launcher's LDS image (since round 6 sized per
    instantiation: its static arrays, 12-32 KB, are what the image cannot use): the plan must
    not pick the MFMA mat-vec there (the launcher would refuse it)"""
    assert not plan(M.Q4_0, 25600, 4096, 5).startswith("mma")
    assert not plan(M.Q4_K, 55552, 4096, 3).startswith("mma")
    assert plan(M.Q4_K, 55296, 4096, 3).startswith("mma")
    assert plan(M.Q4_0, 24576, 4096, 5).startswith("mma")   # (just below: still taken)
