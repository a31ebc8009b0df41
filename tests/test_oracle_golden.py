"""Pin the CPU oracle (oracle/qref.c) to the reference's own outputs (tests/golden/).

The fixtures were produced by oracle/gen_golden.cpp linked against the reference ggml built
from its sources (oracle/ref.mk). Bars:
  * quantize (_ref and imatrix paths), dequantize, activation quantizers: bit-exact;
  * generic vec_dot: bit-exact with ggml_vec_dot_*_generic;
  * SIMD vec_dot / full CPU-backend MUL_MAT and MUL_MAT_ID: NMSE <= 5e-6 (the oracle keeps the
    generic fp32 summation order; the x86 SIMD order differs in the last bits).
"""
import os

import numpy as np
import pytest

import golden_cases as G
import qref

RECORDS = G.manifest()


def _recs(kind):
    return [r for r in RECORDS if r["kind"] == kind]


def test_prng_numpy_matches_c():
    for seed in (0, 1234, 5678, 2**63 + 7):
        np.testing.assert_array_equal(qref.fill_uniform(5000, seed), qref.fill_uniform_c(5000, seed))


def test_inputs_match_fixture():
    x = G.load_bin("input_unif1234.f32", np.float32)
    np.testing.assert_array_equal(x, qref.fill_uniform(4096, 1234))


def test_fp16_roundtrip_exhaustive_sample():
    L = qref.lib()
    # every half value round-trips through f32 exactly
    for h in list(range(0, 0x7C01, 7)) + [0x7C00, 0xFC00, 0x8001, 0x0001, 0x3C00, 0x7BFF]:
        assert L.qref_fp32_to_fp16(L.qref_fp16_to_fp32(h)) == h


@pytest.mark.parametrize("r", _recs("quant"), ids=lambda r: r["name"])
def test_quantize_dequantize_bit_exact(r):
    x = G.load_bin(r["input"], np.float32)
    want_q = G.load_bin(r["name"] + ".q", np.uint8)
    want_d = G.load_bin(r["name"] + ".deq.f32", np.float32)
    im = np.ones(r["n"], np.float32) if r["imatrix"] else None
    got_q = qref.quantize(r["type_id"], x, n_per_row=r["n_per_row"], imatrix=im)
    np.testing.assert_array_equal(got_q, want_q)
    got_d = qref.dequantize(r["type_id"], want_q, r["n"])
    np.testing.assert_array_equal(got_d.view(np.uint32), want_d.view(np.uint32))


@pytest.mark.parametrize("r", _recs("act"), ids=lambda r: r["tag"])
def test_activation_quantizers_bit_exact(r):
    x = G.load_bin(r["input"], np.float32)
    tag = r["tag"]
    np.testing.assert_array_equal(qref.quantize_act(qref.Q8_0, x, qref.ACT_REF), G.load_bin(f"act_q8_0_ref_{tag}.q", np.uint8))
    np.testing.assert_array_equal(qref.quantize_act(qref.Q8_0, x, qref.ACT_X86), G.load_bin(f"act_q8_0_x86_{tag}.q", np.uint8))
    np.testing.assert_array_equal(qref.quantize_act(qref.Q8_1, x), G.load_bin(f"act_q8_1_ref_{tag}.q", np.uint8))
    np.testing.assert_array_equal(qref.quantize_act(qref.Q8_K, x), G.load_bin(f"act_q8_K_{tag}.q", np.uint8))


@pytest.mark.parametrize("r", _recs("vec_dot"), ids=lambda r: f'{r["type"]}_k{r["k"]}')
def test_vec_dot_generic_bit_exact(r):
    t, k = r["type_id"], r["k"]
    w = qref.quantize(t, qref.fill_uniform(4096, r["w_seed"])[:k])
    vt = qref.Q8_0 if t in (qref.Q4_0, qref.Q8_0) else qref.Q8_K
    a = qref.quantize_act(vt, qref.fill_uniform(4096, r["a_seed"])[:k], qref.ACT_X86)
    got = np.float32(qref.vec_dot(t, k, w, a))
    assert got.view(np.uint32) == np.uint32(r["generic_bits"]), (got, r["generic"])
    assert abs(float(got) - r["simd"]) <= 2e-3 * max(1.0, abs(r["simd"]))


def _mm_records():
    return [r for r in _recs("mul_mat") if r["m"] * r["k"] * r["n"] <= 4096 * 4096 * 8]


@pytest.mark.parametrize("r", _mm_records(), ids=lambda r: r["name"])
def test_mul_mat_matches_reference_cpu(r):
    a, b, out_ne = G.mul_mat_operands(r)
    got = G.oracle_mul_mat(a, b, out_ne)
    want = G.load_bin(r["name"] + ".out.f32", np.float32)
    got = got[: want.size]
    assert qref.nmse(got, want) <= 5e-6


@pytest.mark.parametrize("r", _recs("mul_mat_id"), ids=lambda r: r["name"])
def test_mul_mat_id_matches_reference_cpu(r):
    a, b, ids, out_ne = G.mul_mat_id_operands(r)
    got = G.oracle_mul_mat_id(a, b, ids, out_ne)
    want = G.load_bin(r["name"] + ".out.f32", np.float32)
    assert qref.nmse(got, want) <= 5e-6


@pytest.mark.parametrize("r", [r for r in _recs("mul_mat") if "sample_cols" in r], ids=lambda r: r["name"])
def test_big_mul_mat_oracle_vs_reference_sample_and_column_sums(r):
    """the BASELINE Q8_0 4096x4096x512 record: the oracle (threaded) matches the reference's
    sampled columns (every 128-column tile) and every column's f64 (sum, sum of squares)"""
    a, b, out_ne = G.mul_mat_operands(r)
    got = G.oracle_mul_mat(a, b, out_ne, threads=os.cpu_count() or 8).reshape(-1, out_ne[0])
    want = G.load_bin(r["name"] + ".out.f32", np.float32).reshape(len(r["sample_cols"]), -1)
    assert sorted({c // 128 for c in r["sample_cols"]}) == list(range((out_ne[1] + 127) // 128))
    assert qref.nmse(got[r["sample_cols"]], want) <= 5e-6
    cs = G.load_bin(r["colsums"], np.float64).reshape(-1, 2)
    g64 = got.astype(np.float64)
    assert np.all(np.abs(g64.sum(1) - cs[:, 0]) <= 1e-4 * np.sqrt(cs[:, 1]))
    assert np.all(np.abs((g64 ** 2).sum(1) / cs[:, 1] - 1) <= 1e-5)
