"""Graph fusion in the plugin's graph_compute (backend.cpp fuse_matvec / fuse_softmax), driven
through the reference's graph API and allocator by oracle/_ref/fusion_check (GPU box).

Every case is computed by the plugin and by ggml-cpu (NMSE <= 5e-4, test-backend-ops' MUL_MAT
bar). With GGML_MI355X_DEBUG the plugin lists each fused run; the test pins which runs fuse:
the GPT-2 chains do (main-sched.cpp:603-637, 690-706, 744-757, 765-847), a chain whose
intermediate is a requested output or has a second consumer does not (the reference's rule,
src/ggml-impl.h:548-603). GGML_MI355X_FUSION=0 must give the same results with no fused run.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "fusion_check")
LIB = os.path.join(ROOT, "ggml-gfx906_amd", "libggml-hip-mi355x.so")

pytestmark = pytest.mark.gpu


folds = {}   # copies folded into a fused mat-vec, by case (filled by _run)
embeds = {}  # fused embedding launches, by case
layers = {}  # whole GPT-2 layers fused (plan_layers), by case


def _run(fusion: bool, **extra):
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref/fusion_check not built")
    env = dict(os.environ, GGML_MI355X_DEBUG="1", GGML_MI355X_FUSION="1" if fusion else "0", **extra)
    r = subprocess.run([BIN, LIB], capture_output=True, text=True, env=env, timeout=300)
    fails = [l for l in r.stdout.splitlines() if l.startswith("FAIL")]
    assert r.returncode == 0 and "FUSION_CHECK_OK" in r.stdout, (fails, r.stdout[-1500:], r.stderr[-1500:])
    fused, attn, pairs = {}, {}, {}
    folds.clear()
    embeds.clear()
    layers.clear()
    case = None
    for line in r.stderr.splitlines():
        if line.startswith("CASE "):
            case = line[5:].strip()
            fused[case] = []
            attn[case] = 0
            pairs[case] = 0
            folds[case] = 0
            embeds[case] = 0
            layers[case] = 0
        if "layer fused" in line and case is not None:
            layers[case] += 1
        if "fused embedding" in line and case is not None:
            embeds[case] += 1
        if "folded into the mat-vec's epilogue" in line and case is not None:
            folds[case] += 1
        m = re.search(r"fused (\d+) nodes", line)
        if m and case is not None:
            fused[case].append(int(m.group(1)))
        if "fused attention" in line and case is not None:
            attn[case] += 1
        if "fused 2 copies" in line and case is not None:
            pairs[case] += 1
    return fused, attn, pairs


@pytest.mark.parametrize("attn_kernel", ["d64", "generic"])
def test_fused_chains_match_cpu_and_fuse(attn_kernel):
    extra = {"GGML_MI355X_ATTN_GENERIC": "1"} if attn_kernel == "generic" else {}
    fused, attn, pairs = _run(True, **extra)
    for t in ("q4_0", "q8_0", "q4_K", "q5_K", "q6_K"):
        for m in (1, 3, 8):
            tag = f"{t} M={m}"
            assert fused[f"ln_matvec_bias {tag}"] == [5], tag
            assert fused[f"mlp {tag}"] == [6, 3], tag
            assert fused[f"ln_matvec {tag}"] == [4], tag
            # c_attn + bias fuses and both cache writes ride in its epilogue (caches read back whole)
            assert fused[f"qkv_cache {tag}"] == [2] and folds[f"qkv_cache {tag}"] == 2, (tag, fused[f"qkv_cache {tag}"])
            if m > 1:   # wte rows + wpe rows in one launch, bit-identical to ggml-cpu (checked by fusion_check)
                assert embeds[f"embed {tag}"] == 1, tag
    # the norm is an output: at most MUL_MAT + bias fuses ([]: its result landed on the freed input)
    assert fused["neg_output_flag"] in ([2], [])
    assert fused["neg_second_use"] == []        # the mat-vec result has two consumers
    # [2]: ggml-alloc put the sum in place over x, which the mat-vec reads, so only + bias fuses
    assert fused["resid_first_operand"] in ([3], [2])
    assert fused["freed_input"] in ([5], [2])   # [2]: the result landed on the freed input
    for k, v in fused.items():
        if k.startswith("softmax_chain"):
            assert v == [3], k
        elif k.startswith("softmax_mask_only"):
            assert v == [2], k
        elif k.startswith("attention ") or k.startswith("attention_f16"):   # the read side is one launch,
            assert v == [] and attn[k] == 1 and pairs[k] == 1, (k, v, attn[k], pairs[k])  # the cache writes another
        elif k.startswith("attention_sm_output"):  # soft_max is an output: scale/mask/soft_max only
            assert v == [3] and attn[k] == 0, (k, v, attn[k])
    assert sum(1 for k in attn if k.startswith("attention ")) == 6
    # the whole-layer cases: every compute plans the layer as one run (a replayed hipGraph plans
    # nothing), and every step matched ggml-cpu (fusion_check prints FAIL otherwise)
    for t in ("q4_0", "q8_0", "q4_K", "q5_K", "q6_K"):
        assert layers[f"gpt2_layer {t}"] >= 1, (t, layers[f"gpt2_layer {t}"])


def test_unfused_graph_matches_cpu():
    fused, attn, pairs = _run(False)
    assert all(v == [] for v in fused.values()), fused
    assert not any(attn.values()) and not any(pairs.values()) and not any(folds.values()), (attn, pairs, folds)
    assert not any(embeds.values()), embeds
    assert not any(layers.values()), layers
