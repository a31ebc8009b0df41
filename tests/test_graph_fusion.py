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


def _run(fusion: bool):
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref/fusion_check not built")
    env = dict(os.environ, GGML_MI355X_DEBUG="1", GGML_MI355X_FUSION="1" if fusion else "0")
    r = subprocess.run([BIN, LIB], capture_output=True, text=True, env=env, timeout=300)
    fails = [l for l in r.stdout.splitlines() if l.startswith("FAIL")]
    assert r.returncode == 0 and "FUSION_CHECK_OK" in r.stdout, (fails, r.stdout[-1500:], r.stderr[-1500:])
    fused = {}
    case = None
    for line in r.stderr.splitlines():
        if line.startswith("CASE "):
            case = line[5:].strip()
            fused[case] = []
        m = re.search(r"fused (\d+) nodes", line)
        if m and case is not None:
            fused[case].append(int(m.group(1)))
    return fused


def test_fused_chains_match_cpu_and_fuse():
    fused = _run(True)
    for t in ("q4_0", "q8_0", "q4_K", "q5_K", "q6_K"):
        for m in (1, 3, 8):
            tag = f"{t} M={m}"
            assert fused[f"ln_matvec_bias {tag}"] == [5], tag
            assert fused[f"mlp {tag}"] == [6, 3], tag
            assert fused[f"ln_matvec {tag}"] == [4], tag
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


def test_unfused_graph_matches_cpu():
    fused = _run(False)
    assert all(v == [] for v in fused.values()), fused
