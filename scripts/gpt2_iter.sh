#!/bin/bash
# GPT-2 engine iteration on the GPU box: its parity tests, then decode timings (1 and 8 sequences)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2.py tests/test_gpt2_example.py tests/test_gpt2_pipeline.py > gpurun_out/gpt2_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpt2_tests.log; [ $rc -eq 0 ] || exit $rc
for a in "1 256 1" "1 256 1" "8 256 1"; do timeout -k 10 120 python scripts/gpt2_bench.py $a || exit 1; done
