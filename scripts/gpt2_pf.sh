#!/bin/bash
# GPT-2 attention-block iteration: engine + drop-in parity tests, A/B against scratch_libs variants, phase stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2.py tests/test_gpt2_example.py > gpurun_out/gpt2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpt2_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/gpt2_ab.sh head "$@" || exit 1
timeout -k 10 200 python scripts/block_stamps.py 24 64 2>&1 | grep -v amdgpu.ids | head -20 || exit 1
timeout -k 10 200 python scripts/block_stamps.py 24 200 2>&1 | grep -v amdgpu.ids | head -10
