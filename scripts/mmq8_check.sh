#!/bin/bash
# mmq8 iteration loop on the GPU box: mat-mat parity tests, then timings of the BASELINE
# mat-mat shapes (hipGraph period incl. the activation pass) and a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmq8.py tests/test_gpu_parity.py tests/test_mmq_range.py > gpurun_out/mmq8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mmq8_tests.log; [ $rc -eq 0 ] || exit $rc
S=${SHAPES:-"q8_0:4096:4096:512 q4_0:4096:4096:512 q4_K:4096:4096:512 q5_K:4096:4096:512 q6_K:4096:11008:512 q4_K:4096:4096:128 q4_K:4096:4096:32 q8_0:4096:4096:2048"}
timeout -k 10 200 python scripts/mmq_bench.py $S 2>&1 | grep tile || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m8 -o run -- python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 > /dev/null 2>&1 || exit 1
cut -d, -f1-4 gpurun_out/m8/run_kernel_stats.csv | head -8
