#!/bin/bash
# repacked-copy routing check: the repack / mat-mat / drop-in parity tests, then the in-place
# tile vs the repacked buffer (with its routing) over M and N.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_repack.py tests/test_mmq8.py tests/test_drop_in.py > gpurun_out/rp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rp_tests.log; [ $rc -eq 0 ] || exit $rc
S=${SHAPES:-"q8_0:4096:4096:512 q8_0:4096:4096:1024 q8_0:4096:4096:2048 q4_K:4096:4096:512 q4_K:4096:4096:2048 q6_K:4096:11008:512 q8_0:4096:11008:512"}
for mode in 0 1; do
  echo "== MMQ_REPACKED=$mode"
  MMQ_REPACKED=$mode timeout -k 10 200 python scripts/mmq_bench.py $S || exit $?
done
