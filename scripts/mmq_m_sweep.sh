#!/bin/bash
# Q8_0 / Q4_K 4096x4096 mat-mat over M, in-place tile vs repacked tile (hipGraph period incl. the
# activation pass, HBM-cold), three repeats each so the box-to-box spread is visible.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S="q8_0:4096:4096:512 q8_0:4096:4096:1024 q8_0:4096:4096:2048 q4_K:4096:4096:2048"
for rep in 1 2 3; do
  for mode in 0 1; do
    echo "== rep $rep MMQ_REPACKED=$mode"
    MMQ_REPACKED=$mode timeout -k 10 200 python scripts/mmq_bench.py $S || exit $?
  done
done
