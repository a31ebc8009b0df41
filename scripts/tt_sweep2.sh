#!/bin/bash
# in-place int8 tile: 64- vs 128-token tiles between 129 and 255 128-token tiles (no split-K),
# and the repacked copy at the same shapes, two repeats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${SHAPES:-"q8_0:4096:4096:576 q8_0:4096:5120:512 q8_0:4096:6144:512 q8_0:4096:4096:768 q4_K:4096:4096:768 q6_K:4096:4096:768 q4_K:4096:5120:512"}
for rep in 1 2; do
  for tt in 64 128; do
    echo "== rep $rep TT=$tt"
    GGML_MI355X_MMQ8_TT=$tt MMQ_REPACKED=0 timeout -k 10 300 python scripts/mmq_bench.py $S || exit $?
  done
  echo "== rep $rep repacked copy"
  GGML_MI355X_MMQ_RP_ALL=1 MMQ_REPACKED=1 timeout -k 10 300 python scripts/mmq_bench.py $S || exit $?
done
