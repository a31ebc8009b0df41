#!/bin/bash
# in-place int8 tile: 64- vs 128-token tiles (GGML_MI355X_MMQ8_TT) near the switch-over rule
# (128 once >= 256 such tiles), two repeats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${SHAPES:-"q8_0:4096:11008:512 q4_K:4096:11008:512 q6_K:4096:11008:512 q8_0:4096:4096:1024 q4_K:4096:4096:1024 q8_0:4096:4096:768 q8_0:4096:8192:512"}
for rep in 1 2; do
  for tt in 64 128; do
    echo "== rep $rep TT=$tt"
    GGML_MI355X_MMQ8_TT=$tt MMQ_REPACKED=0 timeout -k 10 300 python scripts/mmq_bench.py $S || exit $?
  done
done
