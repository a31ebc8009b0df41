#!/bin/bash
# in-place tile vs the repacked copy at the shapes where the in-place tile runs 128-token tiles
# (GGML_MI355X_MMQ_RP_ALL=1 forces the copy), per type, plus narrow M.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${SHAPES:-"q4_0:4096:11008:512 q8_0:4096:11008:512 q4_K:4096:11008:512 q5_K:4096:11008:512 q6_K:4096:11008:512 q6_K:4096:4096:2048 q5_K:4096:4096:2048 q4_0:4096:4096:2048 q4_K:4096:4096:128 q4_K:4096:4096:256 q6_K:4096:4096:1024"}
for rep in 1 2; do
  echo "== rep $rep in place"
  MMQ_REPACKED=0 timeout -k 10 300 python scripts/mmq_bench.py $S || exit $?
  echo "== rep $rep repacked copy"
  GGML_MI355X_MMQ_RP_ALL=1 MMQ_REPACKED=1 timeout -k 10 300 python scripts/mmq_bench.py $S || exit $?
done
