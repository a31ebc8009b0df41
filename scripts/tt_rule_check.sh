#!/bin/bash
# after the token-tile rule change: full GPU suite + smoke, then the default dispatch and the
# repacked buffer over the swept shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
scripts/gpu_session.sh testsall smoke || exit $?
S="q8_0:4096:4096:512 q8_0:4096:4096:576 q8_0:4096:4096:768 q4_K:4096:4096:768 q6_K:4096:4096:768 q8_0:4096:6144:512 q8_0:4096:11008:512 q6_K:4096:11008:512 q8_0:4096:4096:2048"
for mode in 0 1; do
  echo "== MMQ_REPACKED=$mode"
  MMQ_REPACKED=$mode timeout -k 10 300 python scripts/mmq_bench.py $S || exit $?
done
