#!/bin/bash
# A/B of variant library builds on the headline: scripts/ab_bench.sh lib1.so lib2.so ... (each
# run twice, interleaved, on one box); prints value and the headline kernel's event time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2; do
  for L in "$@"; do
    out=$(timeout -k 10 200 env GGML_MI355X_LIB=$PWD/$L python bench.py --no-extra --no-gpt2 --cpu-seconds 1 2>/dev/null | tail -1) || exit 1
    echo "$(basename $L .so) $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['roofline']['launch_us'], d['roofline']['frac'])" "$out")"
  done
done
