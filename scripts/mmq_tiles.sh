#!/bin/bash
# scripts/mmq_tiles.sh — parity of the mat-mat tile variants (GGML_MI355X_MMQ_TILE) on the
# golden MUL_MAT records, then their timings (scripts/mmq_bench.py). Usage: mmq_tiles.sh tile...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in "$@"; do
    echo "=== parity $t"
    GGML_MI355X_MMQ_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mul_mat_vs" -x -q \
        --timeout 120 --timeout-method thread > gpurun_out/tiles_$t.log 2>&1
    rc=$?; tail -n 3 gpurun_out/tiles_$t.log
    case $rc in 124|134|137|139) echo "crash-class exit $rc"; exit $rc;; esac
done
for t in "$@"; do
    GGML_MI355X_MMQ_TILE=$t timeout -k 10 200 python scripts/mmq_bench.py ${MMQ_SHAPES:-} || exit $?
done
