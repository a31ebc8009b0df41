#!/bin/bash
# mat-vec launch-width sweep (probe): GGML_MI355X_MMVQ_WGS = target workgroups per launch
# usage: scripts/mmvq_sweep.sh "512 1024 ..." [type:K:N:M:batch ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
list=${1:-"512 1024 1536 2048 4096"}; shift
for w in $list; do
    GGML_MI355X_MMVQ_WGS=$w timeout -k 10 300 python scripts/mmvq_bench.py "$@" 2>&1 | grep GB/s || exit $?
done
