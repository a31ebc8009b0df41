#!/bin/bash
# A/B of the mat-vec weight staging (probe): LDS-DMA ring vs register-staged loads, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in 1 0 1 0; do
    GGML_MI355X_MMVQ_DMA=$d timeout -k 10 300 python scripts/mmvq_bench.py "$@" 2>&1 | grep GB/s || exit $?
done
