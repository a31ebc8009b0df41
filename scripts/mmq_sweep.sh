#!/bin/bash
# MMQ tile-shape sweep (probe): one process per tile setting (the choice is read once per process)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for t in ${MMQ_TILES:-auto 64x128 128x64 128x128 128x128w4 64x128w4}; do
    GGML_MI355X_MMQ_TILE=$t timeout -k 10 300 python scripts/mmq_bench.py "$@" || exit $?
done
