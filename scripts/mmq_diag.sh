#!/bin/bash
# MMQ ablation probe: GGML_MI355X_DIAG bits skip parts of the tile kernel
# (1 = MFMA phase, 2 = weight decode, 4 = activation loads, 8 = weight loads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in 0 1 2 4 8 12 15; do
    echo "--- diag=$d"
    GGML_MI355X_DIAG=$d timeout -k 10 120 python scripts/mmq_bench.py "$@" 2>&1 | grep tile || exit $?
done
