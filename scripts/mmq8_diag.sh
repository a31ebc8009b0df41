#!/bin/bash
# where the int8 mat-mat time goes: GGML_MI355X_DIAG bits (1 no activation DMA, 2 no weight
# loads, 4 no compute) on the BASELINE shape and a K-quant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in 0 1 2 4 3 5 6 7; do
  echo "diag=$d"
  timeout -k 10 100 env GGML_MI355X_MMQ=i8 GGML_MI355X_DIAG=$d python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 2>&1 | grep tile || exit 1
done
