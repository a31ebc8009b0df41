#!/bin/bash
# f16 tiles vs the int8 tile variants (rows x tokens per workgroup) on the mat-mat shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=${SHAPES:-"q8_0:4096:4096:512 q4_0:4096:4096:512 q4_K:4096:4096:512 q5_K:4096:4096:512 q6_K:4096:11008:512 q4_K:4096:4096:128 q4_K:4096:4096:32 q8_0:4096:4096:2048 q4_K:4096:4096:2048"}
for v in ${VARIANTS:-f16 i8:128:64 i8:64:64 i8:128:128}; do
  echo "== $v"
  if [ "$v" = f16 ]; then E="GGML_MI355X_MMQ=f16"; else IFS=: read _ tr tt <<< "$v"; E="GGML_MI355X_MMQ=i8 GGML_MI355X_MMQ8_TR=$tr GGML_MI355X_MMQ8_TT=$tt"; fi
  timeout -k 10 150 env $E python scripts/mmq_bench.py $S 2>&1 | grep tile || exit 1
done
