#!/bin/bash
# scripts/gpu_r06_mvgraph.sh — graph periods of the multi-column mat-vec at the reference perf
# shapes, with and without the column pre-pass launch (GGML_MI355X_DIAG=256: measurement only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=""
for t in q4_0 q8_0 q4_K q5_K q6_K; do for n in 1 2 4 8; do S="$S $t:14336:4096:$n"; done; done
for r in 1 2; do
  timeout -k 10 300 python scripts/mv_graph.py $S || exit 1
  GGML_MI355X_DIAG=256 timeout -k 10 300 python scripts/mv_graph.py $S || exit 1
done
