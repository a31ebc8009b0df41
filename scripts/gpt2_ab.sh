#!/bin/bash
# GPT-2 engine decode rate (graph replay, scripts/gpt2_bench.py) under env variants, alternated:
#   scripts/gpt2_ab.sh "" "GGML_MI355X_FUSED_PF=2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in "$@"; do
    for ns in 1 8; do
      r=$(env $v timeout -k 10 120 python scripts/gpt2_bench.py $ns 256 1 2>&1 | tail -1) || exit 1
      echo "[$v] $r"
    done
  done
done
