#!/bin/bash
# scripts/gpt2_geom_sweep.sh — GPT-2 decode tokens/s over fused mat-vec launch geometries
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "256 0" "1024 0" "2048 0" "1024 768" "1024 3072" "2048 3072"; do
    set -- $cfg
    echo "TALL=$1 LPR64_MAXN=$2: $(GGML_MI355X_FUSED_TALL=$1 GGML_MI355X_FUSED_LPR64_MAXN=$2 timeout -k 10 120 python scripts/gpt2_bench.py 1 256 1 2>/dev/null | tail -1)" || exit 1
done
