#!/bin/bash
# scripts/gpu_r06_wgs.sh — the whole-K mat-vec's workgroup target (GGML_MI355X_MMVQ_WGS) on the
# bench's stacked launches, variants interleaved over three rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wgs; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for w in 2048 3072 4096 6144; do
    GGML_MI355X_MMVQ_WGS=$w timeout -k 10 120 python scripts/mmvq_bench.py q4_0:4096:4096:1:64 q4_K:4096:4096:1:64 q4_K:4096:11008:1:24 q5_K:4096:11008:1:24 q6_K:4096:11008:1:24 q8_0:4096:4096:1:64 2>&1 | grep GB/s >> $O/wgs.txt || exit 1
  done
done
cat $O/wgs.txt
