#!/bin/bash
# scripts/gpu_r06_knobs.sh — GPT-2 decode (scripts/gpt2_bench.py, graph replay) and the headline
# launch (64 stacked matrices) under knob variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/knobs; rm -rf $O; mkdir -p $O
for v in "" GGML_MI355X_FUSED_WGS=128 GGML_MI355X_FUSED_WGS=512 GGML_MI355X_FUSED_TALL=128 GGML_MI355X_FUSED_TALL=512 GGML_MI355X_FUSED_LPR64_MAXN=0 GGML_MI355X_FUSED_LPR64_MAXN=4096 GGML_MI355X_LPR=64 GGML_MI355X_LPR=16; do
  echo "== $v" >> $O/gpt2.txt
  timeout -k 10 120 env $v python scripts/gpt2_bench.py 1 256 1 2>&1 | grep tokens >> $O/gpt2.txt || exit 1
done
for v in "" GGML_MI355X_RPW=1 GGML_MI355X_LPR=16 GGML_MI355X_MMVQ_WGS=1024 GGML_MI355X_MMVQ_WGS=4096 GGML_MI355X_MMVQ_WGS=8192; do
  echo "== $v" >> $O/head.txt
  timeout -k 10 120 env $v python scripts/mmvq_bench.py q4_0:4096:4096:1:64 q4_K:4096:4096:1:64 q6_K:4096:11008:1:24 2>&1 | grep GB/s >> $O/head.txt || exit 1
done
cat $O/gpt2.txt $O/head.txt
