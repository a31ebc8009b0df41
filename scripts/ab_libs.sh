#!/bin/bash
# scripts/ab_libs.sh <lib.so> ... — int8 mat-mat diagnostic + timing for variant library builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S="q8_0:4096:4096:512 q4_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512 q8_0:4096:4096:2048"
for L in "$@"; do
  n=$(basename $L .so)
  echo "=== $n"
  timeout -k 10 120 env GGML_MI355X_LIB=$PWD/$L python scripts/mmq8_debug.py > gpurun_out/dbg_$n.log 2>&1 || exit $?
  grep nmse gpurun_out/dbg_$n.log
  timeout -k 10 120 env GGML_MI355X_LIB=$PWD/$L GGML_MI355X_MMQ=i8 python scripts/mmq_bench.py $S > gpurun_out/bench_$n.log 2>&1 || exit $?
  grep tile gpurun_out/bench_$n.log
done
