#!/bin/bash
# rocprof kernel durations of single-matrix mat-vec launches (cold, 64 rotated copies) for
# variant library builds: scripts/ab_singles.sh lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so); O=gpurun_out/abs_$n; rm -rf $O; mkdir -p $O
  for cfg in q4_0:4096:64 q4_K:4096:64 q4_K:11008:64; do
    timeout -k 10 120 env GGML_MI355X_LIB=$PWD/$L rocprofv3 --kernel-trace --output-format csv -d $O/${cfg//:/_} -o run -- python scripts/prof_singles.py 128 $cfg > $O/${cfg//:/_}.log 2>&1 || exit 1
    f=$(find $O/${cfg//:/_} -name '*kernel_trace.csv' | head -1)
    echo "$n $cfg: $(python scripts/trace_summary.py $f 64 | grep mmvq | head -1)"
    rm -f $f
  done
done
