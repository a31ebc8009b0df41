#!/bin/bash
# rocprof kernel durations of single-matrix M = 1 launches (64 rotated copies, HBM-cold) for the
# BASELINE mat-vec shapes, interleaved over library builds and env settings:
#   scripts/singles_ab.sh "LABEL=LIB[:ENV=VAL]" ...   (LIB relative to the repo; ENV optional)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPS=${REPS:-2}
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    label=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""; [ "$rest" != "$lib" ] && envs=${rest#*:}
    for cfg in q4_0:4096:64 q4_K:4096:64 q4_K:11008:64 q5_K:11008:64 q6_K:11008:64; do
      O=gpurun_out/sab/$label/$rep/${cfg//:/_}; rm -rf $O; mkdir -p $O
      timeout -k 10 120 env $envs GGML_MI355X_LIB=$PWD/$lib rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python scripts/prof_singles.py 128 $cfg > $O/log 2>&1 || { echo "$label $cfg failed"; tail -3 $O/log; exit 1; }
      f=$(find $O -name '*kernel_trace.csv' | head -1)
      echo "$label rep$rep $cfg: $(python scripts/trace_summary.py $f 64 | grep mmvq | head -1 | cut -c1-60)"
      rm -f $f
    done
  done
done
