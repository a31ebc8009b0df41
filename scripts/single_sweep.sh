#!/bin/bash
# single-matrix mat-vec sweep under rocprofv3 kernel trace: launch width x rows per wave
# usage: scripts/single_sweep.sh   (writes gpurun_out/sweep_<wgs>_<rpw>/ traces)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "2048 1" "256 1" "256 2" "128 2" "512 2" "1024 2"; do
    set -- $cfg
    GGML_MI355X_MMVQ_WGS=$1 GGML_MI355X_RPW=$2 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv \
        -d gpurun_out/sweep_$1_$2 -o run -- python scripts/prof_singles.py 64 > gpurun_out/sweep_$1_$2.log 2>&1 || exit $?
done
