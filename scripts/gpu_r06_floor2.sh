#!/bin/bash
# scripts/gpu_r06_floor2.sh — one box, one basis: rocprof durations of a bare stream of one Q4_K
# 4096^2 matrix's bytes, the 8-wave mat-vec (the default since the graph-period rules) and the
# single-wave kernel (GGML_MI355X_SOLO=1), then both kernels' hipGraph periods (64 copies)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/floor2; rm -rf $O; mkdir -p $O
[ -x scripts/hbm_probe ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o scripts/hbm_probe scripts/hbm_probe.hip || exit 1
RP="rocprofv3 --kernel-trace --output-format csv"
timeout -k 10 120 $RP -d $O/stream -o run -- scripts/hbm_probe s > $O/stream.log 2>&1 || exit 1
timeout -k 10 120 $RP -d $O/mv8 -o run -- python scripts/prof_singles.py 128 q4_K:4096:64 > $O/mv8.log 2>&1 || exit 1
timeout -k 10 120 env GGML_MI355X_SOLO=1 $RP -d $O/solo -o run -- python scripts/prof_singles.py 128 q4_K:4096:64 > $O/solo.log 2>&1 || exit 1
for d in stream mv8 solo; do echo "## $d"; python scripts/trace_summary.py $(find $O/$d -name '*kernel_trace.csv' | head -1) 100 | grep -v rocclr; done
for v in "" GGML_MI355X_SOLO=1; do timeout -k 10 120 env $v python scripts/mv_graph.py --cold q4_K:4096:4096:1 q4_0:4096:4096:1 || exit 1; done
find $O -name '*.csv' -delete
