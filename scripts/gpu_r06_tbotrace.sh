#!/bin/bash
# scripts/gpu_r06_tbotrace.sh — kernel timeline of the multi-column mat-vec (scripts/mmvq_bench.py,
# back-to-back launches, 2 rotated copies) at the reference perf shapes (K = 14336, N = 4096):
# pre-pass, gap, main kernel, period. (test-backend-ops perf under rocprofv3 --kernel-trace
# segfaulted inside the HIP runtime's graph launch, round 6; the harness alone runs clean.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/mvtrace; rm -rf $O; mkdir -p $O
S=""
for t in q4_0 q8_0 q4_K q5_K q6_K; do for n in 1 2 4 8; do S="$S $t:14336:4096:$n:1"; done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python scripts/mmvq_bench.py $S > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
grep GB/s $O/log
f=$(find $O -name '*kernel_trace.csv' | head -1)
python scripts/trace_pairs.py $f mma_prequant mmvq_mma_kernel
python scripts/trace_pairs.py $f mmvq_prequant mmvq_ring_pre
python scripts/trace_summary.py $f 30 | grep -v -E "rocclr|elementwise"
rm -f $f
