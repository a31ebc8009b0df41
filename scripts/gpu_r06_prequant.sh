#!/bin/bash
# scripts/gpu_r06_prequant.sh — what the MFMA mat-vec's column pre-pass costs: rocprof timeline
# (pre-pass, gap, main) for the tree's library, with one K part (no dst zeroing in the pre-pass),
# and a build whose pre-pass loads no activations (abl/libmma_x1.so, -DMMA_EXP=1, wrong results)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S="q4_0:14336:4096:8:1 q4_K:14336:4096:8:1 q4_0:14336:4096:4:1"
for v in base kh1 x1; do
  O=gpurun_out/preq_$v; rm -rf $O; mkdir -p $O
  L=ggml-gfx906_amd/libggml-hip-mi355x.so; E=""
  [ $v = x1 ] && L=abl/libmma_x1.so
  [ $v = kh1 ] && E="GGML_MI355X_MMA_KH=1"
  timeout -k 10 300 env $E GGML_MI355X_LIB=$PWD/$L rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python scripts/mmvq_bench.py $S > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
  echo "## $v"; grep GB/s $O/log
  f=$(find $O -name '*kernel_trace.csv' | head -1)
  python scripts/trace_pairs.py $f mma_prequant mmvq_mma_kernel
  rm -f $f
done
