#!/bin/bash
# build (here) / time (GPU box) the MMA_EXP measurement variants of the int8-MFMA mat-vec:
#   scripts/mma_exp.sh build 1 2 4 ...   -> scratch_libs/libmma<N>.so
#   scripts/mma_exp.sh run   0 1 2 4 ... -> timings per variant (results are wrong by design)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
S=${SHAPES:-"q4_0:14336:4096:8:1 q4_0:4096:4096:8:1 q4_K:4096:11008:8:1"}
if [ "$mode" = build ]; then
  mkdir -p scratch_libs/obj
  for e in "$@"; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -DMMA_EXP=$e \
      -c ggml-gfx906_amd/csrc/mmvq_mma.hip -o scratch_libs/obj/mma_$e.o
    objs=$(ls ggml-gfx906_amd/build/*.o | grep -v mmvq_mma.o)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o scratch_libs/libmma$e.so $objs scratch_libs/obj/mma_$e.o -ldl
  done
else
  for e in "$@"; do
    echo "== exp $e"
    if [ "$e" = 0 ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/libmma$e.so; fi
    timeout -k 10 120 env GGML_MI355X_MMA=2 GGML_MI355X_LIB=$PWD/$L python scripts/mmvq_bench.py $S 2>&1 | grep " us " || exit 1
  done
fi
