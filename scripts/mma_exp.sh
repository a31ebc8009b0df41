#!/bin/bash
# build (here) / time (GPU box) measurement variants of the int8-MFMA mat-vec:
#   scripts/mma_exp.sh build tag=FLAGS ...   -> scratch_libs/libmma_<tag>.so  (e.g. x3="-DMMA_EXP=3")
#   scripts/mma_exp.sh run   tag ...         -> timings per variant ("base" = the in-tree library)
# MMA_EXP bit 1 = no activation loads, bit 2 = no weight loads (results wrong by design);
# MMA_D = steps in flight per wave + 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
S=${SHAPES:-"q4_0:14336:4096:4:1 q4_0:14336:4096:8:1 q4_K:14336:4096:8:1 q4_0:4096:4096:8:1 q4_K:4096:11008:8:1"}
if [ "$mode" = build ]; then
  mkdir -p scratch_libs/obj
  for v in "$@"; do
    tag=${v%%=*}; flags=${v#*=}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude $flags \
      -c ggml-gfx906_amd/csrc/mmvq_mma.hip -o scratch_libs/obj/mma_$tag.o || exit 1
    objs=$(ls ggml-gfx906_amd/build/*.o | grep -v mmvq_mma.o)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o scratch_libs/libmma_$tag.so $objs scratch_libs/obj/mma_$tag.o -ldl || exit 1
  done
else
  for tag in "$@"; do
    echo "== $tag"
    if [ "$tag" = base ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/libmma_$tag.so; fi
    timeout -k 10 120 env GGML_MI355X_MMA=1 GGML_MI355X_LIB=$PWD/$L python scripts/mmvq_bench.py $S 2>&1 | grep " us " || exit 1
  done
fi
