#!/bin/bash
# build (here) / time (GPU box) the MMQ8_EXP measurement variants of the int8 mat-mat kernel:
#   scripts/mmq8_exp.sh build 1 2 6 8 ...   -> scratch_libs/libexp<N>.so
#   scripts/mmq8_exp.sh run   1 2 6 8 ...   -> timings per variant (results are wrong by design)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
S=${SHAPES:-"q8_0:4096:4096:512 q4_K:4096:4096:512"}
if [ "$mode" = build ]; then
  mkdir -p scratch_libs/obj
  for e in "$@"; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -DMMQ8_EXP=$e \
      -Xclang -target-feature -Xclang -packed-fp32-ops -c ggml-gfx906_amd/csrc/mmq8.hip -o scratch_libs/obj/mmq8_$e.o 2>&1 | grep -v "recognized feature"
    objs=$(ls ggml-gfx906_amd/build/*.o | grep -v mmq8.o)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o scratch_libs/libexp$e.so $objs scratch_libs/obj/mmq8_$e.o -ldl
  done
else
  for e in "$@"; do
    echo "== exp $e"
    if [ "$e" = 0 ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/libexp$e.so; fi
    timeout -k 10 120 env GGML_MI355X_LIB=$PWD/$L python scripts/mmq_bench.py $S 2>&1 | grep tile || exit 1
  done
fi
