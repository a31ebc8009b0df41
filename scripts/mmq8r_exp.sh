#!/bin/bash
# build (here) / time (GPU box) the MMQ8R_EXP measurement variants of the repacked int8 tile:
#   scripts/mmq8r_exp.sh build 1 2 4 ...   -> scratch_libs/librexp<N>.so
#   scripts/mmq8r_exp.sh run   0 1 2 4 ... -> timings per variant (results are wrong by design)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
S=${SHAPES:-"q8_0:4096:4096:512"}
if [ "$mode" = build ]; then
  mkdir -p scratch_libs/obj
  for e in "$@"; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -DMMQ8R_EXP=$e \
      -Xclang -target-feature -Xclang -packed-fp32-ops -c ggml-gfx906_amd/csrc/mmq8.hip -o scratch_libs/obj/mmq8r_$e.o 2>&1 | grep -v "recognized feature"
    objs=$(ls ggml-gfx906_amd/build/*.o | grep -v mmq8.o)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o scratch_libs/librexp$e.so $objs scratch_libs/obj/mmq8r_$e.o -ldl
  done
else
  for e in "$@"; do
    echo "== exp $e"
    if [ "$e" = 0 ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/librexp$e.so; fi
    MMQ_REPACKED=1 timeout -k 10 120 env GGML_MI355X_LIB=$PWD/$L python scripts/mmq_bench.py $S 2>&1 | grep tile || exit 1
  done
fi
