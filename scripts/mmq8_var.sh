#!/bin/bash
# build (here) / time (GPU box) compile-time variants of the int8 mat-mat kernel:
#   scripts/mmq8_var.sh build NAME "-DMMQ8_STAG=1 ..."   -> scratch_libs/libvar_NAME.so
#   scripts/mmq8_var.sh run NAME1 NAME2 ...              -> timings, two interleaved rounds
#                                                           (NAME "head" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
S=${SHAPES:-"q8_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512 q8_0:4096:4096:2048"}
if [ "$mode" = build ]; then
  name=$1; defs=$2
  mkdir -p scratch_libs/obj
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude $defs \
    -Xclang -target-feature -Xclang -packed-fp32-ops -c ggml-gfx906_amd/csrc/mmq8.hip -o scratch_libs/obj/mmq8_$name.o 2>&1 | grep -v "recognized feature"
  objs=$(ls ggml-gfx906_amd/build/*.o | grep -v mmq8.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o scratch_libs/libvar_$name.so $objs scratch_libs/obj/mmq8_$name.o -ldl
else
  for rep in 1 2; do
    for name in "$@"; do
      echo "== $name"
      if [ "$name" = head ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/libvar_$name.so; fi
      timeout -k 10 120 env GGML_MI355X_LIB=$PWD/$L python scripts/mmq_bench.py $S 2>&1 | grep tile || exit 1
    done
  done
fi
