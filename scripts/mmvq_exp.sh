#!/bin/bash
# measurement builds of the mat-vec kernel with parts removed (mmvq_impl.h MMVQ_EXP bits:
# 1 no activation loads, 2 no quantization, 4 no weight loads, 8 no barrier):
#   scripts/mmvq_exp.sh build 0 1 3 4 ...   -> abl/libE<n>.so  (CPU side)
#   scripts/mmvq_exp.sh run 0 1 3 ...       -> rocprof single-launch durations (GPU box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
if [ "$mode" = build ]; then
  make -s -C ggml-gfx906_amd -j8 >/dev/null || exit 1
  mkdir -p abl/obj
  for n in "$@"; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -DMMVQ_EXP=$n \
      -c ggml-gfx906_amd/csrc/mmvq.hip -o abl/obj/mmvq_E$n.o || exit 1
    objs=$(ls ggml-gfx906_amd/build/*.o | grep -v '/mmvq.o$')
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o abl/libE$n.so $objs abl/obj/mmvq_E$n.o -ldl || exit 1
    echo abl/libE$n.so
  done
  exit 0
fi
export TMPDIR=/tmp
cfg=${CFG:-q4_K:4096:64}
for n in "$@"; do
  O=gpurun_out/exp_E$n; rm -rf $O; mkdir -p $O
  timeout -k 10 120 env GGML_MI355X_LIB=$PWD/abl/libE$n.so rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python scripts/prof_singles.py 128 $cfg > $O/log 2>&1 || { echo "E$n failed"; tail -5 $O/log; exit 1; }
  f=$(find $O -name '*kernel_trace.csv' | head -1)
  echo "E$n $cfg: $(python scripts/trace_summary.py $f 64 | grep mmvq | head -1)"
done
