#!/bin/bash
# int8 mat-mat timing of the in-tree library against scratch_libs variants, interleaved:
#   scripts/mmq_lib_ab.sh NAME...   ("head" = in-tree)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for n in head "$@"; do
    if [ "$n" = head ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/lib$n.so; fi
    echo "--- $n"
    GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 python scripts/mmq_bench.py q8_0:4096:4096:512 q4_0:4096:4096:512 q8_0:4096:4096:2048 2>&1 | grep tile= || exit 1
    MMQ_REPACKED=1 GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 python scripts/mmq_bench.py q8_0:4096:4096:512 2>&1 | grep tile= || exit 1
  done
done
