#!/bin/bash
# packed-f32 fault hunt: wrong-position census (tests/diag/mmq8_positions.py) and mat-mat timing
# per library: scripts/mmq8_positions.sh NAME...  ("head" = in-tree, else scratch_libs/lib<NAME>.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for n in "$@"; do
  if [ "$n" = head ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/lib$n.so; fi
  echo "=== $n"
  GGML_MI355X_LIB=$PWD/$L timeout -k 10 200 python tests/diag/mmq8_positions.py q4_0 512 200 4096 60 2>&1 | grep -v amdgpu.ids | tail -6 || exit 1
  GGML_MI355X_LIB=$PWD/$L timeout -k 10 200 python tests/diag/mmq8_positions.py q8_0 4096 512 4096 16 2>&1 | grep -v amdgpu.ids | tail -6 || exit 1
  GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 python scripts/mmq_bench.py q8_0:4096:4096:512 q4_0:4096:4096:512 q4_K:4096:4096:512 2>&1 | grep tile= || exit 1
  MMQ_REPACKED=1 GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 python scripts/mmq_bench.py q8_0:4096:4096:512 2>&1 | grep tile= || exit 1
done
