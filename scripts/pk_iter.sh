#!/bin/bash
# int8 mat-mat iteration: its parity tests (in-place and repacked tiles), then timing of the
# in-tree library against scratch_libs variants: scripts/pk_iter.sh [NAME...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmq8.py tests/test_repack.py > gpurun_out/pk_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pk_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for n in head "$@"; do
    if [ "$n" = head ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/lib$n.so; fi
    echo "--- $n"
    GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 python scripts/mmq_bench.py q8_0:4096:4096:512 q4_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512 || exit 1
    MMQ_REPACKED=1 GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512 || exit 1
  done
done
