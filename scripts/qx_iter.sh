#!/bin/bash
# activation-quantizer iteration: graph-fusion and int8 mat-mat parity, then mat-mat timing with
# 4 super-blocks per quantizer wave (default) against 1 (GGML_MI355X_QX_SBW=1), interleaved
# (GGML_MI355X_QX_SBW and the 4-per-wave quantizer existed only in an uncommitted measurement build; results in profiles/r04_quant_x_sbw_ab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph_fusion.py tests/test_mmq8.py tests/test_repack.py > gpurun_out/qx_tests.log 2>&1
rc=$?; tail -3 gpurun_out/qx_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 4 1; do
    echo "--- QX_SBW=$v"
    GGML_MI355X_QX_SBW=$v timeout -k 10 120 python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 q8_0:4096:4096:2048 2>&1 | grep tile= || exit 1
    MMQ_REPACKED=1 GGML_MI355X_QX_SBW=$v timeout -k 10 120 python scripts/mmq_bench.py q8_0:4096:4096:512 2>&1 | grep tile= || exit 1
  done
done
