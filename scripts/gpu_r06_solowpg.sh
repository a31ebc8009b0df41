#!/bin/bash
# scripts/gpu_r06_solowpg.sh — the single-wave kernel with 1 / 2 / 4 independent waves per
# workgroup (-DSOLO_WPG, abl/libsolo<n>.so): parity, rocprof durations and graph periods
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/solowpg; rm -rf $O; mkdir -p $O
for n in 2 4; do
  GGML_MI355X_LIB=$PWD/abl/libsolo$n.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmvq_solo.py > $O/tests_$n.txt 2>&1 || { tail -20 $O/tests_$n.txt; exit 1; }
  tail -1 $O/tests_$n.txt
done
for L in ggml-gfx906_amd/libggml-hip-mi355x.so abl/libsolo2.so abl/libsolo4.so; do
  echo "## $L"
  timeout -k 10 120 env GGML_MI355X_SOLO=1 GGML_MI355X_LIB=$PWD/$L rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- python scripts/prof_singles.py 128 q4_K:4096:64 > $O/p.log 2>&1 || exit 1
  python scripts/trace_summary.py $(find $O/p -name '*kernel_trace.csv' | head -1) 100 | grep -v rocclr
  rm -rf $O/p
  timeout -k 10 120 env GGML_MI355X_SOLO=1 GGML_MI355X_LIB=$PWD/$L python scripts/mv_graph.py --cold q4_K:4096:4096:1 q4_0:4096:4096:1 q6_K:4096:11008:1 q8_0:4096:4096:1 q4_K:4096:11008:1 || exit 1
done
timeout -k 10 120 python scripts/mv_graph.py --cold q4_K:4096:4096:1 q4_0:4096:4096:1 q6_K:4096:11008:1 q8_0:4096:4096:1 q4_K:4096:11008:1 || exit 1
