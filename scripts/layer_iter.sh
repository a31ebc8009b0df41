#!/bin/bash
# drop-in GPT-2 layer fusion iteration: fusion decisions, the drop-in parity tests, then ms/token
# with the layer fusion on and off (scripts/plugin_gpt2_ab.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/plugin_gpt2_debug.sh "layer" 6 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph_fusion.py "tests/test_gpt2.py::test_reference_scheduler_drives_plugin" tests/test_gpt2_pipeline.py > gpurun_out/layer_tests.log 2>&1
rc=$?; tail -4 gpurun_out/layer_tests.log; [ $rc -eq 0 ] || exit $rc
CFGS="GGML_MI355X_LAYER_FUSION=1 GGML_MI355X_LAYER_FUSION=0" scripts/plugin_gpt2_ab.sh
