#!/bin/bash
# GPT-2 engine: GPU tests, then the decode step under rocprofv3 (kernel stats) and plain timings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpt2.py tests/test_gpt2_example.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/gt.log
for L in ${LPRS:-0}; do
  GGML_MI355X_LPR=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pg$L -o run -- python scripts/gpt2_bench.py 1 256 1 > gpurun_out/pg$L.log 2>&1 || exit 1
  grep ms/step gpurun_out/pg$L.log
  GGML_MI355X_LPR=$L timeout -k 10 120 python scripts/gpt2_bench.py 1 256 1 || exit 1
  GGML_MI355X_LPR=$L timeout -k 10 120 python scripts/gpt2_bench.py 8 128 1 || exit 1
done
