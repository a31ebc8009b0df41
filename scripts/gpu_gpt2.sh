#!/bin/bash
# GPT-2 engine GPU checks (run via gpurun): parity tests, then a short decode timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpt2.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpt2_tests.log 2>&1
rc=$?
echo "gpt2 tests rc=$rc"; tail -n 30 gpurun_out/gpt2_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
exit 0
