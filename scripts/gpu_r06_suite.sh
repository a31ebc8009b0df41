#!/bin/bash
# scripts/gpu_r06_suite.sh — the GPU suite and one bench line at the tree's HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
exit $rc
