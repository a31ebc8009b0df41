#!/bin/bash
# scripts/gpu_r06_suite.sh — the GPU suite, one bench line and the reference perf harness's MUL_MAT
# table at the tree's HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
[ $rc = 0 ] || exit $rc
timeout -k 10 600 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops perf -o MUL_MAT -b MI355X0 > $O/tboperf.log 2>&1 || { tail -5 $O/tboperf.log; exit 1; }
tail -2 $O/tboperf.log
