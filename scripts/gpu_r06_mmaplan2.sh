#!/bin/bash
# scripts/gpu_r06_mmaplan2.sh — the round-6 MFMA mat-vec plan at its final form: parity (MFMA
# mat-vec tests, golden replay, the reference's test-backend-ops MUL_MAT / MUL_MAT_ID through the
# plugin) and the reference perf harness table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mmaplan2; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmvq_mma.py tests/test_gpu_parity.py tests/test_drop_in.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops perf -o MUL_MAT -b MI355X0 > $O/tboperf.log 2>&1 || { tail -5 $O/tboperf.log; exit 1; }
tail -2 $O/tboperf.log
