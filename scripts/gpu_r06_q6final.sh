#!/bin/bash
# scripts/gpu_r06_q6final.sh — the Q6_K MFMA mat-vec as dispatched: parity (MFMA mat-vec tests, the
# reference's golden records replayed, test-backend-ops through the plugin), the reference perf
# harness table, and a depth-4 measurement build (abl/libq6_d4.so, MMA_D=4) against depth 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/q6final; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py tests/test_gpu_parity.py tests/test_drop_in.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops perf -o MUL_MAT -b MI355X0 > $O/tboperf.log 2>&1 || { tail -5 $O/tboperf.log; exit 1; }
bash scripts/mv_sweep.sh $O/sweep.txt "--cold q6_K:14336:4096:3 q6_K:14336:4096:8 q6_K:4096:4096:8 q6_K:28672:4096:3 q6_K:8192:8192:3 q4_K:14336:4096:8 q5_K:14336:4096:8" default LIB=$PWD/abl/libq6_d4.so || exit 1
echo "=== done"
