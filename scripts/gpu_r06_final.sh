#!/bin/bash
# scripts/gpu_r06_final.sh — after the K-quant pairs rule: MFMA mat-vec parity + golden replay +
# drop-in, graph periods of the Q4_K / Q5_K rule shapes (default vs MMA_PAIR=0 vs the VALU kernels)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py tests/test_gpu_parity.py tests/test_drop_in.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
S="--cold q5_K:28672:4096:3 q5_K:28672:4096:5 q5_K:28672:4096:8 q5_K:8192:4096:5 q5_K:4096:4096:5 q5_K:4096:11008:5 q5_K:11008:4096:3 q4_K:14336:4096:3 q4_K:12288:4096:4 q4_K:28672:4096:3"
bash scripts/mv_sweep.sh $O/sweep.txt "$S" default MMA_PAIR=0 MMA=0 || exit 1
echo "=== done"
