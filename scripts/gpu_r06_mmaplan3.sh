#!/bin/bash
# scripts/gpu_r06_mmaplan3.sh — the per-instantiation LDS budget (one K part at K = 14336 with
# 5..8 columns): MFMA mat-vec parity, then graph periods against the previous rule
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mmaplan3; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
bash scripts/mv_sweep.sh $O/sweep.txt ' q4_0:14336:4096:3 q4_0:14336:4096:5 q4_0:14336:4096:8 q4_0:12288:4096:3 q4_0:12288:4096:5 q4_0:12288:4096:8 q4_0:14336:8192:3 q4_0:14336:8192:5 q4_0:14336:8192:8 q4_0:28672:4096:3 q4_0:28672:4096:5 q4_0:28672:4096:8 q8_0:14336:4096:3 q8_0:14336:4096:5 q8_0:14336:4096:8 q8_0:12288:4096:3 q8_0:12288:4096:5 q8_0:12288:4096:8 q8_0:14336:8192:3 q8_0:14336:8192:5 q8_0:14336:8192:8 q8_0:28672:4096:3 q8_0:28672:4096:5 q8_0:28672:4096:8 q4_K:14336:4096:3 q4_K:14336:4096:5 q4_K:14336:4096:8 q4_K:12288:4096:3 q4_K:12288:4096:5 q4_K:12288:4096:8 q4_K:14336:8192:3 q4_K:14336:8192:5 q4_K:14336:8192:8 q4_K:28672:4096:3 q4_K:28672:4096:5 q4_K:28672:4096:8 q5_K:14336:4096:3 q5_K:14336:4096:5 q5_K:14336:4096:8 q5_K:12288:4096:3 q5_K:12288:4096:5 q5_K:12288:4096:8 q5_K:14336:8192:3 q5_K:14336:8192:5 q5_K:14336:8192:8 q5_K:28672:4096:3 q5_K:28672:4096:5 q5_K:28672:4096:8 q4_K:49408:4096:3 q4_K:49408:4096:8 q4_0:25600:4096:5' default LIB=$PWD/abl/libold.so MMA=0 || exit 1
