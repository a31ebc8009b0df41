#!/bin/bash
# scripts/gpu_r06_kmin.sh — the K-quant mins term of the MFMA mat-vec on an f32 MFMA (MMA_KMIN=1,
# default) against per-output fmas (abl/libkmin0.so, MMA_KMIN=0): parity, then graph periods (cold)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/kmin; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py -k "q4_K or q5_K or kquant" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
S="--cold q4_K:14336:4096:3 q4_K:14336:4096:8 q4_K:8192:8192:5 q4_K:4096:4096:8 q5_K:14336:4096:3 q5_K:14336:4096:8 q5_K:28672:4096:3 q5_K:11008:4096:5"
bash scripts/mv_sweep.sh $O/sweep.txt "$S" default LIB=$PWD/abl/libkmin0.so default LIB=$PWD/abl/libkmin0.so || exit 1
echo "=== done"
