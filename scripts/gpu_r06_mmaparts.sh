#!/bin/bash
# scripts/gpu_r06_mmaparts.sh — where the MFMA mat-vec's graph period goes at HEAD: measurement
# builds (abl/libmma_e2.so = no weight loads, abl/libmma_e3.so = no weight and no column loads;
# results wrong by design) with and without the column pre-pass launch (DIAG=256 skips it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mmaparts; rm -rf $O; mkdir -p $O
S="--cold q4_K:14336:4096:3 q4_K:14336:4096:8 q6_K:14336:4096:8 q5_K:14336:4096:3 q4_0:14336:4096:8"
bash scripts/mv_sweep.sh $O/sweep.txt "$S" default DIAG=256 LIB=$PWD/abl/libmma_e2.so LIB=$PWD/abl/libmma_e2.so,DIAG=256 LIB=$PWD/abl/libmma_e3.so,DIAG=256 || exit 1
echo "=== done"
