#!/bin/bash
# scripts/gpu_r06_q6exp.sh — where the Q6_K MFMA mat-vec spends its time: measurement builds
# (abl/libq6_<tag>.so, MMA_EXP bits: al = 4-byte aligned pieces, nosc = no scale loads, both,
# now = no weight loads; results wrong by design) against the in-tree build; Q5_K beside it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/q6exp; rm -rf $O; mkdir -p $O
S="--cold q6_K:4096:4096:4 q6_K:4096:4096:8 q6_K:4096:14336:4 q6_K:4096:14336:8 q6_K:14336:4096:8 q5_K:4096:4096:8 q5_K:4096:14336:8"
bash scripts/mv_sweep.sh $O/sweep.txt "$S" MMA=2 MMA=2,LIB=$PWD/abl/libq6_al.so MMA=2,LIB=$PWD/abl/libq6_nosc.so MMA=2,LIB=$PWD/abl/libq6_both.so MMA=2,LIB=$PWD/abl/libq6_now.so || exit 1
echo "=== done"
