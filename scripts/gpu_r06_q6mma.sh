#!/bin/bash
# scripts/gpu_r06_q6mma.sh — the Q6_K form of the int8-MFMA mat-vec: parity (tests/test_mmvq_mma.py
# Q6_K cases) and hipGraph periods (Infinity-Cache-cold weights) against the VALU kernels that take
# Q6_K at 2..8 columns today, per K part plan
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/q6mma; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py -k q6_K > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
S="--cold"
for kn in 4096:4096 4096:11008 11008:4096 4096:14336 14336:4096 8192:8192 28672:4096 4096:28672; do
  for c in 2 3 4 5 8; do S="$S q6_K:$kn:$c"; done
done
bash scripts/mv_sweep.sh $O/sweep.txt "$S" default MMA=2 MMA=2,MMA_KH=2 || exit 1
echo "=== done"
