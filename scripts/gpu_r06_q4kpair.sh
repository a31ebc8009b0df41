#!/bin/bash
# scripts/gpu_r06_q4kpair.sh — Q4_K paired steps in the MFMA mat-vec (row-contiguous qs loads +
# ds_bpermute): parity, then hipGraph periods (cold) paired vs unpaired (GGML_MI355X_MMA_PAIR)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/q4kpair; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmvq_mma.py -k "kquant_paired or q4_K or q5_K" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
S="--cold"
for sh in q4_K:14336:4096 q4_K:4096:14336 q4_K:8192:8192 q4_K:11008:4096 q4_K:28672:4096 q4_K:4096:4096 q4_K:12288:4096; do
  for c in 3 5 8; do S="$S $sh:$c"; done
done
bash scripts/mv_sweep.sh $O/sweep.txt "$S" MMA=1,MMA_PAIR=0 MMA=1,MMA_PAIR=1 MMA=1,MMA_PAIR=1,MMA_RT=1 || exit 1
echo "=== done"
