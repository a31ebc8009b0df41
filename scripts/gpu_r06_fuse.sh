#!/bin/bash
# scripts/gpu_r06_fuse.sh — the MFMA mat-vec's column pre-pass inside the main launch: parity (MFMA
# mat-vec tests incl. fused vs separate bitwise, golden replay, test-backend-ops through the
# plugin), graph periods fused vs GGML_MI355X_MMA_FUSE=0, and the reference perf harness table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fuse; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mmvq_mma.py -k in_launch > $O/tests_fuse.txt 2>&1 || { tail -30 $O/tests_fuse.txt; exit 1; }
grep -c PASSED $O/tests_fuse.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py tests/test_gpu_parity.py tests/test_drop_in.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
S="--cold"
for sh in q4_0:14336:4096 q8_0:14336:4096 q4_K:14336:4096 q5_K:14336:4096 q6_K:14336:4096 q4_0:4096:4096 q4_K:8192:8192 q6_K:4096:11008 q8_0:4096:14336; do
  for c in 3 5 8; do S="$S $sh:$c"; done
done
bash scripts/mv_sweep.sh $O/sweep.txt "$S" default MMA_FUSE=0 || exit 1
timeout -k 10 600 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops perf -o MUL_MAT -b MI355X0 > $O/tboperf.log 2>&1 || { tail -5 $O/tboperf.log; exit 1; }
echo "=== done"
