#!/bin/bash
# scripts/gpu_r06_solox.sh — the single-wave mat-vec's whole-line column load (GGML_MI355X_SOLO_X=1)
# against per-lane slots (=0): parity, stamps, rocprof single launches. Output gpurun_out/solox/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/solox; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmvq_solo.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in 1 0; do
  for t in "q4_K 4096 4096" "q4_0 4096 4096" "q6_K 4096 11008"; do
    GGML_MI355X_SOLO_X=$v timeout -k 10 120 python scripts/solo_stamps.py $t >> $O/stamps_$v.txt 2>&1 || exit 1
  done
done
REPS=2 bash scripts/singles_ab.sh "xl=ggml-gfx906_amd/libggml-hip-mi355x.so:GGML_MI355X_SOLO_X=1" "slot=ggml-gfx906_amd/libggml-hip-mi355x.so:GGML_MI355X_SOLO_X=0" > $O/singles_ab.txt 2>&1
rc=$?; cat $O/singles_ab.txt; exit $rc
