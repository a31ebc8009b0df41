#!/bin/bash
# scripts/gpu_r06_headab.sh — the bench's headline line with the workgroup target 2048 (round-5
# value) and the per-type default (4096 for Q4_0), interleaved over three rounds on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/headab; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for w in 2048 0; do
    GGML_MI355X_MMVQ_WGS=$w timeout -k 10 300 python bench.py --no-extra --cpu-seconds 1 --steps 200 > $O/b_${w}_$r.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/b_${w}_$r.log').read().strip().splitlines()[-1]); print('wgs=$w round $r', d['value'], d['roofline']['launch_us'], d['roofline']['frac'])" | tee -a $O/summary.txt
  done
done
