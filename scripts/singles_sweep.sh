#!/bin/bash
# single-launch mat-vec (Q4_K 4096x4096 and Q4_0 4096x4096, M = 1, cold) under rocprofv3 for
# mat-vec geometry variants (env), kernel-trace medians per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/singles
i=0
for v in "" "GGML_MI355X_RPW=2" "GGML_MI355X_RPW=4" "GGML_MI355X_LPR=16" "GGML_MI355X_LPR=16 GGML_MI355X_RPW=2" ${EXTRA:-}; do
  i=$((i+1))
  for only in q4_K:4096:64 q4_0:4096:64; do
    env $v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/singles/v$i -o $only -- python scripts/prof_singles.py 200 $only > /dev/null 2>&1 || exit 1
    python - "$v" "$only" gpurun_out/singles/v$i/${only}_kernel_trace.csv <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[3])) if "mmvq" in r["Kernel_Name"]]
d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)[5:]
print(f"{sys.argv[1] or 'default':40s} {sys.argv[2]:14s} n={len(d)} median {statistics.median(d)/1e3:.3f} us  p10 {d[len(d)//10]/1e3:.3f}")
PY
  done
done
