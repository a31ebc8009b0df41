set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/singles2
for v in "GGML_MI355X_RPW=1" "GGML_MI355X_RPW=2"; do
  for only in q4_K:11008:64 q5_K:11008:64 q4_K:4096:64 q4_0:4096:64; do
    env $v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/singles2/$v -o $only -- python scripts/prof_singles.py 200 $only > /dev/null 2>&1 || exit 1
    python - "$v" "$only" gpurun_out/singles2/$v/${only}_kernel_trace.csv <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[3])) if "mmvq" in r["Kernel_Name"]]
d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)[5:]
print(f"{sys.argv[1]:20s} {sys.argv[2]:14s} n={len(d)} median {statistics.median(d)/1e3:.3f} us  p10 {d[len(d)//10]/1e3:.3f}")
PY
  done
done
