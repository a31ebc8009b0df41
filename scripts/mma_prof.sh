#!/bin/bash
# per-kernel device times of the MMA mat-vec variants (scripts/mma_exp.sh build ...):
#   scripts/mma_prof.sh OUT tag ...    ("base" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; shift
S=${SHAPES:-"q4_0:14336:4096:4:1 q4_0:14336:4096:8:1 q4_K:14336:4096:8:1"}
for tag in "$@"; do
  if [ "$tag" = base ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/libmma_$tag.so; fi
  for sh in $S; do
    d=$out/$tag/${sh//:/_}; mkdir -p $d
    GGML_MI355X_MMA=1 GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python scripts/mmvq_bench.py $sh > $d.log 2>&1 || exit 1
    python3 - "$d" "$tag" "$sh" <<'PY'
import csv, glob, sys
d, tag, sh = sys.argv[1:]
for f in glob.glob(d + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mma" in r["Name"]:
            print(f"{tag:6s} {sh:24s} {r['Name'].split('(')[0][8:]:40s} avg {float(r['AverageNs'])/1e3:7.2f} us  min {float(r['MinNs'])/1e3:7.2f} us")
PY
    find $d -name '*kernel_trace.csv' -delete
  done
done
