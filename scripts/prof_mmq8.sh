#!/bin/bash
# rocprof kernel statistics of the int8 mat-mat path (GGML_MI355X_MMQ=i8) on the given shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof_mmq8
rm -rf $O; mkdir -p $O
timeout -k 10 200 env GGML_MI355X_MMQ=i8 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python scripts/mmq_bench.py "$@" > $O/log.txt 2>&1 || exit $?
grep tile $O/log.txt
f=$(find $O -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1000:8.2f} us  min {float(r['MinNs'])/1000:8.2f}")
PY
