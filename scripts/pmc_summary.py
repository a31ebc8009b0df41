"""Average each PMC counter per kernel over the rocprofv3 --pmc output dirs given (counter
collection CSVs). Usage: python scripts/pmc_summary.py dir [dir ...]"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "mmq" not in k and "mmvq" not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.1f}   (n={len(v)})")
