"""Average each PMC counter per kernel over the rocprofv3 --pmc output dirs given (counter
collection CSVs). Usage: python scripts/pmc_summary.py [--match a,b] dir [dir ...]
(--match: kernel-name substrings to keep; default mmq,mmvq)"""
import csv
import glob
import sys
from collections import defaultdict

args = sys.argv[1:]
match = ["mmq", "mmvq"]
if args and args[0] == "--match":
    match = args[1].split(",")
    args = args[2:]
acc = defaultdict(lambda: defaultdict(list))
for d in args:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if not any(m in k for m in match):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.1f}   (n={len(v)})")
