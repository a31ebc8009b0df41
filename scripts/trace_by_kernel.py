"""Aggregate a rocprofv3 kernel_trace.csv by (kernel, grid, workgroup): calls, mean / median
duration in us, and the mean gap from the previous dispatch's end. Usage:
python scripts/trace_by_kernel.py trace.csv [min_calls]"""
import csv
import statistics
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
minc = int(sys.argv[2]) if len(sys.argv) > 2 else 10
agg = defaultdict(lambda: ([], []))
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    key = (r["Kernel_Name"][:80], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
    agg[key][0].append((e - s) / 1e3)
    if prev_end is not None and 0 <= s - prev_end < 50000:
        agg[key][1].append((s - prev_end) / 1e3)
    prev_end = e
for key, (d, g) in sorted(agg.items(), key=lambda kv: -sum(kv[1][0])):
    if len(d) >= minc:
        print(f"{len(d):6d} mean {statistics.mean(d):7.2f} med {statistics.median(d):7.2f}  gap {statistics.mean(g) if g else 0:6.2f}  "
              f"grid {key[1]}x{key[2]}x{key[3]}/{key[4]}  {key[0]}")
