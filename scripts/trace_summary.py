"""Summarize a rocprofv3 kernel_trace.csv into runs of consecutive dispatches of the same kernel
(+grid): count, mean / median / min duration in us. Usage: python scripts/trace_summary.py trace.csv [min_calls]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
minc = int(sys.argv[2]) if len(sys.argv) > 2 else 4
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
runs = []
for r in rows:
    key = (r["Kernel_Name"][:90], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if runs and runs[-1][0] == key:
        runs[-1][1].append(d)
    else:
        runs.append((key, [d]))
for key, ds in runs:
    if len(ds) >= minc:
        print(f"{len(ds):5d} mean {statistics.mean(ds):8.3f} med {statistics.median(ds):8.3f} min {min(ds):8.3f}  "
              f"grid {key[1]}x{key[2]}x{key[3]}/{key[4]}  {key[0]}")
