"""Per-call timeline of a two-kernel MUL_MAT (pre-pass + main kernel) from a rocprofv3
kernel_trace.csv: medians of the pre-pass duration, the gap to the main kernel, the main kernel's
duration and the period between calls, per (pre-pass, main) kernel-name pair.
usage: python scripts/trace_pairs.py trace.csv PREPASS_SUBSTR MAIN_SUBSTR"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pre, main = sys.argv[2], sys.argv[3]
groups = {}
last_main_start = {}
for a, b in zip(rows, rows[1:]):
    if pre in a["Kernel_Name"] and main in b["Kernel_Name"]:
        key = (a["Kernel_Name"][:60], b["Kernel_Name"][:90], b["Grid_Size_X"], b["Grid_Size_Y"], b["Grid_Size_Z"])
        s0, e0 = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
        s1, e1 = int(b["Start_Timestamp"]), int(b["End_Timestamp"])
        g = groups.setdefault(key, {"pre": [], "gap": [], "main": [], "period": []})
        g["pre"].append((e0 - s0) / 1e3)
        g["gap"].append((s1 - e0) / 1e3)
        g["main"].append((e1 - s1) / 1e3)
        if key in last_main_start:
            g["period"].append((s1 - last_main_start[key]) / 1e3)
        last_main_start[key] = s1
for key, g in groups.items():
    med = {k: statistics.median(v) if v else float("nan") for k, v in g.items()}
    print(f"{len(g['main']):5d} calls  pre {med['pre']:6.2f}  gap {med['gap']:6.2f}  main {med['main']:6.2f}  period {med['period']:6.2f} us"
          f"  grid {key[2]}x{key[3]}x{key[4]}  {key[1]}")
