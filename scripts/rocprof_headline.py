"""The headline mat-vec kernel's rocprofv3 durations from a kernel trace of `bench.py`, for the bench
line's roofline (profiles/headline_rocprof.json): the dispatches of the kernel that streams the
64 stacked matrices (the mmvq_kernel launch with the largest grid), their mean / median duration
and the fraction of 8 TB/s those give for the launch's algorithmic bytes.
Usage: python scripts/rocprof_headline.py <kernel_trace.csv> <out.json> <round> [summary file named in the json]"""
import csv
import json
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mmvq_kernel" in r["Kernel_Name"]]
by = {}
for r in rows:
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    by.setdefault((r["Kernel_Name"], grid), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
(name, grid), ds = max(by.items(), key=lambda kv: (kv[0][1], len(kv[1])))
alg = 4096 * 4096 * 18 // 32 * 64 + 4 * 4096 * 64 + 4 * 4096 * 64
mean, med = statistics.mean(ds), statistics.median(ds)
out = {"q4_0_4096x4096_m1_b64": {
    "round": int(sys.argv[3][1:]), "kernel": name, "grid_threads": grid, "launches": len(ds),
    "mean_us": round(mean, 3), "median_us": round(med, 3), "min_us": round(min(ds), 3),
    "frac_mean": round(alg / (mean * 1e-6) / 8e12, 4), "frac_median": round(alg / (med * 1e-6) / 8e12, 4),
    "alg_bytes_per_launch": alg,
    "command": "rocprofv3 --kernel-trace --stats --output-format csv -- python bench.py --no-extra --cpu-seconds 1",
    "summary": sys.argv[4] if len(sys.argv) > 4 else None}}
with open(sys.argv[2], "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
