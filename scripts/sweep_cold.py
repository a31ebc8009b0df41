"""scripts/sweep_cold.py FILE — one row per shape, one column per variant, of scripts/mv_graph.py
lines (µs; 'cold' or the first regime on the line)"""
import collections
import re
import sys

d = collections.defaultdict(dict)
vs = []
for line in open(sys.argv[1]):
    m = re.match(r"(\S+(?: \S+=\S+)*)\s+(q\S+)\s+\w+\s+([\d.]+) us", line)
    if not m:
        continue
    v = m.group(1).replace("GGML_MI355X_", "")
    d[m.group(2)][v] = float(m.group(3))
    if v not in vs:
        vs.append(v)
print(f"{'shape':22s}" + "".join(f"{v:>24s}" for v in vs))
for s in d:
    print(f"{s:22s}" + "".join(f"{d[s].get(v, float('nan')):24.2f}" for v in vs))
