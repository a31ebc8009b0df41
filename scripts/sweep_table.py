"""Per-shape table of graph periods (cold | warm) for every variant in a scripts/mv_sweep.sh output.
usage: python scripts/sweep_table.py sweep.txt [cold|warm] [type-filter]"""
import re
import sys
from collections import defaultdict

rx = re.compile(r"^(.*?)\s+(q\w+:\d+:\d+:\d+)\s+warm\s+([\d.]+) us.*cold\s+([\d.]+) us")
res = defaultdict(dict)
tags = []
for line in open(sys.argv[1]):
    m = rx.match(line.rstrip())
    if not m:
        continue
    tag = m.group(1).replace("GGML_MI355X_", "").replace(" ", ",").strip() or "default"
    if tag not in tags:
        tags.append(tag)
    res[m.group(2)][tag] = (float(m.group(3)), float(m.group(4)))
ix = 0 if (len(sys.argv) > 2 and sys.argv[2] == "warm") else 1
flt = sys.argv[3] if len(sys.argv) > 3 else ""
short = [t.replace("MMA=2,", "").replace("MMA_", "").replace("RING_PRE", "RP") for t in tags]
print(f"{'shape':20s} " + " ".join(f"{s:>9s}" for s in short))
for sh, v in res.items():
    if flt not in sh:
        continue
    vals = [v.get(t, (float('nan'),) * 2)[ix] for t in tags]
    b = min(vals)
    print(f"{sh:20s} " + " ".join(f"{x:8.2f}{'*' if x == b else ' '}" for x in vals))
