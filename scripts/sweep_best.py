"""Best knob setting per shape from scripts/mv_sweep.sh output: default vs the best variant, warm
and cold graph periods. usage: python scripts/sweep_best.py sweep.txt [regime] [min_gain]"""
import re
import sys
from collections import defaultdict

rx = re.compile(r"^(.*?)\s+(q\w+:\d+:\d+:\d+)\s+warm\s+([\d.]+) us.*cold\s+([\d.]+) us")
res = defaultdict(dict)
for line in open(sys.argv[1]):
    m = rx.match(line.rstrip())
    if not m:
        continue
    tag = m.group(1).replace("GGML_MI355X_", "").strip()
    res[m.group(2)][tag] = (float(m.group(3)), float(m.group(4)))
reg = sys.argv[2] if len(sys.argv) > 2 else "cold"
gain = float(sys.argv[3]) if len(sys.argv) > 3 else 0.03
ix = 0 if reg == "warm" else 1
for sh, v in res.items():
    d = v.get("default")
    if d is None:
        continue
    best = min(v.items(), key=lambda kv: kv[1][ix])
    flag = "  <==" if best[1][ix] < d[ix] * (1 - gain) else ""
    print(f"{sh:20s} default {d[0]:6.2f}/{d[1]:6.2f}  best[{reg}] {best[0]:28s} {best[1][0]:6.2f}/{best[1][1]:6.2f}{flag}")
