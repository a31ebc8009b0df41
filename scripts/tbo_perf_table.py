"""Table of the reference's own perf harness on the plugin (test-backend-ops perf -o MUL_MAT -b MI355X0,
tests/test-backend-ops.cpp:1299-1365, cases :6195-6201): per case the harness's us/run, and the GB/s of the
algorithmic bytes (quantized weights + f32 activations + f32 output) the case moves.
usage: python scripts/tbo_perf_table.py gpurun_out/tboperf.log > profiles/r05_tbo_perf_mul_mat.txt"""
import re
import sys

BPW = {"q4_0": 18 / 32, "q8_0": 34 / 32, "q4_K": 144 / 256, "q5_K": 176 / 256, "q6_K": 210 / 256,
       "f16": 2.0, "f32": 4.0, "bf16": 2.0}
ANSI = re.compile(r"\x1b\[[0-9;]*m")
rows = []
for line in open(sys.argv[1], errors="replace"):
    line = ANSI.sub("", line).strip()
    m = re.match(r"MUL_MAT\(type_a=(\w+),type_b=(\w+),m=(\d+),n=(\d+),k=(\d+).*?\):\s+(\d+) runs -\s+([\d.]+) us/run -\s+([\d.]+) (\w+)", line)
    if not m:
        continue
    ta, tb, M, N, K, runs, us = m.group(1), m.group(2), int(m.group(3)), int(m.group(4)), int(m.group(5)), int(m.group(6)), float(m.group(7))
    if ta not in BPW:
        continue
    byts = M * K * BPW[ta] + N * K * 4 + M * N * 4
    rows.append((ta, M, N, K, runs, us, byts / us / 1e3))
print(f"{'type':6s} {'m':>6s} {'n':>4s} {'k':>6s} {'runs':>7s} {'us/run':>9s} {'GB/s':>8s} {'x bs=1 time':>12s}")
base = {}
for ta, M, N, K, runs, us, gbs in rows:
    if N == 1:
        base[(ta, M, K)] = us
for ta, M, N, K, runs, us, gbs in rows:
    rel = us / base[(ta, M, K)] if (ta, M, K) in base else float("nan")
    print(f"{ta:6s} {M:6d} {N:4d} {K:6d} {runs:7d} {us:9.2f} {gbs:8.1f} {rel:12.2f}")
