"""Scan a gfx950 ISA listing (hipcc -S) for VALU reads of MFMA results and report the wait states
between each MFMA and the first VALU instruction that reads one of its result registers.

  python scripts/mfma_hazard_scan.py file.s [kernel-substring]

Wait states are counted as the ISA does: one per issued instruction, N+1 per `s_nop N`
(s_waitcnt and other SOPP count one). Only straight-line distance inside one basic block is
measured (a label resets the scan), which is where the compiler's hazard recognizer places nops.
"""
import re
import sys
from collections import Counter

RANGE = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(tok: str) -> set:
    out = set()
    for m in RANGE.finditer(tok):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def scan(lines):
    live = []          # (mfma line, dst regs, wait states since)
    report = []
    for ln, line in lines:
        s = line.strip()
        if not s or s.startswith(";") or s.startswith("."):
            if s.endswith(":") or s.startswith(".LBB"):
                live = []
            continue
        if s.endswith(":"):
            live = []
            continue
        op = s.split()[0]
        args = s[len(op):].split(";")[0]
        parts = [p.strip() for p in args.split(",")]
        ws = 1
        if op == "s_nop":
            ws = int(parts[0], 0) + 1
        if op.startswith("v_") and not op.startswith("v_mfma"):
            srcs = set()
            for p in parts[1:]:
                srcs |= regs(p)
            for (mln, dst, w) in live:
                if srcs & dst:
                    report.append((op, w, mln, ln))
            live = [(m, d - srcs, w) for (m, d, w) in live if d - srcs]   # first read only
        live = [(m, d, w + ws) for (m, d, w) in live]
        if op.startswith("v_mfma"):
            live.append((ln, regs(parts[0]), 0))
    return report


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else None
    lines, on = [], pat is None
    for i, l in enumerate(open(path), 1):
        if pat and re.match(r"^_Z\w*:", l):
            on = pat in l
        if on:
            lines.append((i, l))
    rep = scan(lines)
    by_op = {}
    for op, w, _, _ in rep:
        by_op.setdefault(op, Counter())[w] += 1
    for op, c in sorted(by_op.items()):
        print(f"{op:24s} first-read wait states: min {min(c)}  histogram {dict(sorted(c.items()))}")


if __name__ == "__main__":
    main()
