"""Scan a gfx950 ISA listing (hipcc --cuda-device-only -S) for the MFMA -> VALU dependences and
check each against the wait states the compiler's gfx950 hazard model requires.

  python scripts/mfma_hazard_scan.py file.s [kernel-substring]

The model (ROCm 7.2 llc, probed with `llc -mcpu=gfx950 -run-pass=post-RA-hazard-rec` on MIR
pairs, scripts/mfma_hazard_probe.py; profiles/r06_mfma_hazards.txt):
  v_mfma_i32_32x32x32_i8 (8 passes)  RAW 12  WAW 12  WAR-srcC 7
  v_mfma_i32_16x16x32_i8 (4 passes)  RAW  8  WAW  8  WAR-srcC 3
  (v_pk_fma_f32 and v_fma_f32 alike; a VALU write -> MFMA source needs 2)
RAW: a VALU reads an MFMA's result; WAW: a VALU writes a register an MFMA in flight writes; WAR:
a VALU writes a register an MFMA in flight reads as its C input. Wait states are counted as the
ISA counts them: one per issued instruction, N+1 per `s_nop N`. The scan runs the listing in
order across labels (fall-through) and, for every backward branch, once more from the branch
target with the state at the branch (loop back-edges). It prints, per category and VALU class
(packed f32 = v_pk_*, the rest scalar), the number of dependences, the minimum distance and
every violation of the model.
"""
import re
import sys
from collections import defaultdict

REQ = {  # mnemonic substring -> (RAW, WAW, WAR on srcC)
    "v_mfma_i32_32x32x32_i8": (12, 12, 7),
    "v_mfma_i32_32x32x16_i8": (12, 12, 7),
    "v_mfma_i32_16x16x32_i8": (8, 8, 3),
    "v_mfma_f32_32x32x16_f16": (12, 12, 7),
    "v_mfma_f32_16x16x32_f16": (8, 8, 3),
}
RANGE = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
HORIZON = 24


def regs(tok: str) -> set:
    out = set()
    for m in RANGE.finditer(tok):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def parse(lines):
    insts, labels = [], {}
    for ln, line in lines:
        s = line.split(";")[0].strip()
        if not s or s.startswith("."):
            if s.startswith(".LBB") and s.endswith(":"):
                labels[s[:-1]] = len(insts)
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(insts)
            continue
        op = s.split()[0]
        parts = [p.strip() for p in s[len(op):].split(",")] if len(s) > len(op) else []
        insts.append((ln, op, parts))
    return insts, labels


def req_of(op):
    for k, v in REQ.items():
        if op.startswith(k):
            return v
    return (12, 12, 7) if op.startswith("v_mfma") else None


def step(state, inst, stats, viol):
    ln, op, parts = inst
    ws = int(parts[0], 0) + 1 if op == "s_nop" else 1
    if op.startswith("v_") and not op.startswith("v_mfma") and parts and parts[0]:
        cls = "packed" if op.startswith("v_pk_") else "scalar"
        dst = regs(parts[0])
        src = set()
        for p in parts[1:]:
            src |= regs(p)
        for (mln, mop, mdst, msrcc, w, rq) in state:
            for cat, hit, need in (("RAW", src & mdst, rq[0]), ("WAW", dst & mdst, rq[1]), ("WAR-srcC", dst & msrcc, rq[2])):
                if hit and w < 64:
                    key = (cat, cls)
                    stats[key][0] += 1
                    stats[key][1] = min(stats[key][1], w)
                    if w < need:
                        viol.append((cat, cls, op, w, need, mln, ln))
    state = [(m, mo, d, c, w + ws, rq) for (m, mo, d, c, w, rq) in state if w + ws < HORIZON]
    if op.startswith("v_mfma"):
        rq = req_of(op)
        state.append((ln, op, regs(parts[0]), regs(parts[3]) if len(parts) > 3 else set(), 0, rq))
    return state


def scan(lines):
    insts, labels = parse(lines)
    stats = defaultdict(lambda: [0, 1 << 30])
    viol = []
    state = []
    for i, inst in enumerate(insts):
        state = step(state, inst, stats, viol)
        op, parts = inst[1], inst[2]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = labels.get(parts[0]) if parts else None
            if tgt is not None and tgt <= i and state:   # back-edge: the loop head after the tail
                st = list(state)
                for j in range(tgt, min(len(insts), tgt + HORIZON)):
                    st = step(st, insts[j], stats, viol)
                    if not st:
                        break
    return stats, viol


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else None
    lines, on = [], pat is None
    for i, l in enumerate(open(path), 1):
        if re.match(r"^_Z\w*:", l):
            on = pat is None or pat in l
        if on:
            lines.append((i, l))
    stats, viol = scan(lines)
    for (cat, cls), (n, mn) in sorted(stats.items()):
        print(f"{cat:9s} {cls:7s} dependences {n:7d}  min wait states {mn}")
    print(f"violations of the model: {len(viol)}")
    for v in viol[:20]:
        print("  %s %s %s at %d < %d (mfma line %d, valu line %d)" % v)


if __name__ == "__main__":
    main()
