"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel
(demangled name, VGPRs, AGPRs, spills, occupancy). usage: python scripts/kernel_resources.py FILE.hip [filter]"""
import re, subprocess, sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude",
       "-c", src, "-o", "/tmp/kr.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark: +(VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = m.group(2)
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.splitlines()
for r, n in zip(rows, names):
    if flt in n:
        print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('AGPRs','0'):>3} agpr spill {r.get('VGPRs Spill','0'):>4} occ {r.get('Occupancy [waves/SIMD]','?')}  {n}")
