"""Probe the compiler's gfx950 MFMA hazard model: tiny MIR functions (an MFMA and one VALU
instruction on chosen physical registers) run through `llc -mcpu=gfx950 -run-pass=post-RA-hazard-rec`;
the S_NOP the pass inserts is the number of wait states it requires (s_nop N = N + 1 states).
Covers RAW / WAW / WAR-on-srcC and VALU -> MFMA operand for v_mfma_i32_32x32x32_i8 and
v_mfma_i32_16x16x32_i8, packed (v_pk_fma_f32, v_pk_add_f32) against scalar (v_fma_f32).
Usage: python scripts/mfma_hazard_probe.py   (CPU only; writes its .mir files to the cwd)"""
import subprocess, sys
HDR = """---
name: k
tracksRegLiveness: false
machineFunctionInfo:
  isEntryFunction: true
  scratchRSrcReg: '$sgpr0_sgpr1_sgpr2_sgpr3'
  stackPtrOffsetReg: '$sgpr32'
body: |
  bb.0:
"""
V16 = lambda b: "_".join(f"$vgpr{i}" for i in range(b, b+16)).replace("_$", "_")
def v(b, n): return "_".join(f"vgpr{i}" for i in range(b, b+n)).join(["$",""])
MFMA = "    {dst} = V_MFMA_I32_32X32X32_I8_vgprcd_e64 {a}, {b}, {c}, 0, 0, 0, implicit $mode, implicit $exec\n"
PK = "    {dst} = nofpexcept V_PK_FMA_F32 8, {s0}, 8, {s1}, 8, {s2}, 0, 0, 0, 0, 0, implicit $mode, implicit $exec\n"
SC = "    {dst} = nofpexcept V_FMA_F32_e64 0, {s0}, 0, {s1}, 0, {s2}, 0, 0, implicit $mode, implicit $exec\n"
MOV = "    {dst} = V_MOV_B32_e32 {s0}, implicit $exec\n"
PKMOV = "    {dst} = V_PK_MOV_B32 8, {s0}, 8, {s1}, 0, 0, 0, 0, 0, implicit $exec\n"
PKADD = "    {dst} = nofpexcept V_PK_ADD_F32 8, {s0}, 8, {s1}, 0, 0, 0, 0, 0, implicit $mode, implicit $exec\n"
def run(name, body):
    mir = HDR + body + "    S_ENDPGM 0\n...\n"
    open(name + ".mir", "w").write(mir)
    r = subprocess.run(["/opt/rocm/lib/llvm/bin/llc", "-mtriple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-run-pass=post-RA-hazard-rec",
                        name + ".mir", "-o", "-"], capture_output=True, text=True)
    if r.returncode:
        print(name, "ERR", r.stderr[:800]); return
    out = r.stdout[r.stdout.find("body:"):]
    nops = [l.strip() for l in out.splitlines() if "S_NOP" in l]
    print(f"{name:40s}", nops)
m = MFMA.format(dst=v(32,16), a=v(0,4), b=v(4,4), c=v(48,16))
cases = {
 "RAW mfma->pk_fma read": m + PK.format(dst=v(100,2), s0=v(32,2), s1=v(90,2), s2=v(92,2)),
 "RAW mfma->fma read": m + SC.format(dst="$vgpr100", s0="$vgpr32", s1="$vgpr90", s2="$vgpr92"),
 "RAW mfma->pk_fma read hi": m + PK.format(dst=v(100,2), s0=v(46,2), s1=v(90,2), s2=v(92,2)),
 "WAW mfma->pk_fma write": m + PK.format(dst=v(32,2), s0=v(80,2), s1=v(90,2), s2=v(92,2)),
 "WAW mfma->fma write": m + SC.format(dst="$vgpr32", s0="$vgpr80", s1="$vgpr90", s2="$vgpr92"),
 "WAR srcC->pk_fma write": m + PK.format(dst=v(48,2), s0=v(80,2), s1=v(90,2), s2=v(92,2)),
 "WAR srcC->fma write": m + SC.format(dst="$vgpr48", s0="$vgpr80", s1="$vgpr90", s2="$vgpr92"),
 "WAR srcC->mov write": m + MOV.format(dst="$vgpr48", s0="$vgpr80"),
 "WAR srcA->pk_fma write": m + PK.format(dst=v(0,2), s0=v(80,2), s1=v(90,2), s2=v(92,2)),
 "VALU pk write->mfma srcA": PK.format(dst=v(0,2), s0=v(80,2), s1=v(90,2), s2=v(92,2)) + m,
 "VALU fma write->mfma srcA": SC.format(dst="$vgpr0", s0="$vgpr80", s1="$vgpr90", s2="$vgpr92") + m,
 "VALU pk write->mfma srcC": PK.format(dst=v(48,2), s0=v(80,2), s1=v(90,2), s2=v(92,2)) + m,
 "VALU fma write->mfma srcC": SC.format(dst="$vgpr48", s0="$vgpr80", s1="$vgpr90", s2="$vgpr92") + m,
 "pk_add RAW": m + PKADD.format(dst=v(100,2), s0=v(32,2), s1=v(90,2)),
 "mfma;mfma(dep C)": m + MFMA.format(dst=v(120,16), a=v(0,4), b=v(4,4), c=v(32,16)),
}
for k, b in cases.items():
    run(k.replace(" ", "_").replace(">", "").replace(";", "_").replace("(", "").replace(")", ""), b)
print("--- v_mfma_i32_16x16x32_i8")
M16 = "    {dst} = V_MFMA_I32_16X16X32I8_vgprcd_e64 {a}, {b}, {c}, 0, 0, 0, implicit $mode, implicit $exec\n"
m = M16.format(dst=v(32,4), a=v(0,2), b=v(4,2), c=v(48,4))
for k, b in {"RAW16 pk": m + PK.format(dst=v(100,2), s0=v(32,2), s1=v(90,2), s2=v(92,2)),
             "RAW16 cvt": m + "    $vgpr100 = nofpexcept V_CVT_F32_I32_e32 $vgpr32, implicit $mode, implicit $exec\n",
             "WAW16 pk": m + PK.format(dst=v(32,2), s0=v(80,2), s1=v(90,2), s2=v(92,2)),
             "WAR16 srcC pk": m + PK.format(dst=v(48,2), s0=v(80,2), s1=v(90,2), s2=v(92,2))}.items():
    run(k.replace(" ", "_"), b)
