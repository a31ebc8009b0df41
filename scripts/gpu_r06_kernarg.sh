#!/bin/bash
# scripts/gpu_r06_kernarg.sh — does the kernel-argument segment's placement show in the launch
# prologues? The same probes with HIP_FORCE_DEV_KERNARG=0 and =1 (kernargs in host-coherent vs
# device memory): GPT-2 block stamps, GPT-2 decode, the single-wave mat-vec's stamps, single and
# stacked mat-vec launches. Output: gpurun_out/kernarg_<v>.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1; do
    o=gpurun_out/kernarg_$v.txt
    echo "# HIP_FORCE_DEV_KERNARG=$v" > $o
    export HIP_FORCE_DEV_KERNARG=$v
    timeout -k 10 120 python scripts/block_stamps.py 24 64 >> $o 2>&1 || exit $?
    timeout -k 10 120 python scripts/gpt2_bench.py 1 256 1 >> $o 2>&1 || exit $?
    timeout -k 10 120 python scripts/solo_stamps.py q4_K 4096 4096 >> $o 2>&1 || exit $?
    timeout -k 10 120 python scripts/mmvq_bench.py q4_K:4096:4096:1:1 q4_0:4096:4096:1:1 q4_0:4096:4096:1:64 q4_0:14336:4096:8:1 >> $o 2>&1 || exit $?
    echo "=== kernarg $v done"
done
