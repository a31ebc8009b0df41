#!/bin/bash
# scripts/gpu_r06_rowc.sh — measurement build (abl/libq4k_rowc.so, MMA_EXP=4, results wrong by
# design): does the MFMA mat-vec's weight stream get faster when each Q4_K load instruction reads
# 8 rows x 128 contiguous bytes instead of 16 rows x 64 (same rows and bytes per wave pair)?
# With and without the column pre-pass (DIAG=256 skips it). Build the variant here first:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -Xclang -target-feature \
#     -Xclang -packed-fp32-ops -DMMA_EXP=4 -c ggml-gfx906_amd/csrc/mmvq_mma.hip -o abl/obj/mma_rowc.o
#   hipcc --offload-arch=gfx950 -shared -o abl/libq4k_rowc.so <ggml-gfx906_amd/build/*.o but mmvq_mma.o> abl/obj/mma_rowc.o -ldl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rowc; rm -rf $O; mkdir -p $O
S="--cold q4_K:14336:4096:8 q4_K:14336:4096:3 q4_K:4096:14336:8 q4_K:8192:8192:8"
bash scripts/mv_sweep.sh $O/sweep.txt "$S" MMA=1 MMA=1,LIB=$PWD/abl/libq4k_rowc.so MMA=1,DIAG=256 MMA=1,DIAG=256,LIB=$PWD/abl/libq4k_rowc.so || exit 1
echo "=== done"
