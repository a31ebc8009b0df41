#!/bin/bash
# scripts/gpu_r06_mmq8pf.sh — A/B of the int8 tile with LDS fragments fetched one block ahead
# (abl/libpf.so, -DMMQ8_LDSPF=1) against the tree's library; parity of the variant first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mmq8pf; mkdir -p $O
GGML_MI355X_LIB=$PWD/abl/libpf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmq8.py -k "q8_0 or q4_0 or Q8_0 or Q4_0" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
S="q8_0:4096:4096:512 q4_0:4096:4096:512 q8_0:4096:11008:512 q8_0:4096:4096:2048"
for r in 1 2; do
  for L in ggml-gfx906_amd/libggml-hip-mi355x.so abl/libpf.so; do
    echo "== $L rep $r"
    GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 python scripts/mmq_bench.py $S 2>&1 | grep tile || exit 1
  done
done
