#!/bin/bash
# scripts/pmc_l2.sh — L2 (TCC) hit/miss and fabric read requests of the mat-mat kernels, one
# rocprofv3 --pmc pass per counter block. Usage: GGML_MI355X_MMQ_TILE=... pmc_l2.sh shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
SH=${*:-q4_K:4096:4096:512}
i=0
for C in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCP_TCC_READ_REQ_sum TCC_REQ_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_l2_$i -o run -- python scripts/mmq_bench.py $SH > gpurun_out/pmc_l2_$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc_l2_$i.log; }
done
python scripts/pmc_summary.py gpurun_out/pmc_l2_1 gpurun_out/pmc_l2_2 gpurun_out/pmc_l2_3
rm -rf gpurun_out/pmc_l2_*/
