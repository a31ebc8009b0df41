#!/bin/bash
# scripts/pmc_mmq.sh — SQ/TA counter passes (one rocprofv3 --pmc run each) over the mat-mat
# tile selected by GGML_MI355X_MMQ_TILE, for the shapes given (default Q8_0 4096x4096x512).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
SH=${*:-q8_0:4096:4096:512}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA"
P3="TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
i=0
for C in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_mmq$i -o run -- python scripts/mmq_bench.py $SH > gpurun_out/pmc_mmq$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_mmq$i.log; }
done
python scripts/pmc_summary.py gpurun_out/pmc_mmq1 gpurun_out/pmc_mmq2 gpurun_out/pmc_mmq3
