#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each) over the int8 mat-mat path; DIAG=<bits>
# selects a diagnostic variant (GGML_MI355X_DIAG, see mmq8_kernel). Usage: pmc_mmq8.sh <tag> <shape>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-base}; SH=${2:-q8_0:4096:4096:512}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA"
P3="SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P4="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_SPI_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
P5="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"
i=0
for C in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    i=$((i+1))
    timeout -s KILL 90 env GGML_MI355X_MMQ=i8 GGML_MI355X_DIAG=${DIAG:-0} rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc8_${TAG}_$i -o run -- python scripts/mmq_bench.py $SH > gpurun_out/pmc8_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc8_${TAG}_$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out/pmc8_${TAG}_[1-5] > gpurun_out/pmc8_${TAG}.txt
cat gpurun_out/pmc8_${TAG}.txt
find gpurun_out/pmc8_${TAG}_* -name '*.csv' -size +1M -delete
