#!/bin/bash
# counter passes (one rocprofv3 --pmc run each) over one mat-vec shape: MMA=<GGML_MI355X_MMA>
# picks the int8-MFMA path (1) or the VALU kernels (0). Usage: pmc_mma.sh <tag> <shape>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-mma}; SH=${2:-q4_0:14336:4096:8:1}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA"
P3="SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P4="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_SPI_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
P5="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"
P6="FETCH_SIZE"
i=0
for C in "$P1" "$P2" "$P3" "$P4" "$P5" "$P6"; do
    i=$((i+1))
    timeout -s KILL 90 env GGML_MI355X_MMA=${MMA:-1} rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmcm_${TAG}_$i -o run -- python scripts/mmvq_bench.py $SH > gpurun_out/pmcm_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcm_${TAG}_$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out/pmcm_${TAG}_[1-6] > gpurun_out/pmcm_${TAG}.txt
cat gpurun_out/pmcm_${TAG}.txt
find gpurun_out/pmcm_${TAG}_* -name '*.csv' -size +1M -delete
