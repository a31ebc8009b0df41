#!/bin/bash
# PMC counters of the GPT-2 engine's decode kernels (graph replay, scripts/gpt2_bench.py).
# Every pass runs with --kernel-trace: a --pmc-only pass of bench.py's GPT-2 leg segfaults inside
# the profiler's launch intercept (profiles/README.md); with kernel tracing on it completes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_gpt2; rm -rf $O; mkdir -p $O
i=0
for cs in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY" \
          "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $cs --kernel-trace --output-format csv -d $O/p$i -o run -- python scripts/gpt2_bench.py 1 16 1 > $O/p$i.log 2>&1
  echo "pass $i ($cs): exit $?"
  find $O/p$i -name '*kernel_trace.csv' -delete
done
python scripts/pmc_summary.py --match block_kernel,resid,mmvq,argmax $O/p*
