#!/bin/bash
# Reproduce round 2's profiler crash: a --pmc pass over bench.py WITH its GPT-2 leg
# (round 2 ran the counter passes with --no-gpt2 because this segfaulted).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_bench_gpt2; rm -rf $O; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/kt -o run -- python bench.py --no-extra --cpu-seconds 1 --steps 5 --warmup 1 --gpt2-ticks 16 > $O/kt.log 2>&1
echo "pmc + kernel-trace, bench with GPT-2 leg: exit $?"
grep -iE "segmentation|signal|error" $O/kt.log | head -5
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o run -- python bench.py --no-extra --cpu-seconds 1 --steps 5 --warmup 1 --gpt2-ticks 16 > $O/pmc.log 2>&1
echo "pmc only, bench with GPT-2 leg: exit $?"
grep -iE "segmentation|signal|error" $O/pmc.log | head -5
find $O -name '*.csv' -size +2M -delete
