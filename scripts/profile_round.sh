#!/bin/bash
# scripts/profile_round.sh — the profiler evidence of one round, on a 1-GPU MI355X box (via
# gpurun). Every rocprofv3 run has its own time limit; counters get passes of their own.
# Outputs under gpurun_out/prof_<round>/; copy the summaries into profiles/ afterwards.
#   scripts/profile_round.sh r02
set -u
R=${1:-r02}
# PART=a: bench line, its rocprof profile and the PMC passes; PART=b: everything else (each part
# fits one gpurun call); default both
PART=${PART:-all}
in_a() { [ "$PART" = all ] || [ "$PART" = a ]; }
in_b() { [ "$PART" = all ] || [ "$PART" = b ]; }
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/prof_$R
mkdir -p $O
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    case $rc in 124|134|137|139) echo "crash-class exit $rc: stopping"; exit $rc;; esac
    return 0
}
RP="rocprofv3 --kernel-trace --stats --output-format csv"
# keep the box's output small (gpurun copies back <= 64 MiB): summarize traces, drop raw CSVs
squash() {  # squash <dir>
    local d=$1
    for t in $(find $d -name '*kernel_trace.csv'); do python scripts/trace_summary.py $t 2 > ${t%.csv}_summary.txt; rm -f $t; done
    find $d -name '*counter_collection.csv' -size +2M -delete
}
# the HBM floor probe (built here when the tree does not carry the binary)
[ -x scripts/hbm_probe ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o scripts/hbm_probe scripts/hbm_probe.hip || exit 1
if in_a; then
[ -s $O/bench.log ] || step bench 600 python bench.py
step prof_bench 600 $RP -d $O/bench -o run -- python bench.py --no-extra --cpu-seconds 1
python scripts/rocprof_headline.py $(find $O/bench -name '*kernel_trace.csv' | head -1) $O/headline_rocprof.json $R profiles/${R}_bench_trace_summary.txt > /dev/null
squash $O/bench
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc -- python bench.py --no-extra --no-gpt2 --cpu-seconds 1 --steps 5 --warmup 1
python scripts/traffic_from_pmc.py $(find $O/pmc_fetch -name '*counter_collection.csv' | head -1) $O/traffic.json $R > /dev/null
python scripts/pmc_summary.py $O/pmc_fetch > $O/pmc_fetch_summary.txt
squash $O/pmc_fetch
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc -- python bench.py --no-extra --no-gpt2 --cpu-seconds 1 --steps 5 --warmup 1
python scripts/pmc_summary.py $O/pmc_write > $O/pmc_write_summary.txt
squash $O/pmc_write
fi
if in_b; then
step prof_singles 300 $RP -d $O/singles -o run -- python scripts/prof_singles.py
squash $O/singles
step prof_mmq 300 $RP -d $O/mmq -o run -- python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512 q4_K:4096:4096:32 q8_0:4096:4096:2048
squash $O/mmq
step prof_mmq_rp 300 env MMQ_REPACKED=1 $RP -d $O/mmq_rp -o run -- python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512
squash $O/mmq_rp
step prof_gpt2 300 $RP -d $O/gpt2 -o run -- python scripts/gpt2_bench.py 1 256 1
squash $O/gpt2
step block_stamps 200 bash -c 'python scripts/block_stamps.py 24 64 && python scripts/block_stamps.py 24 600'
step hbm_floor 120 scripts/hbm_probe
# the single-launch floor on one basis: rocprofv3 durations of a bare stream of one Q4_K 4096^2
# matrix's bytes (hbm_probe s) and of the mat-vec on the same bytes
step floor_stream 120 $RP -d $O/floor_stream -o run -- scripts/hbm_probe s
squash $O/floor_stream
step floor_mv 120 $RP -d $O/floor_mv -o run -- python scripts/prof_singles.py 128 q4_K:4096:64
squash $O/floor_mv
fi
du -sh $O
echo "=== done"
