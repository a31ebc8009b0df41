set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_repack.py tests/test_mmq8.py tests/test_gpu_parity.py tests/test_mmq_range.py > gpurun_out/q_tests.log 2>&1
rc=$?; tail -4 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
S="q8_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512 q8_0:4096:4096:2048"
timeout -k 10 200 python scripts/mmq_bench.py $S 2>&1 | grep tile || exit 1
MMQ_REPACKED=1 timeout -k 10 200 python scripts/mmq_bench.py $S 2>&1 | grep tile || exit 1
MMQ_REPACKED=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp1 -o run -- python scripts/mmq_bench.py q8_0:4096:4096:512 > /dev/null 2>&1 || exit 1
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/rp1/run_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'], r['MinNs'])
PY
