set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_repack.py > gpurun_out/rp_tests.log 2>&1
rc=$?; tail -15 gpurun_out/rp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmq8.py > gpurun_out/rp_mmq8.log 2>&1
rc=$?; tail -15 gpurun_out/rp_mmq8.log; [ $rc -eq 0 ] || exit $rc
S="q8_0:4096:4096:512 q4_0:4096:4096:512 q4_K:4096:4096:512 q5_K:4096:4096:512 q6_K:4096:11008:512 q8_0:4096:4096:2048"
timeout -k 10 200 python scripts/mmq_bench.py $S 2>&1 | grep tile
MMQ_REPACKED=1 timeout -k 10 200 python scripts/mmq_bench.py $S 2>&1 | grep tile
GGML_MI355X_MMQ_REPACK_MIN=9 timeout -k 10 200 python scripts/mmq_bench.py $S 2>&1 | grep tile
MMQ_REPACKED=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp1 -o run -- python scripts/mmq_bench.py q8_0:4096:4096:512 > /dev/null 2>&1 || exit 1
cut -d, -f1-4 gpurun_out/rp1/run_kernel_stats.csv | head -8
timeout -k 10 300 ./oracle/_ref/repack_check ggml-gfx906_amd/libggml-hip-mi355x.so > gpurun_out/repack_check.log 2>&1; rc=$?; tail -20 gpurun_out/repack_check.log; exit $rc
