set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mmq8.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_mmq8.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t_mmq8.log
case $rc in 124|134|137|139) exit $rc;; esac
S="q8_0:4096:4096:512 q4_0:4096:4096:512 q4_K:4096:4096:512 q5_K:4096:4096:512 q6_K:4096:11008:512 q4_K:4096:4096:128 q8_0:4096:4096:2048 q4_K:4096:4096:32"
timeout -k 10 200 env GGML_MI355X_MMQ=f16 python scripts/mmq_bench.py $S > gpurun_out/mmq_f16.log 2>&1 || exit $?
timeout -k 10 200 env GGML_MI355X_MMQ=i8 python scripts/mmq_bench.py $S > gpurun_out/mmq_i8.log 2>&1 || exit $?
cat gpurun_out/mmq_f16.log gpurun_out/mmq_i8.log | grep tile
