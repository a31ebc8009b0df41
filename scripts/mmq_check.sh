cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_mmq_range.py -q -x --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1; tail -3 gpurun_out/par.log
timeout -k 10 200 python scripts/mmq_bench.py q4_K:4096:4096:32 q4_K:4096:4096:128 q8_0:4096:4096:64 q4_0:4096:4096:16 q4_K:4096:11008:64 q8_0:4096:4096:512
