cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/eager -o run -- python scripts/gpt2_bench.py 1 64 0 > gpurun_out/eager.log 2>&1
