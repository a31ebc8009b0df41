cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 0 1; do echo "HIP_FORCE_DEV_KERNARG=$v"; HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python scripts/gpt2_bench.py 1 256 1 || exit 1; HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python scripts/prof_singles.py 64 q4_K:4096:64 || exit 1; done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/karg -o run -- python scripts/gpt2_bench.py 1 256 1 > gpurun_out/karg.log 2>&1
