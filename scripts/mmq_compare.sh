cd $GRAFT_REPO_ROOT
S="q8_0:4096:4096:512 q4_K:4096:4096:512 q4_0:4096:4096:512 q5_K:4096:4096:512 q6_K:4096:11008:512 q4_K:4096:4096:128 q8_0:4096:4096:64 q4_K:4096:4096:32 q8_0:4096:4096:2048"
for t in auto wave64 wave32; do GGML_MI355X_MMQ_TILE=$t timeout -k 10 200 python scripts/mmq_bench.py $S || exit $?; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc -o run -- python scripts/mmq_bench.py q8_0:4096:4096:512 > gpurun_out/profc.log 2>&1
