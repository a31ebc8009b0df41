# round-6 session step: headline / batched mat-vec with and without the issue-order barrier
# (abl/libE16.so = without), three interleaved rounds; then the full GPU suite
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4; mkdir -p $O
S="q4_0:4096:4096:1:64 q4_K:4096:4096:1:64 q4_K:4096:11008:1:24 q5_K:4096:11008:1:24 q6_K:4096:11008:1:24 q8_0:4096:4096:1:64 q4_0:4096:4096:2:32 q4_0:4096:4096:4:16"
for rep in 1 2 3; do for L in HEAD E16; do
  timeout -k 10 180 env GGML_MI355X_LIB=$PWD/abl/lib$L.so python scripts/mmvq_bench.py $S 2>&1 | grep -v amdgpu.ids | sed "s/^/$L rep$rep /" >> $O/batched.txt || exit 1
done; done
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; echo "tests rc=$?" >> $O/gpu_tests.txt
