# round-6 session step: packed-f32 reproducer, the quantizer A/B (libHEAD = one unit per wave,
# libQX = eight), the mat-mat GPU tests and the new golden records
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3; mkdir -p $O
timeout -k 10 120 scripts/pkfma_mfma_repro > $O/repro.txt 2>&1 || { echo "repro rc=$?"; exit 1; }
for rep in 1 2; do for L in HEAD QX; do
  timeout -k 10 180 env GGML_MI355X_LIB=$PWD/abl/lib$L.so python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512 q4_K:4096:4096:128 q8_0:4096:4096:2048 > $O/mmq_${L}_$rep.txt 2>&1 || exit 1
  sed "s/^/$L rep$rep /" $O/mmq_${L}_$rep.txt >> $O/mmq.txt
done; done
for L in HEAD QX; do
  d=$O/prof_$L; mkdir -p $d
  timeout -k 10 180 env GGML_MI355X_LIB=$PWD/abl/lib$L.so rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 > $d/log 2>&1 || exit 1
  python scripts/trace_summary.py $(find $d -name '*kernel_trace.csv' | head -1) 8 > $d/summary.txt
  rm -f $(find $d -name '*kernel_trace.csv')
done
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmq8.py tests/test_mmq8_stream_k.py tests/test_gpu_parity.py -k "mmq8 or mm_17 or mm_18 or mmid" > $O/tests.txt 2>&1; echo "tests rc=$?" >> $O/tests.txt
S="q4_0:4096:4096:3:16 q4_0:4096:4096:8:16 q8_0:4096:4096:5:16 q4_K:4096:4096:3:16 q4_K:4096:4096:5:16 q4_K:4096:4096:8:16 q5_K:4096:4096:8:16"
for rep in 1 2; do
  timeout -k 10 180 env GGML_MI355X_MMA=0 python scripts/mmvq_bench.py $S >> $O/fuse.txt 2>&1 || exit 1
  timeout -k 10 180 env GGML_MI355X_MMA=2 GGML_MI355X_MMA_FUSE=0 python scripts/mmvq_bench.py $S >> $O/fuse.txt 2>&1 || exit 1
  timeout -k 10 180 env GGML_MI355X_MMA=2 GGML_MI355X_MMA_FUSE=1 python scripts/mmvq_bench.py $S >> $O/fuse.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py > $O/tests_mma.txt 2>&1; echo "tests rc=$?" >> $O/tests_mma.txt
