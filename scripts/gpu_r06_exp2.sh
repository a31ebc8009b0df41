set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2; mkdir -p $O
timeout -k 10 120 scripts/pkfma_mfma_repro > $O/repro.txt 2>&1 || { echo "repro rc=$?"; exit 1; }
scripts/mmvq_exp.sh run 0 16 > $O/exp.txt 2>&1 || exit 1
for L in 0 16; do
  d=$O/rpw2_E$L; mkdir -p $d
  timeout -k 10 120 env GGML_MI355X_RPW=2 GGML_MI355X_LIB=$PWD/abl/libE$L.so rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python scripts/prof_singles.py 128 q4_K:4096:64 > $d/log 2>&1 || exit 1
  echo "RPW2 E$L: $(python scripts/trace_summary.py $(find $d -name '*kernel_trace.csv' | head -1) 64 | grep mmvq | head -1)" >> $O/exp.txt
done
for L in 0 16; do
  echo "== stamps E$L" >> $O/exp.txt
  timeout -k 10 120 env GGML_MI355X_LIB=$PWD/abl/libE$L.so python scripts/stamps_probe.py q4_K 4096 4096 1 >> $O/exp.txt 2>&1 || exit 1
  echo "== stamps E$L RPW2" >> $O/exp.txt
  timeout -k 10 120 env GGML_MI355X_RPW=2 GGML_MI355X_LIB=$PWD/abl/libE$L.so python scripts/stamps_probe.py q4_K 4096 4096 1 >> $O/exp.txt 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py tests/test_mmq8_stream_k.py tests/test_repack.py tests/test_mmq_range.py tests/test_dispatch_plan.py > $O/tests.txt 2>&1; echo "tests rc=$?" >> $O/tests.txt
