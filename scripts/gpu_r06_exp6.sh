# round-6 session step: the MFMA mat-vec with two LDS scale slots for paired steps (libSLOT) vs
# one (libPRE), three interleaved rounds; 8 stacked matrices (HBM-cold), MFMA forced from 3 columns
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
S="q4_0:14336:4096:4:8 q4_0:14336:4096:8:8 q4_0:4096:11008:8:8 q8_0:14336:4096:4:8 q8_0:14336:4096:8:8 q8_0:4096:11008:5:8"
for rep in 1 2 3; do for L in PRE SLOT; do
  timeout -k 10 180 env GGML_MI355X_MMA=3 GGML_MI355X_LIB=$PWD/abl/lib$L.so python scripts/mmvq_bench.py $S 2>&1 | grep -v amdgpu.ids | sed "s/^/$L rep$rep /" >> $O/slot.txt || exit 1
done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmvq_mma.py > $O/tests.txt 2>&1; echo "tests rc=$?" >> $O/tests.txt
