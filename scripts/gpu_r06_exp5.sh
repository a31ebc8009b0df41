# round-6 session step: the single-wave mat-vec (GGML_MI355X_SOLO) against the 8-wave kernel on
# the single-matrix BASELINE shapes, and its parity tests
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mmvq_solo.py > $O/tests.txt 2>&1 || { echo "solo tests failed"; tail -20 $O/tests.txt; exit 1; }
REPS=2 scripts/singles_ab.sh "base=abl/libSOLO.so" "solo4=abl/libSOLO.so:GGML_MI355X_SOLO=4" "solo2=abl/libSOLO.so:GGML_MI355X_SOLO=2" "solo8=abl/libSOLO.so:GGML_MI355X_SOLO=8" > $O/sab.txt 2>&1
