#!/bin/bash
# The drop-in GPT-2 path (reference ggml_backend_sched + our plugin) under plugin switches:
# ms/token per setting (each twice, interleaved; CFGS="VAR=v VAR=w ..." overrides the list), and
# the fusion decisions of one decode graph. PROF=1 adds a kernel trace of the default setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
python -c "
import sys; sys.path[:0]=['oracle','tests']
import gpt2_synth, qref
gpt2_synth.write_model('/tmp/g117.bin', gpt2_synth.GPT2_117M, qref.Q4_0, 1234)" || exit 1
R="./oracle/_ref/gpt2_ref /tmp/g117.bin --tokens 40 --threads 16 --plugin $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so --devices 1"
timeout -k 10 120 env GGML_MI355X_DEBUG=1 $R --time-tokens 4 > /dev/null 2> gpurun_out/plugin_debug.log || exit 1
echo "per decode graph (last of 4): $(grep -c 'folded' gpurun_out/plugin_debug.log) folds, $(grep -c 'fused' gpurun_out/plugin_debug.log) fused runs in all graphs"
grep -E "capture|changed" gpurun_out/plugin_debug.log | tail -3
for rep in 1 2; do
  for cfg in ${CFGS:-GGML_MI355X_GRAPHS=1 GGML_MI355X_GRAPHS=0}; do
    echo "$cfg $(timeout -k 10 120 env $cfg $R --time-tokens 64 2>/dev/null | tail -1)"
  done
done
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/plugprof -o run -- $R --time-tokens 64 > /dev/null 2>&1 || exit 1
  python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/plugprof/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"kernel time, whole run (40-token prompt + 64 + warm-up decode steps): {tot/1e6:.3f} ms in {calls} launches")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f"  {r['Name'][:70]:70s} {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:7.2f} us")
PY
fi
