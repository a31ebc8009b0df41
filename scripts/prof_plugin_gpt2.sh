#!/bin/bash
# The drop-in GPT-2 path (reference ggml_backend_sched + our plugin): host phase times per token,
# then a rocprofv3 kernel-trace summary of the same run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/plugin_gpt2; rm -rf $O; mkdir -p $O
python -c "
import sys; sys.path[:0]=['oracle','tests']
import gpt2_synth, qref
gpt2_synth.write_model('/tmp/g117.bin', gpt2_synth.GPT2_117M, qref.Q4_0, 1234)" || exit 1
T=${THREADS:-16}
timeout -k 10 120 ./oracle/_ref/gpt2_ref /tmp/g117.bin --tokens 40 --threads $T --plugin $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so --devices 1 --time-tokens 64 > $O/run.json 2> $O/run.err || { tail -5 $O/run.err; exit 1; }
tail -1 $O/run.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- ./oracle/_ref/gpt2_ref /tmp/g117.bin --tokens 40 --threads $T --plugin $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so --devices 1 --time-tokens 64 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
calls = sum(int(r['Calls']) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms over {calls} dispatches")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:20]:
    print(f"{r['Name'][:80]:80s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1000:7.2f} us  total {float(r['TotalDurationNs'])/1e6:7.2f} ms")
PY
find $O/prof -name '*kernel_trace.csv' -size +1M -delete
