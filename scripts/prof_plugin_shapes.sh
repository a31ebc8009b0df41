#!/bin/bash
# Per-(kernel, grid) durations of the drop-in GPT-2 decode (reference scheduler + plugin):
# splits the fused mat-vec by matrix shape (grid size), which the --stats summary merges.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/plugin_shapes; rm -rf $O; mkdir -p $O
python -c "
import sys; sys.path[:0]=['oracle','tests']
import gpt2_synth, qref
gpt2_synth.write_model('/tmp/g117.bin', gpt2_synth.GPT2_117M, qref.Q4_0, 1234)" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- ./oracle/_ref/gpt2_ref /tmp/g117.bin --tokens 40 --threads 16 --plugin $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so --devices 1 --time-tokens 64 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    k = (r['Kernel_Name'][:60], r.get('Grid_Size_X', r.get('Grid_Size', '?')), r.get('Grid_Size_Z', ''), r.get('Workgroup_Size_X', ''))
    agg[k].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
tot = sum(sum(v) for v in agg.values())
print(f"total {tot/1e6:.2f} ms, {sum(len(v) for v in agg.values())} dispatches")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:25]:
    v.sort()
    print(f"{k[0]:60s} grid {k[1]:>7s} z {k[2]:>3s} n {len(v):6d} avg {sum(v)/len(v)/1e3:7.2f} us  med {v[len(v)//2]/1e3:7.2f}  total {sum(v)/1e6:6.2f} ms")
PY
rm -f $f
