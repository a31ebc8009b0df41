#!/bin/bash
# drop-in GPT-2 on the small golden checkpoint of one type, GGML_MI355X_DEBUG log summary:
#   scripts/plugin_small_debug.sh q8_0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
t=${1:-q8_0}
python -c "
import sys, json; sys.path[:0]=['oracle','tests']
import gpt2_synth, qref
m=json.load(open('tests/golden/gpt2_manifest.json'))
gpt2_synth.write_model('/tmp/gs.bin', m['hparams'], qref.BY_NAME['$t'], m['seed'])
print(','.join(map(str, m['cases']['$t']['tokens'][:24])))" > /tmp/gs.tok || exit 1
GGML_MI355X_DEBUG=1 timeout -k 10 100 ./oracle/_ref/gpt2_ref /tmp/gs.bin --tokens $(cat /tmp/gs.tok) --out /tmp/gs.out --plugin $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so --devices 1 > /dev/null 2> gpurun_out/small_debug.log || exit 1
echo "layer fused: $(grep -c 'layer fused' gpurun_out/small_debug.log)  not fused: $(grep -c 'not fused' gpurun_out/small_debug.log)"
grep -v "fused\|folded\|copies" gpurun_out/small_debug.log | sort | uniq -c | sort -rn | head -20
