#!/bin/bash
# The drop-in GPT-2 path (reference ggml_backend_sched hosting our plugin) across variant
# libraries abl/lib<NAME>.so, interleaved, three repetitions: scripts/plugin_lib_abl.sh NAME [NAME...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
python -c "
import sys; sys.path[:0]=['oracle','tests']
import gpt2_synth, qref
gpt2_synth.write_model('/tmp/g117.bin', gpt2_synth.GPT2_117M, qref.Q4_0, 1234)" || exit 1
for rep in 1 2 3; do
  for n in "$@"; do
    echo "$n $(timeout -k 10 120 ./oracle/_ref/gpt2_ref /tmp/g117.bin --tokens 40 --threads 16 --plugin $PWD/abl/lib$n.so --devices 1 --time-tokens 64 2>/dev/null | tail -1)" || exit 1
  done
done
