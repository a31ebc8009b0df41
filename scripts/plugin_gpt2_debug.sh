#!/bin/bash
# fusion decisions of the drop-in GPT-2 decode graphs (GGML_MI355X_DEBUG=1), last lines matching $1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python -c "
import sys; sys.path[:0]=['oracle','tests']
import gpt2_synth, qref
gpt2_synth.write_model('/tmp/g117.bin', gpt2_synth.GPT2_117M, qref.Q4_0, 1234)" || exit 1
GGML_MI355X_DEBUG=1 timeout -k 10 100 ./oracle/_ref/gpt2_ref /tmp/g117.bin --tokens 40 --threads 16 --plugin $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so --devices 1 --time-tokens 2 > /dev/null 2> gpurun_out/plugin_debug.log || exit 1
grep -E "${1:-fold}" gpurun_out/plugin_debug.log | tail -${2:-8}
