#!/bin/bash
# drop-in GPT-2 ms/token (reference scheduler + plugin, GPT-2 117M Q4_0) for the in-tree library
# and scratch_libs variants, interleaved: scripts/plugin_lib_ab.sh NAME...  ("head" = in-tree)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
python -c "
import sys; sys.path[:0]=['oracle','tests']
import gpt2_synth, qref
gpt2_synth.write_model('/tmp/g117.bin', gpt2_synth.GPT2_117M, qref.Q4_0, 1234)" || exit 1
for rep in 1 2 3; do
  for n in "$@"; do
    if [ "$n" = head ]; then L=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so; else L=$PWD/scratch_libs/lib$n.so; fi
    echo "$n $(timeout -k 10 120 ./oracle/_ref/gpt2_ref /tmp/g117.bin --tokens 40 --threads 16 --plugin $L --devices 1 --time-tokens 64 2>/dev/null | tail -1)"
  done
done
