#!/bin/bash
# Drop-in GPT-2 decode rate (reference scheduler + our plugin) under env variants:
#   scripts/plugin_gpt2_env.sh "" "GGML_MI355X_FUSED_LPR64_MAXN=4096" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python -c "
import sys; sys.path[:0]=['oracle','tests']
import gpt2_synth, qref
gpt2_synth.write_model('/tmp/g117.bin', gpt2_synth.GPT2_117M, qref.Q4_0, 1234)" || exit 1
for v in "$@"; do
  for rep in 1 2; do
    r=$(env $v timeout -k 10 60 ./oracle/_ref/gpt2_ref /tmp/g117.bin --tokens 40 --threads 16 --plugin $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so --devices 1 --time-tokens 128 2>/dev/null | tail -1) || exit 1
    echo "[$v] $r"
  done
done
