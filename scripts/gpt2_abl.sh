#!/bin/bash
# A/B the GPT-2 engine decode across variant libraries in abl/ (lib<NAME>.so), interleaved,
# three repetitions: scripts/gpt2_abl.sh NAME [NAME...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
  for n in "$@"; do
    for a in "1 256 1" "8 128 1"; do
      echo -n "$n: "; GGML_MI355X_LIB=$PWD/abl/lib$n.so timeout -k 10 120 python scripts/gpt2_bench.py $a || exit 1
    done
  done
done
