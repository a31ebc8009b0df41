#!/bin/bash
# A/B the GPT-2 decode between the in-tree library and scratch_libs variants, interleaved:
#   scripts/gpt2_ab.sh NAME [NAME...]   (NAME = scratch_libs/lib<NAME>.so; "head" = in-tree)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
  for n in "$@"; do
    if [ "$n" = head ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/lib$n.so; fi
    for a in "1 256 1" "8 128 1"; do
      echo -n "$n: "; GGML_MI355X_LIB=$PWD/$L timeout -k 10 120 python scripts/gpt2_bench.py $a || exit 1
    done
  done
done
