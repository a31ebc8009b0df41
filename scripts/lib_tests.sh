#!/bin/bash
# one pytest selection against several libraries (in-tree "head" or scratch_libs/lib<NAME>.so),
# without stopping at the first failing library: scripts/lib_tests.sh "<pytest args>" NAME...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
args=$1; shift
for n in "$@"; do
  if [ "$n" = head ]; then L=ggml-gfx906_amd/libggml-hip-mi355x.so; else L=scratch_libs/lib$n.so; fi
  GGML_MI355X_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread $args > gpurun_out/lt_$n.log 2>&1
  rc=$?; echo "$n rc=$rc: $(tail -1 gpurun_out/lt_$n.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
