#!/bin/bash
# scripts/mv_sweep.sh OUT "SHAPES" "VARIANT" ... — graph periods (scripts/mv_graph.py, warm and
# cold) of the mat-vec shapes under each knob setting; VARIANT = "default" or space-free
# KEY=VAL,KEY=VAL (GGML_MI355X_ prefix added)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; shapes=$2; shift 2
mkdir -p "$(dirname "$out")"
for v in "$@"; do
  envs=""
  if [ "$v" != default ]; then for kv in ${v//,/ }; do envs="$envs GGML_MI355X_$kv"; done; fi
  timeout -k 10 900 env $envs python scripts/mv_graph.py $shapes >> "$out" 2>&1 || { echo "variant $v failed"; tail -5 "$out"; exit 1; }
done
