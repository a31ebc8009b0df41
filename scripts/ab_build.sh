#!/bin/bash
# build an A/B variant library: scripts/ab_build.sh NAME REV FILE [FILE...]
#   compiles FILE(s) as they are at git revision REV (other objects as built in-tree) into
#   scratch_libs/lib<NAME>.so; run with GGML_MI355X_LIB=$PWD/scratch_libs/lib<NAME>.so
set -eu
cd "$(dirname "$0")/.."
name=$1; rev=$2; shift 2
mkdir -p scratch_libs/obj/$name
objs=""
for f in "$@"; do
  base=$(basename "$f"); stem=${base%.*}
  git show "$rev:$f" > scratch_libs/obj/$name/$base
  cp ggml-gfx906_amd/csrc/*.h scratch_libs/obj/$name/ 2>/dev/null || true
  x=""; [ "$stem" = mmq8 ] && x="-Xclang -target-feature -Xclang -packed-fp32-ops"   # as the Makefile
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -Iggml-gfx906_amd/csrc $x \
      -c scratch_libs/obj/$name/$base -o scratch_libs/obj/$name/$stem.o 2>&1 | grep -v "recognized feature" || true
  objs="$objs scratch_libs/obj/$name/$stem.o"
done
keep=""
for o in ggml-gfx906_amd/build/*.o; do
  skip=0
  for f in "$@"; do b=$(basename "$f"); [ "$(basename "$o")" = "${b%.*}.o" ] && skip=1; done
  [ $skip = 0 ] && keep="$keep $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o scratch_libs/lib$name.so $keep $objs -ldl
echo "scratch_libs/lib$name.so"
