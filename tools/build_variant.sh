#!/bin/bash
# Build an A/B library variant: exp/lib_<name>.so = the listed .hip sources recompiled with the
# given flags + every other object of the default build (run `make` in csrc first).
# Usage: tools/build_variant.sh <name> "<flags>" kernels_persist.hip [more.hip ...]
set -eu
name=$1 flags=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
csrc=$root/real-time-voice-cloning_amd/csrc
out=$root/exp/obj_$name
mkdir -p "$out"
objs=()
for o in "$csrc"/build/*.o; do
  b=$(basename "$o" .o)
  skip=0
  for s in "$@"; do [ "$(basename "$s" .hip)" = "$b" ] && skip=1; done
  # kernels_persist.hip rebuilt whole (part 0) replaces both of its default parts
  [ "$b" = kernels_persist_mol ] && for s in "$@"; do [ "$s" = kernels_persist.hip ] && skip=1; done
  [ $skip = 0 ] && objs+=("$o")
done
for s in "$@"; do
  b=$(basename "$s" .hip)
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fno-slp-vectorize -fPIC --offload-arch=gfx950 -I"$root/include" \
    -Wall -Wno-unused-function $flags -c "$csrc/$s" -o "$out/$b.o"
  objs+=("$out/$b.o")
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$root/exp/lib_$name.so" "${objs[@]}"
echo "built exp/lib_$name.so"
