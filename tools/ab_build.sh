#!/bin/bash
# A/B library variants: recompile filter.hip, aggregate.hip and runtime.cpp with extra defines, link them with the in-tree objects
# of the other sources into tools/ablib/<name>.so (load it with PHIP_LIB=tools/ablib/<name>.so).
# usage: tools/ab_build.sh <name> "-DPHIP_FUSED_WAVES=4 ..."
set -eu
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/pinot_amd/csrc
B=/tmp/abbuild/$NAME
mkdir -p "$B" "$ROOT/tools/ablib"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics -fvisibility=hidden"
(cd "$C" && make -s)
for f in filter.hip aggregate.hip runtime.cpp; do
  (cd "$C" && /opt/rocm/bin/hipcc $FLAGS $DEFS -c -o "$B/${f%.*}.o" $f) &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fvisibility=hidden -o "$ROOT/tools/ablib/$NAME.so" \
  "$B/filter.o" "$B/aggregate.o" "$C/load.o" "$C/trim.o" "$C/limit.o" "$C/select.o" "$B/runtime.o"
echo "built tools/ablib/$NAME.so"
