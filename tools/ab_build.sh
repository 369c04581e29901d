#!/bin/bash
# A/B library variants: recompile some translation units with extra defines (default: the filter kernel variants,
# filter_k_*.hip), link them with the in-tree objects of the others into tools/ablib/<name>.so (load it with
# PHIP_LIB=tools/ablib/<name>.so).
# usage: tools/ab_build.sh <name> "-DPHIP_FUSED_WAVES=4 ..." ["filter_k_fused1.hip runtime.cpp ..."]
set -eu
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/pinot_amd/csrc
SRCS=${3:-$(cd "$C" && ls filter_k_*.hip)}
B=/tmp/abbuild/$NAME
mkdir -p "$B" "$ROOT/tools/ablib"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics -fvisibility=hidden"
(cd "$C" && make -s -j8)
OBJS=""
for o in $(cd "$C" && ls *.o); do
  src=""
  for s in $SRCS; do [ "${s%.*}.o" = "$o" ] && src=$s; done
  if [ -n "$src" ]; then
    (cd "$C" && /opt/rocm/bin/hipcc $FLAGS $DEFS -c -o "$B/$o" $src) &
    OBJS="$OBJS $B/$o"
  else
    OBJS="$OBJS $C/$o"
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fvisibility=hidden -o "$ROOT/tools/ablib/$NAME.so" $OBJS
echo "built tools/ablib/$NAME.so"
