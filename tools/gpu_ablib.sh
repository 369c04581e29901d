#!/bin/bash
# A/B of library builds (tools/ab_build.sh): tools/gb_ab.py once per library, same queries / layout.
# usage: QUERIES=Q1.1,Q1.2 LAYOUT=sorted tools/gpu_ablib.sh <tag> base tools/ablib/w5.so ...
set -u
TAG=$1; shift
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib" >> gpurun_out/ablib_$TAG.log
  if [ "$lib" = base ]; then unset PHIP_LIB; else export PHIP_LIB=$lib; fi
  timeout -k 10 300 python -u tools/gb_ab.py --queries ${QUERIES:-Q1.1,Q1.2,Q1.3} --layout ${LAYOUT:-sorted} \
    --reps ${REPS:-30} >> gpurun_out/ablib_$TAG.log 2>&1 || exit $?
done
