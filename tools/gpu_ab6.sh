#!/bin/bash
# round 3: one dwordx2 per decoded id (vs two dword loads: PHIP_LIB=ab/libpinot_hip_base.so) on both layouts, then
# unsorted filter evaluation knobs (sparse walk bound, P-layout width, workgroups per CU, stream-only probe)
set -u
mkdir -p gpurun_out
bash tools/ab_env.sh ${TAG:-ab6a} "PHIP_LIB=ab/libpinot_hip_base.so" "PHIP_X=1" "PHIP_LIB=ab/libpinot_hip_base.so PHIP_X=2" \
  "PHIP_X=2" || exit 1
BENCH_ARGS="--layout unsorted" bash tools/ab_env.sh ${TAG:-ab6} "PHIP_X=1" "PHIP_SPARSE_MAX=12" \
  "PHIP_SPARSE_MAX=3" "PHIP_NO_SPARSE=1" "PHIP_CONJ_P=4" "PHIP_FILTER_PROBE=1" "PHIP_FILTER_BPC=4" "PHIP_FILTER_BPC=8" || exit 1
