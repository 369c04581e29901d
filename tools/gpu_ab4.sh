#!/bin/bash
# round 3: sorted Q1.1's aggregation -- staged (LDS-DMA) dense-tile walk vs the per-doc ring walk
set -u
mkdir -p gpurun_out
BENCH_ARGS="--layout sorted --queries Q1.1" bash tools/ab_env.sh ${TAG:-ab4} "PHIP_X=1" \
  "PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=1" "PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=128" "PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=640" \
  "PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=1 PHIP_AGG_STAGE=0" "PHIP_FUSE=1" || exit 1
