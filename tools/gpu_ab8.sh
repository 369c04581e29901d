#!/bin/bash
# round 3: fusion policy after the bit-sliced conjunction -- split (default) vs fused (values streamed / gathered)
set -u
mkdir -p gpurun_out
BENCH_ARGS="--layout both" bash tools/ab_env.sh ${TAG:-ab8} "PHIP_X=1" "PHIP_FUSE=1" "PHIP_FUSE=1 PHIP_STREAM_VALUES=0" \
  "PHIP_FUSE=1 PHIP_FUSED_DEFER=0" "PHIP_X=2" || exit 1
