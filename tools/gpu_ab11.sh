#!/bin/bash
# round 3: workgroups per CU of the fused large-scan launch (the runtime's rule vs fixed 2..6)
set -u
mkdir -p gpurun_out
BENCH_ARGS="--layout both" bash tools/ab_env.sh ${TAG:-ab11} "PHIP_X=1" "PHIP_FILTER_BPC=6" "PHIP_FILTER_BPC=4" \
  "PHIP_FILTER_BPC=3" "PHIP_FILTER_BPC=2" "PHIP_X=2" || exit 1
