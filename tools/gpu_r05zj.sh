#!/bin/bash
# sorted Q1.1 deferred path after packed values: workgroups per CU
set -u
mkdir -p gpurun_out
BENCH_ARGS="--layout sorted" bash tools/ab_env.sh r05zj "PHIP_X=0" "PHIP_FILTER_BPC=2" "PHIP_FILTER_BPC=4" "PHIP_FILTER_BPC=5" "PHIP_FILTER_BPC=6" || exit 1
