#!/bin/bash
# sorted Q1.1: stream the packed values with every tile (dense over the sorted range) vs deferred gathers; ring shapes
set -u
mkdir -p gpurun_out
BENCH_ARGS="--layout sorted" bash tools/ab_env.sh r05zh "PHIP_X=0" "PHIP_STREAM_VALUES=1" "PHIP_STREAM_VALUES=1 PHIP_FILTER_BPC=2" "PHIP_STREAM_VALUES=1 PHIP_FILTER_BPC=1" "PHIP_STREAM_VALUES=1 PHIP_FILTER_BPC=4" || exit 1
