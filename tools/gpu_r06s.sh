#!/bin/bash
# round 6 (verdict r05 #5): the unsorted fused filter and its stream-only probe under 2-6 workgroups per CU
export BENCH_ARGS="--layout unsorted --configs= --group-by= --no-parity --no-concurrent --c5 off"
bash tools/ab_env.sh r06s_bpc "PHIP_FILTER_PROBE=1 PHIP_FUSE=0" "PHIP_FILTER_PROBE=1 PHIP_FUSE=0 PHIP_FILTER_BPC=2" \
  "PHIP_FILTER_PROBE=1 PHIP_FUSE=0 PHIP_FILTER_BPC=3" "PHIP_FILTER_PROBE=1 PHIP_FUSE=0 PHIP_FILTER_BPC=6" \
  "PHIP_KERNEL_TIMING=1" "PHIP_FILTER_BPC=2" "PHIP_FILTER_BPC=3" "PHIP_FILTER_BPC=6"
