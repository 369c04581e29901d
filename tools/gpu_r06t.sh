#!/bin/bash
# round 6 (verdict r05 #5): the unsorted fused scans with the value columns streamed with every tile vs gathered
export BENCH_ARGS="--layout unsorted --configs= --group-by= --no-parity --no-concurrent --c5 off"
bash tools/ab_env.sh r06t_sv "PHIP_KERNEL_TIMING=1" "PHIP_STREAM_VALUES=1" "PHIP_STREAM_VALUES=1 PHIP_STREAM_PACKED=0" "PHIP_FUSED_DEFER=0"
