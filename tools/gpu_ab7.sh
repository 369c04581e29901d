#!/bin/bash
# round 3: aggregation-kernel value dictionaries of <= 64 entries read by ds_bpermute from registers (default) vs
# gathered from HBM (PHIP_AGG_SMALL_DICT=0); parity tests first
set -u
mkdir -p gpurun_out
bash tools/gpu_t.sh tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_fused_stage.py || exit 1
BENCH_ARGS="--layout both" bash tools/ab_env.sh ${TAG:-ab7} "PHIP_AGG_SMALL_DICT=0" "PHIP_AGG_SMALL_DICT=1" \
  "PHIP_AGG_SMALL_DICT=0" "PHIP_AGG_SMALL_DICT=1" || exit 1
