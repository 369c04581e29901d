#!/bin/bash
# round 3: fused launches keep 6 workgroups per CU (no mid-size reduction); fused parity first
set -u
mkdir -p gpurun_out
bash tools/gpu_t.sh tests/test_gpu_fused.py tests/test_gpu_fused_stage.py || exit 1
BENCH_ARGS="--layout both" bash tools/ab_env.sh ${TAG:-ab12} "PHIP_X=1" "PHIP_X=2" || exit 1
