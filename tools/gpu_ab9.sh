#!/bin/bash
# round 3: large conjunctive scans fused with deferred gathers (default) vs the size rule alone; fused parity tests first
set -u
mkdir -p gpurun_out
bash tools/gpu_t.sh tests/test_gpu_fused.py tests/test_gpu_fused_stage.py tests/test_gpu_parity.py tests/test_gpu_bitslice.py || exit 1
BENCH_ARGS="--layout both" bash tools/ab_env.sh ${TAG:-ab9} "PHIP_X=1" "PHIP_FUSE_LARGE=0" "PHIP_X=2" "PHIP_FUSE_LARGE=0 PHIP_X=2" || exit 1
