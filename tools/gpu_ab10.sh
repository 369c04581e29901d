#!/bin/bash
# round 3: fused deferred ring 1024 -> 512 entries per wave (eighth-tile pieces), more fused waves per CU;
# base = the previous library (ab/libpinot_hip_base.so); fused parity tests first
set -u
mkdir -p gpurun_out
bash tools/gpu_t.sh tests/test_gpu_fused.py tests/test_gpu_fused_stage.py tests/test_gpu_parity.py || exit 1
BENCH_ARGS="--layout both" bash tools/ab_env.sh ${TAG:-ab10} "PHIP_LIB=ab/libpinot_hip_base.so" "PHIP_X=1" \
  "PHIP_LIB=ab/libpinot_hip_base.so PHIP_X=2" "PHIP_X=2" || exit 1
