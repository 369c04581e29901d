#!/bin/bash
# round 3: fusion policy on the unsorted layout (sparse Q1.2 / Q1.3 fused by estimated matches per tile since
# 388bd6c) -- A/B of the fused walk, deferral and the size-only rule; then the distributed GPU tests.
set -u
mkdir -p gpurun_out
bash tools/ab_env.sh ${TAG:-ab3} "PHIP_X=1" "PHIP_FUSE_PER_TILE=0" "PHIP_FILTER_WALK=contig" "PHIP_FUSED_DEFER=0" \
  "PHIP_FILTER_WALK=contig PHIP_FUSED_DEFER=0" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_dist.log; exit $rc
