#!/bin/bash
# round 3: GPU parity suite, then bench A/B of the aggregation walk / fusion policy against the round-2 library
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh ${TAG:-ab1} "PHIP_LIB=ab/libpinot_hip_r02.so" "PHIP_X=1" "PHIP_FUSE_PER_TILE=0" "PHIP_FUSE_PER_TILE=64" "PHIP_FUSE=1" "PHIP_FUSE=1 PHIP_FILTER_WALK=contig"
