#!/bin/bash
# fused aggregation's deferred ring depth (kFusedRingDefer 512 default vs 1024 / 256): sorted and unsorted Q1.x
set -u
mkdir -p gpurun_out
QUERIES=Q1.1,Q1.2,Q1.3 LAYOUT=sorted bash tools/gpu_ablib.sh r05zr base tools/ablib/rd1024.so || exit 1
QUERIES=Q1.1,Q1.2,Q1.3 LAYOUT=unsorted REPS=20 bash tools/gpu_ablib.sh r05zr_u base tools/ablib/rd1024.so || exit 1
grep -h '"query"' gpurun_out/ablib_r05zr.log gpurun_out/ablib_r05zr_u.log | cut -c1-160
