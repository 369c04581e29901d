#!/bin/bash
# A/B of two library builds on the headline queries in one GPU call (measurement aid)
set -u
mkdir -p gpurun_out
for round in 1 2; do
for lib in ab/libpinot_hip_base.so pinot_amd/libpinot_hip.so; do
  PHIP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/explore.py --reps 9 Q1.1 Q1.2 Q1.3 "select sum(LO_DISCOUNT) from lineorder" > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
  echo "== $lib"; grep query gpurun_out/ab.log | python3 -c "import sys,json; [print(d['query'][:30].ljust(30), d['scan_ms'], d['device_ms']) for d in map(json.loads, sys.stdin)]"
done
done
