#!/bin/bash
# A/B of the sparse-conjunction bound (PHIP_SPARSE_MAX) on the headline queries (measurement aid)
set -u
mkdir -p gpurun_out
for v in 6 9 12 16; do
  PHIP_SPARSE_MAX=$v timeout -k 10 200 python -u tools/explore.py --reps 9 Q1.1 Q1.2 Q1.3 > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
  echo "== $v"; grep query gpurun_out/ab.log | python3 -c "import sys,json; [print(d['query'][:20].ljust(20), d['scan_ms'], d['device_ms']) for d in map(json.loads, sys.stdin)]"
done
