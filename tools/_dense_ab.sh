#!/bin/bash
# A/B of the aggregation walks inside one GPU call (measurement aid)
set -u
mkdir -p gpurun_out
Q=("select sum(LO_DISCOUNT) from lineorder" "select sum(LO_DISCOUNT), count(*) from lineorder where LO_QUANTITY < 40" "select sum(LO_EXTENDEDPRICE) from lineorder" Q1.1)
for cfg in "PHIP_AGG_LDS_DICT=0" "X=1"; do
  env $cfg timeout -k 10 200 python -u tools/explore.py --reps 7 "${Q[@]}" > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
  echo "== $cfg"; grep query gpurun_out/ab.log | python3 -c "import sys,json; [print(d['query'][:50].ljust(50), d['scan_ms'], d['device_ms'], d['alg_GBps']) for d in map(json.loads, sys.stdin)]"
done
