#!/bin/bash
# All SSB queries + C5 + unfiltered aggregations through tools/explore.py (measurement aid)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/explore.py --reps 7 Q1.1 Q1.2 Q1.3 Q2.1 Q2.2 Q2.3 Q3.1 Q3.2 Q3.3 Q3.4 Q4.1 Q4.2 Q4.3 C5 \
  "select sum(LO_EXTENDEDPRICE) from lineorder" "select sum(LO_DISCOUNT) from lineorder" \
  "select count(*) from lineorder where LO_DISCOUNT between 1 and 3" > gpurun_out/allq.log 2>&1 || { tail -30 gpurun_out/allq.log; exit 1; }
grep query gpurun_out/allq.log | python3 -c "import sys,json; [print(d['query'][:44].ljust(44), d['scan_ms'], d['device_ms'], d['wall_ms'], d['alg_GBps'], d['docs_scanned']) for d in map(json.loads, sys.stdin)]"
