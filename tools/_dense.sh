#!/bin/bash
# parity tests + dense / sparse aggregation timings (measurement aid)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u tools/explore.py --reps 7 Q1.1 Q1.2 Q1.3 Q2.1 Q3.1 Q4.1 C5 \
  "select sum(LO_EXTENDEDPRICE) from lineorder" "select sum(LO_DISCOUNT) from lineorder" \
  "select sum(LO_DISCOUNT), count(*) from lineorder where LO_QUANTITY < 40" \
  "select sum(CAST(LO_EXTENDEDPRICE AS DOUBLE) * LO_DISCOUNT) from lineorder where LO_QUANTITY < 25" > gpurun_out/dense.log 2>&1 || { tail -30 gpurun_out/dense.log; exit 1; }
grep query gpurun_out/dense.log | python3 -c "import sys,json; [print(d['query'][:50].ljust(50), d['scan_ms'], d['device_ms'], d['wall_ms'], d['alg_GBps'], d['docs_scanned']) for d in map(json.loads, sys.stdin)]"
