#!/bin/bash
# GPU parity tests + filter probe (measurement aid); VARIANTS="tag:ENV=val ..." adds A/B runs
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
A="select count(*) from lineorder where LO_DISCOUNT between 1 and 3"
E="select count(*) from lineorder where D_YEAR = 1993 and LO_DISCOUNT between 1 and 3 and LO_QUANTITY < 25"
F="select count(*) from lineorder where D_YEARMONTHNUM = 199401 and LO_DISCOUNT between 4 and 6 and LO_QUANTITY between 26 and 35"
for v in base:PHIP_X=1 ${VARIANTS:-}; do
  tag=${v%%:*}; ev=${v#*:}
  env $ev timeout -k 10 200 python -u tools/explore.py --reps 7 "$A" "$E" "$F" Q1.1 Q1.2 Q1.3 ${EXTRA:-} > gpurun_out/quick_$tag.log 2>&1 || { tail gpurun_out/quick_$tag.log; exit 1; }
  echo "== $tag ($ev)"
  grep query gpurun_out/quick_$tag.log | python3 -c "import sys,json; [print(d['query'][:60].ljust(60), d['scan_ms'], d['device_ms'], d['alg_GBps']) for d in map(json.loads, sys.stdin)]"
done
