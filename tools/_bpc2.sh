#!/bin/bash
set -u
mkdir -p gpurun_out
A="select count(*) from lineorder where LO_DISCOUNT between 1 and 3"
E="select count(*) from lineorder where D_YEAR = 1993 and LO_DISCOUNT between 1 and 3 and LO_QUANTITY < 25"
for b in ${BPCS:-6 7 8}; do
  echo "== bpc $b"
  PHIP_FILTER_BPC=$b timeout -k 10 200 python -u tools/explore.py --reps 7 "$A" "$E" Q1.1 > gpurun_out/bpc_$b.log 2>&1 || { tail gpurun_out/bpc_$b.log; exit 1; }
  grep query gpurun_out/bpc_$b.log | python3 -c "import sys,json; [print(d['query'][:60].ljust(60), d['scan_ms'], d['device_ms'], d['alg_GBps']) for d in map(json.loads, sys.stdin)]"
done
