#!/bin/bash
# round 6: which earlier query slows Q3.1 afterwards
mkdir -p gpurun_out
: > gpurun_out/r06zi_order.log
for spec in "Q2.1,Q3.1" "Q2.1,Q3.1 PHIP_GB_RECORD=0" "Q2.3,Q3.1" "Q4.2,Q3.1" "C5,Q3.1"; do
  set -- $spec
  q=$1; shift
  echo "== $q $*" >> gpurun_out/r06zi_order.log
  timeout -k 10 300 env $* python -u tools/gb_ab.py --queries $q --layout sorted --reps 15 --warmup 3 >> gpurun_out/r06zi_order.log 2>&1 || { tail -5 gpurun_out/r06zi_order.log; exit 1; }
done
grep -E "^==|query" gpurun_out/r06zi_order.log | cut -c1-100
