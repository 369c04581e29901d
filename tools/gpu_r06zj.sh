#!/bin/bash
# round 6: Q3.1's walk / record flag alone and after Q2.1 (PHIP_WALK_TRACE)
mkdir -p gpurun_out
: > gpurun_out/r06zj_trace.log
for q in Q3.1 Q2.1,Q3.1; do
  echo "== $q" >> gpurun_out/r06zj_trace.log
  PHIP_WALK_TRACE=1 timeout -k 10 300 python -u tools/gb_ab.py --queries $q --layout sorted --reps 4 --warmup 1 >> gpurun_out/r06zj_trace.log 2>&1 || { tail -5 gpurun_out/r06zj_trace.log; exit 1; }
done
grep -E "^==|query|phip_walk" gpurun_out/r06zj_trace.log | cut -c1-140
