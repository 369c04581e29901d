#!/bin/bash
# round 6: Q3.1 alone (no other query's records resident) on the library before / after the group-by records
mkdir -p gpurun_out
: > gpurun_out/r06zc_q31.log
for v in pre cur pre cur; do
  if [ $v = pre ]; then export PHIP_LIB=tools/ablib/pre_rec.so; else unset PHIP_LIB; fi
  echo "== $v" >> gpurun_out/r06zc_q31.log
  timeout -k 10 300 python -u tools/gb_ab.py --queries Q3.1 --layout sorted --reps 15 --warmup 3 >> gpurun_out/r06zc_q31.log 2>&1 || { tail -5 gpurun_out/r06zc_q31.log; exit 1; }
done
unset PHIP_LIB
echo "== cur after Q4.1,Q2.1 records" >> gpurun_out/r06zc_q31.log
timeout -k 10 300 python -u tools/gb_ab.py --queries Q4.1,Q2.1,Q3.1 --layout sorted --reps 15 --warmup 3 >> gpurun_out/r06zc_q31.log 2>&1 || { tail -5 gpurun_out/r06zc_q31.log; exit 1; }
echo "== cur, records off (none built)" >> gpurun_out/r06zc_q31.log
PHIP_GB_RECORD=0 timeout -k 10 300 python -u tools/gb_ab.py --queries Q4.1,Q2.1,Q3.1 --layout sorted --reps 15 --warmup 3 >> gpurun_out/r06zc_q31.log 2>&1 || { tail -5 gpurun_out/r06zc_q31.log; exit 1; }
grep -E "^==|query" gpurun_out/r06zc_q31.log | cut -c1-110
