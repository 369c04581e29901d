#!/bin/bash
# round 6: KBATCH=8 A/B of the group-by walk (tools/ablib/kb8.so: 8 chunks of 64 matched docs per gather round trip
# instead of 4), two processes per variant on the same box; then the agg-kernel PMC passes (gpu_round6.sh gbpmc)
mkdir -p gpurun_out
: > gpurun_out/r06j_kb8_ab.log
Q=C5,Q3.1,Q4.1,Q2.1,Q2.2,Q4.2
for rep in 1 2; do
  for v in default kb8; do
    if [ $v = kb8 ]; then export PHIP_LIB=tools/ablib/kb8.so; else unset PHIP_LIB; fi
    echo "== $v $rep" >> gpurun_out/r06j_kb8_ab.log
    timeout -k 10 200 python -u tools/gb_ab.py --queries $Q --layout sorted --reps 15 --warmup 3 >> gpurun_out/r06j_kb8_ab.log 2>&1 || { tail -5 gpurun_out/r06j_kb8_ab.log; exit 1; }
  done
done
unset PHIP_LIB
grep -v loaded_segments gpurun_out/r06j_kb8_ab.log | cut -c1-160
bash tools/gpu_round6.sh gbpmc r06j
