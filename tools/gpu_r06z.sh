#!/bin/bash
# round 6: the library before the group-by records (tools/ablib/pre_rec.so) against the current one, alternating
mkdir -p gpurun_out
: > gpurun_out/r06z_lib_ab.log
for rep in 1 2; do
  for v in pre cur; do
    if [ $v = pre ]; then export PHIP_LIB=tools/ablib/pre_rec.so; else unset PHIP_LIB; fi
    echo "== $v $rep" >> gpurun_out/r06z_lib_ab.log
    timeout -k 10 300 python -u tools/gb_ab.py --queries Q2.1,Q2.2,Q3.1,Q4.1,Q4.2,C5 --layout sorted --reps 15 --warmup 3 >> gpurun_out/r06z_lib_ab.log 2>&1 || { tail -5 gpurun_out/r06z_lib_ab.log; exit 1; }
  done
done
grep -v loaded_segments gpurun_out/r06z_lib_ab.log | cut -c1-100
