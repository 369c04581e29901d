#!/bin/bash
# round 6: group-by walk A/Bs -- (1) the batched LDS-table walk forced (PHIP_GB_BATCH=1) for the hot HLL / value
# group-bys that default to the one-chunk walk (C5, Q3.1, Q4.1); (2) KBATCH=8 (tools/ablib/kb8.so: 8 chunks of 64
# matched docs per gather round trip) against the default, two processes per variant; then the agg-kernel PMC passes
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gb_ab.py --queries C5,Q3.1,Q4.1 --layout sorted --reps 15 --warmup 3 --set "" --set "PHIP_GB_BATCH=1" --set "PHIP_GB_MODE=global" > gpurun_out/r06j_gbbatch_ab.log 2>&1 || { tail -5 gpurun_out/r06j_gbbatch_ab.log; exit 1; }
grep -v loaded_segments gpurun_out/r06j_gbbatch_ab.log | cut -c1-170
bash tools/gpu_round6.sh gbpmc r06j || exit 1
[ -f tools/ablib/kb8.so ] || exit 0
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
grep -v loaded_segments gpurun_out/r06j_kb8_ab.log | cut -c1-140
