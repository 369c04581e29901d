#!/bin/bash
# round 6: node-plan hash-table exchange tests, then the batched group-by walk against the default over every SSB
# group-by and C5 (two alternating processes per variant)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_node.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r06k_pytest_node.log 2>&1 || { tail -30 gpurun_out/r06k_pytest_node.log; exit 1; }
tail -3 gpurun_out/r06k_pytest_node.log
: > gpurun_out/r06k_gbbatch_ab.log
Q=Q2.1,Q2.2,Q2.3,Q3.1,Q3.2,Q3.3,Q3.4,Q4.1,Q4.2,Q4.3,C5
for rep in 1 2; do
  echo "== rep $rep" >> gpurun_out/r06k_gbbatch_ab.log
  timeout -k 10 300 python -u tools/gb_ab.py --queries $Q --layout sorted --reps 15 --warmup 3 --set "" --set "PHIP_GB_BATCH=1" --set "PHIP_GB_BATCH=0" >> gpurun_out/r06k_gbbatch_ab.log 2>&1 || { tail -5 gpurun_out/r06k_gbbatch_ab.log; exit 1; }
done
grep -v loaded_segments gpurun_out/r06k_gbbatch_ab.log | cut -c1-110
