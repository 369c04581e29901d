#!/bin/bash
# round 6: 16-wave workgroups for every LDS group table that keeps more waves resident -- parity of the group-by tests,
# then the waves x walk A/B over every SSB group-by and C5 (two processes per variant set)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filtered_group_by.py tests/test_gpu_null_handling.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06l_pytest_gb.log 2>&1 || { tail -30 gpurun_out/r06l_pytest_gb.log; exit 1; }
tail -3 gpurun_out/r06l_pytest_gb.log
: > gpurun_out/r06l_waves_ab.log
Q=Q2.1,Q2.2,Q2.3,Q3.1,Q4.1,Q4.2,Q4.3,C5
for rep in 1 2; do
  echo "== rep $rep" >> gpurun_out/r06l_waves_ab.log
  timeout -k 10 300 python -u tools/gb_ab.py --queries $Q --layout sorted --reps 15 --warmup 3 --set "" --set "PHIP_GB_WAVES=8" --set "PHIP_GB_BATCH=1" --set "PHIP_GB_BATCH=1 PHIP_GB_WAVES=8" --set "PHIP_GB_BATCH=0" >> gpurun_out/r06l_waves_ab.log 2>&1 || { tail -5 gpurun_out/r06l_waves_ab.log; exit 1; }
done
grep -v loaded_segments gpurun_out/r06l_waves_ab.log | cut -c1-110
