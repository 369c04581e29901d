#!/bin/bash
# round 6: the prefetched one-chunk group-by walk (agg_kernel.h group_chunk_pf) -- group-by parity, then the A/B
# against the per-load decode (PHIP_GB_PF=0) and the batched walk
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filtered_group_by.py tests/test_gpu_null_handling.py tests/test_gpu_node.py tests/test_gpu_group_one_trip.py tests/test_gpu_tuple_keys.py tests/test_gpu_raw_columns.py tests/test_gpu_limits.py tests/test_gpu_widened.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06o_pytest_gb.log 2>&1 || { tail -30 gpurun_out/r06o_pytest_gb.log; exit 1; }
tail -2 gpurun_out/r06o_pytest_gb.log
W="from lineorder where C_REGION = 'AMERICA' and S_REGION = 'AMERICA'"
timeout -k 10 400 python -u tools/gb_ab.py --layout sorted --reps 15 --warmup 3 \
  --sql "C5cnt::select D_YEAR, C_NATION, count(*) $W group by D_YEAR, C_NATION limit 100000" \
  --sql "C5sum::select D_YEAR, C_NATION, sum(LO_REVENUE - LO_SUPPLYCOST) $W group by D_YEAR, C_NATION limit 100000" \
  --queries Q2.1,Q2.2,Q2.3,Q3.1,Q4.1,Q4.2,Q4.3,C5,C5cnt,C5sum --set "" --set "PHIP_GB_PF=0" --set "PHIP_GB_BATCH=0" --set "PHIP_GB_BATCH=1" > gpurun_out/r06o_pf_ab.log 2>&1 || { tail -5 gpurun_out/r06o_pf_ab.log; exit 1; }
grep -v loaded_segments gpurun_out/r06o_pf_ab.log | cut -c1-120
