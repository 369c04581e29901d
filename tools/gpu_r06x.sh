#!/bin/bash
# round 6: group-by records -- the dedicated parity tests, the group-by suites, then the A/B and the bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_group_records.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06x_pytest_rec.log 2>&1 || { tail -40 gpurun_out/r06x_pytest_rec.log; exit 1; }
tail -2 gpurun_out/r06x_pytest_rec.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filtered_group_by.py tests/test_gpu_null_handling.py tests/test_gpu_node.py tests/test_gpu_group_one_trip.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06x_pytest_gb.log 2>&1 || { tail -40 gpurun_out/r06x_pytest_gb.log; exit 1; }
tail -2 gpurun_out/r06x_pytest_gb.log
W="from lineorder where C_REGION = 'AMERICA' and S_REGION = 'AMERICA'"
timeout -k 10 500 python -u tools/gb_ab.py --layout sorted --reps 15 --warmup 3 --set "" --set "PHIP_GB_RECORD=0" --set "PHIP_GB_BATCH=0" --set "PHIP_GB_BATCH=1" > gpurun_out/r06x_rec_ab.log 2>&1 || { tail -5 gpurun_out/r06x_rec_ab.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r06x_bench.log 2>&1 || { tail -20 gpurun_out/r06x_bench.log; exit 1; }
tail -1 gpurun_out/r06x_bench.log | cut -c1-200
