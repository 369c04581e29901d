#!/bin/bash
# round 6: the adaptive group-by walk (Plan::walk_adaptive) -- group-by parity, the per-query A/B against the forced
# walks, then the default bench line
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filtered_group_by.py tests/test_gpu_null_handling.py tests/test_gpu_node.py tests/test_gpu_group_one_trip.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06m_pytest_gb.log 2>&1 || { tail -30 gpurun_out/r06m_pytest_gb.log; exit 1; }
tail -2 gpurun_out/r06m_pytest_gb.log
timeout -k 10 300 python -u tools/gb_ab.py --layout sorted --reps 15 --warmup 3 --set "" --set "PHIP_GB_BATCH=0" --set "PHIP_GB_BATCH=1" > gpurun_out/r06m_walk_ab.log 2>&1 || { tail -5 gpurun_out/r06m_walk_ab.log; exit 1; }
grep -v loaded_segments gpurun_out/r06m_walk_ab.log | cut -c1-110
timeout -k 10 600 python -u bench.py > gpurun_out/r06m_bench.log 2>&1 || { tail -20 gpurun_out/r06m_bench.log; exit 1; }
tail -1 gpurun_out/r06m_bench.log | cut -c1-600
