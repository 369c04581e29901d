#!/bin/bash
# round 6: group-by records (DevSeg.rec) -- group-by parity first, then the A/B against the columns' own layouts
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filtered_group_by.py tests/test_gpu_null_handling.py tests/test_gpu_node.py tests/test_gpu_group_one_trip.py tests/test_gpu_tuple_keys.py tests/test_gpu_raw_columns.py tests/test_gpu_limits.py tests/test_gpu_widened.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06v_pytest_gb.log 2>&1 || { tail -40 gpurun_out/r06v_pytest_gb.log; exit 1; }
tail -2 gpurun_out/r06v_pytest_gb.log
timeout -k 10 500 python -u tools/gb_ab.py --layout sorted --reps 15 --warmup 3 --set "" --set "PHIP_GB_RECORD=0" --set "PHIP_GB_BATCH=0" --set "PHIP_GB_BATCH=1" > gpurun_out/r06v_rec_ab.log 2>&1 || { tail -5 gpurun_out/r06v_rec_ab.log; exit 1; }
grep -v loaded_segments gpurun_out/r06v_rec_ab.log | cut -c1-120
