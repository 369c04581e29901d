#!/bin/bash
# round 6: the id-histogram aggregation (agg_kernel kHist) -- parity, then C4 / C1 against the value gathers
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_filter_programs.py tests/test_gpu_widened.py tests/test_gpu_filtered_group_by.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06zt_pytest.log 2>&1 || { tail -40 gpurun_out/r06zt_pytest.log; exit 1; }
tail -1 gpurun_out/r06zt_pytest.log
timeout -k 10 600 python -u tools/cfg_ab.py --configs c4,c1 --reps 10 --warmup 3 --set "" --set "PHIP_AGG_HIST=0" > gpurun_out/r06zt_hist_ab.log 2>&1 || { tail -5 gpurun_out/r06zt_hist_ab.log; exit 1; }
grep '"query"' gpurun_out/r06zt_hist_ab.log | cut -c1-200
