#!/bin/bash
mkdir -p gpurun_out
PHIP_WALK_TRACE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_agg_hist.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r06zw_pytest_hist.log 2>&1 || { tail -40 gpurun_out/r06zw_pytest_hist.log; exit 1; }
grep -c "phip_hist.*on" gpurun_out/r06zw_pytest_hist.log; grep -c "phip_hist.*off" gpurun_out/r06zw_pytest_hist.log; tail -1 gpurun_out/r06zw_pytest_hist.log
