#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_agg_hist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06zv_pytest_hist.log 2>&1 || { tail -40 gpurun_out/r06zv_pytest_hist.log; exit 1; }
tail -1 gpurun_out/r06zv_pytest_hist.log
