#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_node.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06zr_pytest_node.log 2>&1 || { tail -40 gpurun_out/r06zr_pytest_node.log; exit 1; }
tail -2 gpurun_out/r06zr_pytest_node.log
