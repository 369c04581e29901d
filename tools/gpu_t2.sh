#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_startree.py tests/test_gpu_pinot_startree.py tests/test_gpu_parity.py -k "star or raw_column" -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_t2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_t2.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab5.sh
