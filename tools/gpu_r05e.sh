#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_group_one_trip.py tests/test_gpu_materialize.py tests/test_gpu_limits.py tests/test_gpu_widened.py \
  > gpurun_out/r05m_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r05m_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/gb_ab.py --queries Q2.1,Q2.2,Q2.3,Q3.1,Q4.1,Q4.2,C5 --layout sorted --reps 20 \
  --set "" --set PHIP_GB_WAVES=8 > gpurun_out/r05m_gb16.log 2>&1 || exit $?
bash tools/host_trace.sh > gpurun_out/r05m_host_trace.log 2>&1 || exit $?
