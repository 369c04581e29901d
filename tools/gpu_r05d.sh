#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py \
  tests/test_gpu_materialize.py tests/test_gpu_fused_stage.py tests/test_gpu_parity.py > gpurun_out/r05k_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r05k_tests.log; [ $rc -le 1 ] || exit $rc
for lay in sorted unsorted; do
  timeout -k 10 300 python -u tools/gb_ab.py --queries Q1.1,Q1.2,Q1.3 --layout $lay --reps 30 --set "" --set PHIP_FUSED_PIPE=0 > gpurun_out/r05k_pipe_$lay.log 2>&1 || exit $?
  PHIP_LIB=tools/ablib/prepipe.so timeout -k 10 300 python -u tools/gb_ab.py --queries Q1.1,Q1.2,Q1.3 --layout $lay --reps 30 > gpurun_out/r05k_prepipe_$lay.log 2>&1 || exit $?
done
