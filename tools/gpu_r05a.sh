#!/bin/bash
# round-5 measurement batch: new GPU tests, then A/Bs of the fused dense tiles and the filter grid, then the host
# breakdown of the C3 group-bys (sorted layout). Every GPU step has its own time limit; a failing step ends the batch.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_widened.py \
  tests/test_gpu_filter_stats.py tests/test_gpu_null_handling.py tests/test_gpu_query_options.py \
  tests/test_gpu_bitslice.py tests/test_gpu_startree.py tests/test_gpu_fused.py tests/test_gpu_materialize.py \
  tests/test_gpu_pinot_startree.py > gpurun_out/r05f_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r05f_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # (1 = a test failed: still measure; anything else ends here)
timeout -k 10 500 python -u tools/gb_ab.py --queries Q1.1,Q1.2,Q1.3 --layout sorted --set "" \
  --set PHIP_FUSED_DENSE_MIN=0 --set PHIP_FUSED_DENSE_MIN=128 --set PHIP_FUSED_DENSE_MIN=256 \
  --set PHIP_FILTER_MIN_TILES=2 --set PHIP_FILTER_MIN_TILES=4 > gpurun_out/r05e_dense.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gb_ab.py --queries Q2.1,Q3.2,Q4.3,C5 --layout sorted --set "" \
  --set PHIP_FILTER_MIN_TILES=2 --set PHIP_FILTER_MIN_TILES=4 > gpurun_out/r05e_min_tiles.log 2>&1 || exit $?
PHIP_HOST_TRACE=1 timeout -k 10 300 python -u tools/host_gb_probe.py --layout sorted \
  --queries Q2.1,Q2.3,Q3.2,Q3.4,Q4.3,C5 --reps 20 > gpurun_out/r05g_gb_host.log 2> gpurun_out/r05g_gb_host.err || exit $?
