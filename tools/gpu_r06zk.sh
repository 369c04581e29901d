#!/bin/bash
# round 6: records for most of a plan's docs or none -- parity, every group-by (records on / off), the bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_group_records.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06zk_pytest.log 2>&1 || { tail -40 gpurun_out/r06zk_pytest.log; exit 1; }
tail -1 gpurun_out/r06zk_pytest.log
timeout -k 10 500 python -u tools/gb_ab.py --layout sorted --reps 15 --warmup 3 --set "" --set "PHIP_GB_RECORD=0" > gpurun_out/r06zk_rec_ab.log 2>&1 || { tail -5 gpurun_out/r06zk_rec_ab.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r06zk_bench.log 2>&1 || { tail -20 gpurun_out/r06zk_bench.log; exit 1; }
tail -1 gpurun_out/r06zk_bench.log | cut -c1-200
