#!/bin/bash
# round 6: group-by records as their own agg_kernel variant -- parity, then the library before records against this one
# (Q3.1 keeps its columns: it must be back to the pre-record time), then the bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_group_records.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06za_pytest_rec.log 2>&1 || { tail -40 gpurun_out/r06za_pytest_rec.log; exit 1; }
tail -1 gpurun_out/r06za_pytest_rec.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filtered_group_by.py tests/test_gpu_null_handling.py tests/test_gpu_node.py tests/test_gpu_group_one_trip.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06za_pytest_gb.log 2>&1 || { tail -40 gpurun_out/r06za_pytest_gb.log; exit 1; }
tail -1 gpurun_out/r06za_pytest_gb.log
: > gpurun_out/r06za_lib_ab.log
for rep in 1 2; do
  for v in pre cur; do
    if [ $v = pre ]; then export PHIP_LIB=tools/ablib/pre_rec.so; else unset PHIP_LIB; fi
    echo "== $v $rep" >> gpurun_out/r06za_lib_ab.log
    timeout -k 10 300 python -u tools/gb_ab.py --layout sorted --reps 15 --warmup 3 >> gpurun_out/r06za_lib_ab.log 2>&1 || { tail -5 gpurun_out/r06za_lib_ab.log; exit 1; }
  done
done
unset PHIP_LIB
timeout -k 10 600 python -u bench.py > gpurun_out/r06za_bench.log 2>&1 || { tail -20 gpurun_out/r06za_bench.log; exit 1; }
tail -1 gpurun_out/r06za_bench.log | cut -c1-200
