#!/bin/bash
# round 6: completion polling + timing markers off -- correctness subset, then a host A/B of the sorted headline step
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_concurrency.py tests/test_gpu_query_options.py tests/test_gpu_filter_programs.py tests/test_gpu_poll_done.py tests/test_gpu_hash_growth.py tests/test_gpu_raw_columns.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06i_pytest.log 2>&1 || { tail -30 gpurun_out/r06i_pytest.log; exit 1; }
tail -2 gpurun_out/r06i_pytest.log
B="--group-by= --configs= --layout sorted --no-cpu-baseline --no-parity --no-concurrent --steps 30 --warmup 5"
: > gpurun_out/r06i_ab.log
for rep in 1 2; do
  for v in default poll0 markers; do
    case $v in
      default) E=""; X="";;
      poll0) E="PHIP_POLL_DONE=0"; X="";;
      markers) E=""; X="--timed-markers";;
    esac
    env $E timeout -k 10 120 python -u bench.py $B $X > gpurun_out/r06i_$v.log 2>&1 || { tail -5 gpurun_out/r06i_$v.log; exit 1; }
    python3 -c "
import json,sys
p=json.loads([l for l in open('gpurun_out/r06i_$v.log') if l.startswith('{')][-1])
print('$v', $rep, p['ms_per_step'], p['value'], p['p50_latency_ms'], p['roofline']['kernels']['fused_filter_agg']['per_query_ms'])" >> gpurun_out/r06i_ab.log
  done
done
cat gpurun_out/r06i_ab.log
