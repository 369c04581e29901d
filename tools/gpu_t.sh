#!/bin/bash
# targeted GPU tests (args = pytest paths / -k), then optionally a bench (BENCH=1); stops at the first failure
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_t.log
[ $rc -ne 0 ] && exit $rc
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_t.log 2>&1 || { tail -20 gpurun_out/bench_t.log; exit 1; }
  tail -1 gpurun_out/bench_t.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); u=j.get('unsorted_layout',{}); print('sorted', j['value'], j['ms_per_step'], j['p50_latency_ms']); print('unsorted', u.get('value'), u.get('ms_per_step'), u.get('p50_latency_ms'))"
fi
