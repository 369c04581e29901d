#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprof kernel trace, FETCH/WRITE PMC passes for the
# traffic figure. Stops at the first failure / timeout (never retries).
# usage: tools/gpu_round.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
mkdir -p gpurun_out
: > gpurun_out/steps.log
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$name] start $(date +%T)" >> gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(date +%T)" >> gpurun_out/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -30 "gpurun_out/$name.log"; exit $rc; fi
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 400 python -u bench.py --steps 10 --warmup 3 "$@"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@"
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$TAG -o run -- python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@"
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$TAG -o run -- python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@"
python3 tools/traffic.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG --steps 10 --warmup 3 --queries Q1.1,Q1.2,Q1.3 --sf 100 -o gpurun_out/traffic_$TAG.json
cat gpurun_out/steps.log
tail -2 gpurun_out/bench.log
