#!/bin/bash
# One GPU call: parity tests, smoke, bench (both SSB layouts + CPU baseline), rocprof kernel trace, PMC passes
# (FETCH_SIZE / WRITE_SIZE per layout for the traffic figure, one SQ pass for VALU / LDS / stall counters).
# Stops at the first failure / timeout (never retries). usage: tools/gpu_round.sh <tag> [bench args...]
set -u
TAG=${1:-r02}; shift || true
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
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
  step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python -u bench.py --steps 10 --warmup 3 "$@"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="--no-cpu-baseline --steps 10 --warmup 3 $*"
# one kernel-trace summary per layout, so the headline (sorted) kernels' averages read straight from their own file
for L in sorted unsorted; do
  step rocprof_$L 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
done
for L in sorted unsorted; do
  step pmcf_$L 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
  step pmcw_$L 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
done
step pmcsq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcsq_$TAG -o run -- python3 -u bench.py $B --layout unsorted
# the headline's dominant kernel (sorted Q1.1's aggregation): instruction mix, waits, L2 hits / misses
B1="--no-cpu-baseline --steps 5 --warmup 2 --layout sorted --queries Q1.1"
step pmcq11sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmcq11sq_$TAG -o run -- python3 -u bench.py $B1
step pmcq11tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcq11tcc_$TAG -o run -- python3 -u bench.py $B1
python3 tools/pmc_summary.py gpurun_out/pmcq11sq_$TAG > gpurun_out/pmcq11sq_$TAG.txt 2>&1 || true
python3 tools/pmc_summary.py gpurun_out/pmcq11tcc_$TAG > gpurun_out/pmcq11tcc_$TAG.txt 2>&1 || true
python3 tools/traffic.py --layout sorted gpurun_out/pmcf_${TAG}_sorted gpurun_out/pmcw_${TAG}_sorted \
  --layout unsorted gpurun_out/pmcf_${TAG}_unsorted gpurun_out/pmcw_${TAG}_unsorted \
  --queries Q1.1,Q1.2,Q1.3 --sf 100 -o gpurun_out/traffic_$TAG.json
python3 tools/pmc_summary.py gpurun_out/pmcsq_$TAG > gpurun_out/pmcsq_$TAG.txt 2>&1 || true
cat gpurun_out/steps.log
tail -2 gpurun_out/bench.log
