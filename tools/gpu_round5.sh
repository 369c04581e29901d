#!/bin/bash
# Round-5 evidence in two GPU calls (each inside gpurun's 20-minute limit; every step under its own time limit,
# stopping at the first failure -- never retried):
#   tools/gpu_round5.sh tests <tag>   GPU tests, smoke, bench (both layouts, C3 / C5 legs, CPU baselines, parity)
#   tools/gpu_round5.sh prof <tag>    rocprof kernel trace of the bench per layout, PMC FETCH / WRITE per layout, the
#                                     stream-only calibration pass, touched 64-B lines (-> traffic / touched json for
#                                     bench's roofline.traffic), SQ counters of the headline fused kernel and of the
#                                     fused group-by (Q3.2)
set -u
MODE=$1; TAG=$2; shift 2
mkdir -p gpurun_out
: > gpurun_out/steps_$MODE.log
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$name] start $(date +%T)" >> gpurun_out/steps_$MODE.log
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(date +%T)" >> gpurun_out/steps_$MODE.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -30 "gpurun_out/${TAG}_$name.log"; exit $rc; fi
}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ "$MODE" = tests ]; then
  step pytest_gpu 780 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
  step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
  step bench 400 python -u bench.py --steps 20 --warmup 5
  tail -3 gpurun_out/${TAG}_pytest_gpu.log
  tail -c 600 gpurun_out/${TAG}_bench.log
  exit 0
fi
B="--no-cpu-baseline --no-parity --group-by= --steps 10 --warmup 3"
for L in sorted unsorted; do
  step rocprof_$L 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
done
for L in sorted unsorted; do
  step pmcf_$L 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
  step pmcw_$L 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
done
# stream-only calibration: the plain filter kernel with the evaluation skipped streams exactly its staged bytes
export PHIP_FILTER_PROBE=1 PHIP_FUSE=0
step calib_bench 200 python3 -u bench.py $B --layout unsorted
step pmcf_calib 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_${TAG}_calib -o run -- python3 -u bench.py $B --layout unsorted
unset PHIP_FILTER_PROBE PHIP_FUSE
python3 tools/traffic.py --layout sorted gpurun_out/pmcf_${TAG}_sorted gpurun_out/pmcw_${TAG}_sorted \
  --layout unsorted gpurun_out/pmcf_${TAG}_unsorted gpurun_out/pmcw_${TAG}_unsorted \
  --calib gpurun_out/pmcf_${TAG}_calib gpurun_out/${TAG}_calib_bench.log \
  --queries Q1.1,Q1.2,Q1.3 --sf 100 -o gpurun_out/traffic_$TAG.json > gpurun_out/${TAG}_traffic.log 2>&1 || { cat gpurun_out/${TAG}_traffic.log; exit 1; }
step touched 240 python3 -u tools/touched_lines.py --layout sorted --layout unsorted -o gpurun_out/touched_$TAG.json
B1="--no-cpu-baseline --no-parity --group-by= --steps 5 --warmup 2 --layout sorted --queries Q1.1"
step pmcq11sq 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmcq11sq_$TAG -o run -- python3 -u bench.py $B1
step pmcq11tcc 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcq11tcc_$TAG -o run -- python3 -u bench.py $B1
step gbsq_Q3.2 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/gbsq_${TAG}_Q3.2 -o run -- python3 -u tools/gb_ab.py --queries Q3.2 --reps 5 --warmup 2
for d in pmcq11sq pmcq11tcc gbsq; do
  for x in gpurun_out/${d}_${TAG}*; do [ -d "$x" ] && python3 tools/pmc_summary.py "$x" > "$x.txt" 2>&1; done
done
cat gpurun_out/steps_$MODE.log
