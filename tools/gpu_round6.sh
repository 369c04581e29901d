#!/bin/bash
# Round-6 evidence, one GPU call per mode (each inside gpurun's 20-minute limit; every step under its own time limit,
# stopping at the first failure -- never retried):
#   tools/gpu_round6.sh tests <tag>   GPU tests, smoke, bench (both layouts, C3 / C5 legs, CPU baselines, parity),
#                                     the N = 2 rehearsal (bench.py --gpus 2 starts its own ranks, gloo, one GPU)
#   tools/gpu_round6.sh bench <tag>   bench only
#   tools/gpu_round6.sh trace <tag>   rocprofv3 kernel traces with the concurrent-client leg off (every launch
#                                     sequential): the headline per layout, the group-by queries (gb_ab.py with idle
#                                     gaps between queries); per-query averages + recomputed frac (trace_summary.py)
#   tools/gpu_round6.sh traffic <tag> PMC FETCH / WRITE per layout + the stream-only calibration -> traffic json;
#                                     touched 64-B lines -> touched json
#   tools/gpu_round6.sh gbpmc <tag>   SQ / TCC / FETCH / WRITE passes of the group-by aggregation kernels (C5, Q3.1,
#                                     Q2.1; the bench's sorted layout) and the headline's fused kernel (sorted Q1.1)
set -u
MODE=$1; TAG=$2; shift 2
mkdir -p gpurun_out
: > gpurun_out/steps_${TAG}_$MODE.log
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$name] start $(date +%T)" >> gpurun_out/steps_${TAG}_$MODE.log
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(date +%T)" >> gpurun_out/steps_${TAG}_$MODE.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -30 "gpurun_out/${TAG}_$name.log"; exit $rc; fi
}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
GBQ=Q2.1,Q2.2,Q2.3,Q3.1,Q3.2,Q3.3,Q3.4,Q4.1,Q4.2,Q4.3,C5
case "$MODE" in
tests)
  step pytest_gpu 780 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
  step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
  step bench 420 python -u bench.py --steps 20 --warmup 5
  step n2 300 python -u bench.py --gpus 2 --dist-backend gloo --segs-per-gpu 8 --steps 5 --warmup 2 --layout sorted
  tail -3 gpurun_out/${TAG}_pytest_gpu.log
  tail -c 600 gpurun_out/${TAG}_bench.log
  ;;
bench)
  step bench 420 python -u bench.py --steps 20 --warmup 5
  tail -c 600 gpurun_out/${TAG}_bench.log
  ;;
n2)
  step n2 300 python -u bench.py --gpus 2 --dist-backend gloo --segs-per-gpu 8 --steps 5 --warmup 2 --layout sorted
  tail -c 1500 gpurun_out/${TAG}_n2.log
  ;;
trace)
  B="--no-cpu-baseline --no-parity --no-concurrent --group-by= --configs= --steps 10 --warmup 3"
  for L in sorted unsorted; do
    step trace_$L 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
    python3 tools/trace_summary.py cycle gpurun_out/prof_${TAG}_$L/run_kernel_trace.csv --queries Q1.1,Q1.2,Q1.3 \
      --family fused_filter_agg --bench gpurun_out/${TAG}_trace_$L.log --layout $L -o gpurun_out/trace_${TAG}_$L.json \
      > /dev/null 2> gpurun_out/trace_${TAG}_$L.err || cat gpurun_out/trace_${TAG}_$L.err
  done
  step trace_gb 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_gb -o run -- python3 -u tools/gb_ab.py --queries $GBQ --layout sorted --reps 10 --warmup 3 --gap 0.25
  python3 tools/trace_summary.py gaps gpurun_out/prof_${TAG}_gb/run_kernel_trace.csv --gb-ab gpurun_out/${TAG}_trace_gb.log \
    -o gpurun_out/trace_${TAG}_gb.json > /dev/null 2> gpurun_out/trace_${TAG}_gb.err || cat gpurun_out/trace_${TAG}_gb.err
  ;;
traffic)
  B="--no-cpu-baseline --no-parity --no-concurrent --group-by= --configs= --steps 10 --warmup 3"
  for L in sorted unsorted; do
    step pmcf_$L 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
    step pmcw_$L 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_${TAG}_$L -o run -- python3 -u bench.py $B --layout $L
  done
  export PHIP_FILTER_PROBE=1 PHIP_FUSE=0
  step calib_bench 200 python3 -u bench.py $B --layout unsorted
  step pmcf_calib 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_${TAG}_calib -o run -- python3 -u bench.py $B --layout unsorted
  unset PHIP_FILTER_PROBE PHIP_FUSE
  python3 tools/traffic.py --layout sorted gpurun_out/pmcf_${TAG}_sorted gpurun_out/pmcw_${TAG}_sorted \
    --layout unsorted gpurun_out/pmcf_${TAG}_unsorted gpurun_out/pmcw_${TAG}_unsorted \
    --calib gpurun_out/pmcf_${TAG}_calib gpurun_out/${TAG}_calib_bench.log \
    --queries Q1.1,Q1.2,Q1.3 --sf 100 -o gpurun_out/traffic_$TAG.json > gpurun_out/${TAG}_traffic.log 2>&1 || { cat gpurun_out/${TAG}_traffic.log; exit 1; }
  step touched 240 python3 -u tools/touched_lines.py --layout sorted --layout unsorted -o gpurun_out/touched_$TAG.json
  ;;
gbpmc)
  SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  G="--layout sorted --reps 5 --warmup 2"
  for Q in ${GBPMC_QUERIES:-C5 Q3.1 Q2.1}; do
    step gbsq_$Q 200 timeout -s KILL 180 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/gbsq_${TAG}_$Q -o run -- python3 -u tools/gb_ab.py --queries $Q $G
    step gbtcc_$Q 200 timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/gbtcc_${TAG}_$Q -o run -- python3 -u tools/gb_ab.py --queries $Q $G
    step gbfetch_$Q 200 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/gbfetch_${TAG}_$Q -o run -- python3 -u tools/gb_ab.py --queries $Q $G
    step gbwrite_$Q 200 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/gbwrite_${TAG}_$Q -o run -- python3 -u tools/gb_ab.py --queries $Q $G
  done
  B1="--no-cpu-baseline --no-parity --no-concurrent --group-by= --configs= --steps 5 --warmup 2 --layout sorted --queries Q1.1"
  step q11sq 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/q11sq_$TAG -o run -- python3 -u bench.py $B1
  for x in gpurun_out/gbsq_${TAG}_* gpurun_out/gbtcc_${TAG}_* gpurun_out/gbfetch_${TAG}_* gpurun_out/gbwrite_${TAG}_* gpurun_out/q11sq_$TAG; do
    [ -d "$x" ] && python3 tools/pmc_summary.py "$x" > "$x.txt" 2>&1
  done
  ;;
*) echo "unknown mode $MODE"; exit 2;;
esac
cat gpurun_out/steps_${TAG}_$MODE.log
