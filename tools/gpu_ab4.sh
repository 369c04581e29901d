#!/bin/bash
# round 3: finalize folded into the last workgroup (parity suite, then A/B vs the separate launch), and sorted
# Q1.1's aggregation walk variants (staged dense-tile walk vs the per-doc ring walk, fused)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh ${TAG:-ab4f} "PHIP_X=1" "PHIP_FOLD_FINAL=0" "PHIP_X=2" "PHIP_FOLD_FINAL=0 PHIP_X=2" || exit 1
BENCH_ARGS="--layout sorted --queries Q1.1" bash tools/ab_env.sh ${TAG:-ab4} "PHIP_X=1" \
  "PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=1" "PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=128" \
  "PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=1 PHIP_AGG_STAGE=0" "PHIP_FUSE=1" || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="--no-cpu-baseline --steps 5 --warmup 2 --layout sorted --queries Q1.1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_q11_sq -o run -- python3 -u bench.py $B > gpurun_out/pmc_q11_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_q11_tcc -o run -- python3 -u bench.py $B > gpurun_out/pmc_q11_tcc.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_q11_sq > gpurun_out/pmc_q11_sq.txt 2>&1 || true
python3 tools/pmc_summary.py gpurun_out/pmc_q11_tcc > gpurun_out/pmc_q11_tcc.txt 2>&1 || true
