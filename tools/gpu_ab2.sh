#!/bin/bash
# round 3: GPU parity suite, bench A/B of the aggregation / fusion variants, and PMC passes on sorted Q1.1's
# aggregation (SQ stall / instruction mix, L2 hit rate)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --segs-per-gpu 6 --dist-backend gloo > gpurun_out/bench_n2_gloo.log 2>&1 || { tail -30 gpurun_out/bench_n2_gloo.log; exit 1; }
tail -1 gpurun_out/bench_n2_gloo.log
bash tools/ab_env.sh ${TAG:-ab2} "PHIP_X=1" "PHIP_FUSE_PER_TILE=0" "PHIP_FUSED_DEFER=0" "PHIP_FUSE=1" \
  "PHIP_FUSE=0 PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=1" "PHIP_FUSE=0 PHIP_DENSE_BATCH=1 PHIP_DENSE_MIN=128" || exit 1
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
B="--no-cpu-baseline --steps 5 --warmup 2 --layout sorted --queries Q1.1"
PHIP_FUSE=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_q11_sq -o run -- python3 -u bench.py $B > gpurun_out/pmc_q11_sq.log 2>&1 || exit 1
PHIP_FUSE=0 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_q11_tcc -o run -- python3 -u bench.py $B > gpurun_out/pmc_q11_tcc.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_q11_sq > gpurun_out/pmc_q11_sq.txt 2>&1 || true
python3 tools/pmc_summary.py gpurun_out/pmc_q11_tcc > gpurun_out/pmc_q11_tcc.txt 2>&1 || true
