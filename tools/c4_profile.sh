#!/bin/bash
# C4 (inverted-index-heavy) measurement in one GPU call: p50 per selectivity, rocprof kernel stats, two SQ
# counter passes. Stops at the first failure. usage: tools/c4_profile.sh <tag>
set -u
TAG=${1:-c4}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
A="--configs C4 --no-cpu --c4-distinct 4 --c4-copies 25"
timeout -k 10 300 python -u tools/configs_bench.py $A --reps 10 --warmup 3 > gpurun_out/${TAG}.jsonl 2>&1 || { tail -20 gpurun_out/${TAG}.jsonl; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u tools/configs_bench.py $A --reps 3 --warmup 1 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_sq$i -o run -- python3 -u tools/configs_bench.py $A --reps 2 --warmup 1 > gpurun_out/${TAG}_sq$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_sq$i.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/${TAG}_sq$i > gpurun_out/${TAG}_sq$i.txt 2>&1 || true
done
cut -c1-240 gpurun_out/${TAG}.jsonl | grep C4
grep -A9 "filter_kernel\|roaring" gpurun_out/${TAG}_sq1.txt gpurun_out/${TAG}_sq2.txt | head -60
