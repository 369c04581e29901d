#!/bin/bash
# SQ counter passes over one bench configuration (one rocprofv3 --pmc run per pass, each under its own time
# limit); summaries via tools/pmc_summary.py. usage: tools/sq_passes.sh <tag> [bench args...]
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
B="--no-cpu-baseline --steps 5 --warmup 2 $*"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq_${TAG}_$i -o run -- python3 -u bench.py $B > gpurun_out/sq_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_${TAG}_$i.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/sq_${TAG}_$i > gpurun_out/sq_${TAG}_$i.txt 2>&1 || true
done
grep -A9 "filter_kernel" gpurun_out/sq_${TAG}_1.txt gpurun_out/sq_${TAG}_2.txt | head -40
