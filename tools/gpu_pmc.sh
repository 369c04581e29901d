#!/bin/bash
# PMC passes (one counter group per run, as MI355X_MICROARCH.md prescribes) over tools/explore.py.
# usage: tools/gpu_pmc.sh <tag> [explore args...]   -> gpurun_out/pmc_<tag>/
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
[ -f gpurun_out/counters.txt ] || timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/explore.py "$@" > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail $OUT/trace.log; exit 1; }
i=0
# passes: default groups, or PMC_PASSES="group1;group2;..." (counters of one group space-separated)
PASSES=${PMC_PASSES:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA;FETCH_SIZE;GRBM_GUI_ACTIVE GRBM_COUNT"}
IFS=';' read -ra PGROUPS <<< "$PASSES"
for ctr in "${PGROUPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc$i -o run -- python3 tools/explore.py "$@" > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($ctr) failed rc=$?"; exit 1; }
done
echo "pmc done"
