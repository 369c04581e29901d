#!/bin/bash
# SQ wave-state counters of the filter / aggregation kernels for the given SSB queries (one pass each), summaries only.
# usage: QUERIES=Q3.2,Q2.1 LAYOUT=sorted tools/gpu_sq.sh <tag>
set -u
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
for q in $(echo ${QUERIES:-Q3.2} | tr ',' ' '); do
  timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-include-regex "filter_kernel|agg_kernel|slab_reduce|group_" -d /tmp/sq_${TAG}_$q \
    -o run --output-format csv -- python3 tools/ssb_probe.py --queries $q --layout ${LAYOUT:-sorted} --reps 10 \
    > gpurun_out/sq_${TAG}_$q.log 2>&1 || exit $?
  python3 tools/pmc_summary.py /tmp/sq_${TAG}_$q "phip::" > gpurun_out/sq_${TAG}_$q.txt 2>&1 || exit $?
done
