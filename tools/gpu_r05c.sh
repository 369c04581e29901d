#!/bin/bash
# SQ wave-state breakdown of the sorted Q1.1 kernels: fused (default) and split (PHIP_FUSE=0); summaries only
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
for arm in fused split; do
  envv=""; [ $arm = split ] && envv="PHIP_FUSE=0"
  env $envv true
  if [ $arm = split ]; then export PHIP_FUSE=0; fi
  timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-include-regex "filter_kernel|agg_kernel" -d /tmp/r05i_$arm -o run --output-format csv -- \
    python3 tools/ssb_probe.py --queries ${Q:-Q1.1} --layout sorted --reps 10 > gpurun_out/r05i_sq_$arm.log 2>&1 || exit $?
  python3 tools/pmc_summary.py /tmp/r05i_$arm "kernel<" > gpurun_out/r05i_sq_$arm.txt 2>&1 || exit $?
done
