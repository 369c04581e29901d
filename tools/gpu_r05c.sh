#!/bin/bash
# SQ wave-state breakdown of the sorted Q1.1 kernels: fused (default) and split (PHIP_FUSE=0)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
timeout -s KILL 240 rocprofv3 --pmc $SQ -d gpurun_out/r05i_sq_fused -o run -- python3 tools/ssb_probe.py --queries Q1.1 --layout sorted --reps 10 > gpurun_out/r05i_sq_fused.log 2>&1 || exit $?
PHIP_FUSE=0 timeout -s KILL 240 rocprofv3 --pmc $SQ -d gpurun_out/r05i_sq_split -o run -- python3 tools/ssb_probe.py --queries Q1.1 --layout sorted --reps 10 > gpurun_out/r05i_sq_split.log 2>&1 || exit $?
