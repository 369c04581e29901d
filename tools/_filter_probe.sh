#!/bin/bash
# Filter-kernel probe (measurement aid): width sweep, ring-depth (workgroups per CU) sweep, SQ counters.
set -u
mkdir -p gpurun_out
A="select count(*) from lineorder where LO_DISCOUNT between 1 and 3"
B="select count(*) from lineorder where LO_QUANTITY between 10 and 30"
C="select count(*) from lineorder where LO_SUPPLYCOST between 1000 and 50000"
D="select count(*) from lineorder where LO_EXTENDEDPRICE between 100000 and 2000000"
E="select count(*) from lineorder where D_YEAR = 1993 and LO_DISCOUNT between 1 and 3 and LO_QUANTITY < 25"
echo "== widths (default)"
timeout -k 10 200 python -u tools/explore.py --reps 7 "$A" "$B" "$C" "$D" "$E" > gpurun_out/probe_w.log 2>&1 || { tail gpurun_out/probe_w.log; exit 1; }
grep query gpurun_out/probe_w.log
for bpc in 1 2 3 4 5 6 8; do
  echo "== PHIP_FILTER_BPC=$bpc"
  PHIP_FILTER_BPC=$bpc timeout -k 10 200 python -u tools/explore.py --reps 7 "$A" "$E" > gpurun_out/probe_b$bpc.log 2>&1 || { tail gpurun_out/probe_b$bpc.log; exit 1; }
  grep query gpurun_out/probe_b$bpc.log
done
for q in A E; do
  PMC_PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM;GRBM_GUI_ACTIVE GRBM_COUNT" \
    bash tools/gpu_pmc.sh probe$q --reps 3 "${!q}" || exit 1
  echo "== PMC $q"
  python3 tools/pmc_summary.py gpurun_out/pmc_probe$q filter_kernel 2>&1 | tee gpurun_out/pmc_probe$q/summary.txt
done
