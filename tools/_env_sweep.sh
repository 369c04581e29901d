#!/bin/bash
# A/B an environment knob of libpinot_hip on the SSB SF100 explore set (measurement aid).
# usage: VAR=PHIP_FILTER_WALK VALS="xcd contig" bash tools/_env_sweep.sh [explore queries...]
set -u
mkdir -p gpurun_out
if [ $# -gt 0 ]; then Q=("$@"); else Q=("select count(*) from lineorder where LO_DISCOUNT between 1 and 3" "select count(*) from lineorder where D_YEAR = 1993 and LO_DISCOUNT between 1 and 3 and LO_QUANTITY < 25" Q1.1 Q1.2 Q1.3); fi
for v in $VALS; do
  echo "== $VAR=$v"
  env "$VAR=$v" timeout -k 10 200 python -u tools/explore.py --reps 7 "${Q[@]}" > "gpurun_out/sweep_$v.log" 2>&1 || { echo fail; tail "gpurun_out/sweep_$v.log"; exit 1; }
  grep query "gpurun_out/sweep_$v.log" | python3 -c "import sys,json; [print(d['query'][:48], d['scan_ms'], d['alg_GBps']) for d in map(json.loads, sys.stdin)]"
done
