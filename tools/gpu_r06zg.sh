#!/bin/bash
# round 6: does HBM that the queries never touch slow Q3.1's gathers? (1 GiB allocations beside the segments)
mkdir -p gpurun_out
: > gpurun_out/r06zg_hog.log
for g in 0 10 30 0 10; do
  echo "== hog $g GiB" >> gpurun_out/r06zg_hog.log
  timeout -k 10 300 python -u tools/gb_ab.py --queries Q3.1,Q2.1 --layout sorted --reps 15 --warmup 3 --hog-gib $g >> gpurun_out/r06zg_hog.log 2>&1 || { tail -5 gpurun_out/r06zg_hog.log; exit 1; }
done
grep -E "^==|query" gpurun_out/r06zg_hog.log | cut -c1-110
