#!/bin/bash
# round 6: many medium allocations (records-like: 48 MiB each) vs few large ones beside the segments, Q3.1 after them
mkdir -p gpurun_out
: > gpurun_out/r06zh_hog.log
for c in 48 1024 48 8; do
  echo "== hog 10 GiB in $c MiB allocations" >> gpurun_out/r06zh_hog.log
  timeout -k 10 300 python -u tools/gb_ab.py --queries Q3.1 --layout sorted --reps 15 --warmup 3 --hog-gib 10 --hog-chunk-mib $c >> gpurun_out/r06zh_hog.log 2>&1 || { tail -5 gpurun_out/r06zh_hog.log; exit 1; }
done
echo "== records of Q4.1 only, then Q3.1" >> gpurun_out/r06zh_hog.log
timeout -k 10 300 python -u tools/gb_ab.py --queries Q4.1,Q3.1 --layout sorted --reps 15 --warmup 3 >> gpurun_out/r06zh_hog.log 2>&1 || { tail -5 gpurun_out/r06zh_hog.log; exit 1; }
grep -E "^==|query" gpurun_out/r06zh_hog.log | cut -c1-110
