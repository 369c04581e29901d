#!/bin/bash
# configs C1/C3/C4/C5 measurement (tools/configs_bench.py), one step per config
set -u
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
for c in C1 C4 C3 C5; do
  timeout -k 10 400 python -u tools/configs_bench.py --configs $c >> gpurun_out/configs.jsonl 2> gpurun_out/configs_$c.err || { echo "config $c failed"; tail -20 gpurun_out/configs_$c.err; exit 1; }
  echo "$c done $(date +%T)"
done
