#!/bin/bash
# A/B of two library builds on configs (default C4 + C3) in one GPU call (measurement aid)
set -u
mkdir -p gpurun_out
CFGS=${CFGS:-C4,C3}
for lib in ab/libpinot_hip_base.so pinot_amd/libpinot_hip.so ab/libpinot_hip_base.so pinot_amd/libpinot_hip.so; do
  PHIP_LIB=$PWD/$lib timeout -k 10 300 python -u tools/configs_bench.py --configs $CFGS --no-cpu --reps 9 --warmup 3 > gpurun_out/cfg_ab.jsonl 2> gpurun_out/cfg_ab.err || { tail -30 gpurun_out/cfg_ab.err; exit 1; }
  echo "== $lib"; python3 -c "import sys,json; [print(d['config'], d['query'][:24].ljust(24), d['kernel_ms'], d['p50_ms']) for d in map(json.loads, open('gpurun_out/cfg_ab.jsonl'))]"
done
