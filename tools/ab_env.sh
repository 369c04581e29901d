#!/bin/bash
# A/B of library settings inside one GPU call (boxes differ by ~8 %): runs bench.py once per "NAME=VALUE ..."
# argument set, recording the JSON lines. usage: tools/ab_env.sh <tag> "PHIP_FUSE=0" "PHIP_FUSE=1" ...
set -u
TAG=$1; shift
mkdir -p gpurun_out
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/ab_$TAG.log
  env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/ab_tmp.log 2>&1 || { tail -20 gpurun_out/ab_tmp.log; exit 1; }
  tail -1 gpurun_out/ab_tmp.log >> gpurun_out/ab_$TAG.log
done
python3 - "$TAG" <<'PY'
import json, sys
tag = sys.argv[1]
cfg = None
for line in open(f"gpurun_out/ab_{tag}.log"):
    if line.startswith("== "):
        cfg = line[3:].strip(); continue
    try:
        j = json.loads(line)
    except Exception:
        continue
    u = j.get("unsorted_layout", {})
    def k(r):
        ks = r["roofline"]["kernels"]
        return {n: v["per_query_ms"] for n, v in ks.items()}
    print(f"{cfg:40s} sorted {j['value']:8.1f} ms/step {j['ms_per_step']:.3f} p50 {j['p50_latency_ms']} kern {k(j)}")
    if u:
        print(f"{'':40s} unsorted {u['value']:8.1f} ms/step {u['ms_per_step']:.3f} p50 {u['p50_latency_ms']} kern {k(u)}")
PY
