#!/bin/bash
# Host-path A/B on the headline step: tools/host_probe.py (per-query wall / execute / decode / device / kernel ms) and
# the PHIP_HOST_TRACE phases, once per "NAME=VALUE ..." setting. usage: tools/host_ab.sh <tag> "" "PHIP_X=1" ...
set -u
TAG=$1; shift
mkdir -p gpurun_out
for cfg in "$@"; do
  echo "== ${cfg:-default}" >> gpurun_out/host_ab_$TAG.log
  env $cfg PHIP_HOST_TRACE=1 timeout -k 10 300 python -u tools/host_probe.py --reps 100 > gpurun_out/host_ab_tmp.log 2> gpurun_out/host_ab_tmp.err || { tail -20 gpurun_out/host_ab_tmp.err; exit 1; }
  cat gpurun_out/host_ab_tmp.log >> gpurun_out/host_ab_$TAG.log
  python3 - >> gpurun_out/host_ab_$TAG.log <<'PY'
import numpy as np
rows = [l.split() for l in open("gpurun_out/host_ab_tmp.err") if l.startswith("phip_host_trace")]
vals = np.array([[float(r[i]) for i in (2, 4, 6, 8, 10, 12)] for r in rows])[-300:]
for qi, q in enumerate(("Q1.1", "Q1.2", "Q1.3")):
    m = np.median(vals[qi::3], axis=0)
    print(q, "us: lane %.1f enqueue %.1f sync %.1f result %.1f total %.1f device %.1f" % tuple(m))
PY
done
cat gpurun_out/host_ab_$TAG.log
