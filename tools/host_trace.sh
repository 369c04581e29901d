#!/bin/bash
# host phases of phip_plan_execute on the headline step (PHIP_HOST_TRACE=1): lane acquire, enqueue (launches +
# event records), stream sync, result assembly -- medians per query over tools/host_probe.py's reps
set -u
mkdir -p gpurun_out
PHIP_HOST_TRACE=1 timeout -k 10 300 python -u tools/host_probe.py --reps 50 > gpurun_out/host_probe_t.log 2> gpurun_out/host_trace.err || { tail -20 gpurun_out/host_trace.err; exit 1; }
cat gpurun_out/host_probe_t.log
python3 - <<'PY'
import numpy as np
rows = [l.split() for l in open("gpurun_out/host_trace.err") if l.startswith("phip_host_trace")]
vals = np.array([[float(r[i]) for i in (2, 4, 6, 8, 10, 12)] for r in rows])
vals = vals[-150:]  # the 50 timed reps x 3 queries
for qi, q in enumerate(("Q1.1", "Q1.2", "Q1.3")):
    m = np.median(vals[qi::3], axis=0)
    print(q, "us: lane %.1f enqueue %.1f sync %.1f result %.1f total %.1f device %.1f" % tuple(m))
PY
