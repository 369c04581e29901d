#!/bin/bash
# round 6: kernel trace of STARTREE_SUM_QUERY (C1)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r06zp -o run -- python3 -u tools/cfg_ab.py --configs c1 --queries STARTREE_SUM_QUERY --reps 4 --warmup 1 > gpurun_out/r06zp_st.log 2>&1 || { tail -20 gpurun_out/r06zp_st.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_r06zp/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms  n={r["Calls"]:>5}  avg {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
