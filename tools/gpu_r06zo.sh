#!/bin/bash
# round 6: where STARTREE_SUM_QUERY's 3.4 ms go (C1: 10M groups, one per doc) -- host phases per execution
mkdir -p gpurun_out
PHIP_HOST_TRACE=1 timeout -k 10 300 python -u tools/cfg_ab.py --configs c1 --queries STARTREE_SUM_QUERY,GROUP_BY_LOW_CARD --reps 6 --warmup 2 > gpurun_out/r06zo_st.log 2>&1 || { tail -20 gpurun_out/r06zo_st.log; exit 1; }
grep -v "^phip_host_trace" gpurun_out/r06zo_st.log | cut -c1-200
grep "^phip_host_trace" gpurun_out/r06zo_st.log | tail -12
