#!/bin/bash
# round 6: which group-by walk each C5 execution takes (PHIP_WALK_TRACE), default against forced batched
mkdir -p gpurun_out
PHIP_WALK_TRACE=1 timeout -k 10 300 python -u tools/gb_ab.py --queries C5,Q4.1 --layout sorted --reps 6 --warmup 2 --set "" --set "PHIP_GB_BATCH=1" > gpurun_out/r06zf_walk.log 2>&1 || { tail -5 gpurun_out/r06zf_walk.log; exit 1; }
grep -v loaded_segments gpurun_out/r06zf_walk.log | cut -c1-160
