#!/bin/bash
# round 6: group-by records with the per-device budget -- A/B against the columns' layouts and both walks, then the bench
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/gb_ab.py --layout sorted --reps 15 --warmup 3 --set "" --set "PHIP_GB_RECORD=0" --set "PHIP_GB_BATCH=0" --set "PHIP_GB_BATCH=1" > gpurun_out/r06w_rec_ab.log 2>&1 || { tail -5 gpurun_out/r06w_rec_ab.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r06w_bench.log 2>&1 || { tail -20 gpurun_out/r06w_bench.log; exit 1; }
tail -1 gpurun_out/r06w_bench.log | cut -c1-300
