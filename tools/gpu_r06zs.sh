#!/bin/bash
# round 6: the driver's N>1 shape rehearsed on one GPU -- bench.py --gpus 2 with its default segments per rank
# (125 per rank of an SF250 table, sorted layout: rank 1's dates lie past Q1.1's year), gloo between the ranks
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > gpurun_out/r06zs_n2_default.log 2>&1 || { tail -30 gpurun_out/r06zs_n2_default.log; exit 1; }
tail -1 gpurun_out/r06zs_n2_default.log | cut -c1-400
