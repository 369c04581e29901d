#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 120 ./tools/stream_bench 2 > gpurun_out/r06r_stream_bench.log 2>&1 || { cat gpurun_out/r06r_stream_bench.log; exit 1; }
cat gpurun_out/r06r_stream_bench.log
