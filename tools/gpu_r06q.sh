#!/bin/bash
# round 6: the N = 2 rehearsal again (bench.py --gpus 2 spawning its ranks) and the read ceilings of the filter's DMA
# shapes (tools/stream_bench: plain / non-temporal / one-region DMA / multi-column DMA)
mkdir -p gpurun_out
timeout -k 10 120 ./tools/stream_bench 2 > gpurun_out/r06q_stream_bench.log 2>&1 || { cat gpurun_out/r06q_stream_bench.log; exit 1; }
cat gpurun_out/r06q_stream_bench.log
bash tools/gpu_round6.sh n2 r06q
