#!/bin/bash
# round 3: fusion policy with the value ids gathered (not streamed) and the fused kernel at 6 workgroups per CU
set -u
mkdir -p gpurun_out
bash tools/ab_env.sh ${TAG:-ab5} "PHIP_X=1" "PHIP_FUSE=1 PHIP_STREAM_VALUES=0 PHIP_FILTER_BPC=6" \
  "PHIP_FUSE=1 PHIP_STREAM_VALUES=0 PHIP_FILTER_BPC=8" "PHIP_STREAM_VALUES=0 PHIP_FILTER_BPC=6" "PHIP_X=2" || exit 1
