#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_profile.py > gpurun_out/r06zn_host_profile.log 2>&1 || { tail -20 gpurun_out/r06zn_host_profile.log; exit 1; }
head -60 gpurun_out/r06zn_host_profile.log
