#!/bin/bash
# One GPU call: kernel-time decomposition of the SSB queries (tools/explore.py); optional gpu tests first.
# usage: tools/gpu_explore.sh [--tests] [explore args...]
set -u
mkdir -p gpurun_out
if [ "${1:-}" = "--tests" ]; then
  shift
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
timeout -k 10 500 python -u tools/explore.py "$@" > gpurun_out/explore.log 2>&1
rc=$?
cat gpurun_out/explore.log | grep -v amdgpu.ids
exit $rc
