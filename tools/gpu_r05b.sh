#!/bin/bash
# full GPU suite, smoke, default bench, host breakdown of the C3 group-bys
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05h_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r05h_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05h_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r05h_bench.json 2> gpurun_out/r05h_bench.err || exit $?
PHIP_HOST_TRACE=1 timeout -k 10 300 python -u tools/host_gb_probe.py --layout sorted \
  --queries Q2.1,Q2.3,Q3.2,Q3.4,Q4.3,C5 --reps 20 > gpurun_out/r05h_gb_host.log 2> gpurun_out/r05h_gb_host.err || exit $?
