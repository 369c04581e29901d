#!/bin/bash
# packed doc-order values: parity, then A/B on the headline (both layouts) and the group-by configs
set -u
mkdir -p gpurun_out
bash tools/gpu_t.sh tests/test_gpu_materialize.py tests/test_gpu_fused.py tests/test_gpu_parity.py || exit 1
cp gpurun_out/pytest_t.log gpurun_out/r05zd_pytest.log
BENCH_ARGS="--layout both" bash tools/ab_env.sh r05zd "PHIP_VPACK=0" "PHIP_STREAM_PACKED=0" "PHIP_VPACK=1" || exit 1
timeout -k 10 400 python -u tools/gb_ab.py --queries C5,Q2.1,Q3.1,Q4.1 --set PHIP_VPACK=0 --set "" > gpurun_out/r05zd_gb_ab.log 2>&1 || { tail -20 gpurun_out/r05zd_gb_ab.log; exit 1; }
cat gpurun_out/r05zd_gb_ab.log
