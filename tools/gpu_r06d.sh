mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "c4 or c1 or ssb_vs_oracle" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06d_pytest.log 2>&1 || { tail -30 gpurun_out/r06d_pytest.log; exit 1; }
tail -2 gpurun_out/r06d_pytest.log
timeout -k 10 300 python -u tools/cfg_ab.py --configs c4 --set "" --set "PHIP_AGG_LDS_DICT_MAX=1024" --reps 10 --warmup 3 > gpurun_out/r06d_c4_ab.log 2>&1 || { tail -5 gpurun_out/r06d_c4_ab.log; exit 1; }
timeout -k 10 300 python -u tools/cfg_ab.py --configs c1 --set "" --set "PHIP_FUSED_SMALL=0" --set "PHIP_FUSE=0" --set "PHIP_FUSED_SMALL=0 PHIP_FILTER_BPC=8" --reps 10 --warmup 3 > gpurun_out/r06d_c1_ab.log 2>&1 || { tail -5 gpurun_out/r06d_c1_ab.log; exit 1; }
cat gpurun_out/r06d_c4_ab.log | cut -c1-220
