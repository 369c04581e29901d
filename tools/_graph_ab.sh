set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for g in graph nograph; do
  if [ $g = nograph ]; then export PHIP_NO_GRAPH=1; fi
  timeout -k 10 200 python -u tools/explore.py --reps 9 Q1.1 Q1.2 Q1.3 > gpurun_out/ex_$g.log 2>&1 || { tail gpurun_out/ex_$g.log; exit 1; }
  echo "== $g"; grep query gpurun_out/ex_$g.log
done
