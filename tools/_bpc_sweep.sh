set -u
mkdir -p gpurun_out
Q='"select count(*) from lineorder where LO_DISCOUNT between 1 and 3" "select count(*) from lineorder where D_YEAR = 1993 and LO_DISCOUNT between 1 and 3 and LO_QUANTITY < 25" Q1.1 Q1.2 Q1.3'
for b in ${BPCS:-4 5 8}; do
  echo "== BPC $b"
  eval PHIP_FILTER_BPC=$b timeout -k 10 200 python -u tools/explore.py --reps 5 $Q > gpurun_out/ex_bpc$b.log 2>&1 || { echo fail; tail gpurun_out/ex_bpc$b.log; exit 1; }
  grep query gpurun_out/ex_bpc$b.log | python3 -c "import sys,json; [print(d['query'][:40], d['scan_ms'], d['alg_GBps']) for d in map(json.loads, sys.stdin)]"
done
