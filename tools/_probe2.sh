#!/bin/bash
set -u
mkdir -p gpurun_out
A="select count(*) from lineorder where LO_DISCOUNT between 1 and 3"
E="select count(*) from lineorder where D_YEAR = 1993 and LO_DISCOUNT between 1 and 3 and LO_QUANTITY < 25"
run() {  # tag, env..., -- explore args
  local tag=$1; shift
  local ev=(); while [ $# -gt 0 ] && [ "$1" != "--sf" ]; do ev+=("$1"); shift; done
  env "${ev[@]}" timeout -k 10 200 python -u tools/explore.py --reps 7 "$@" "$A" "$E" > gpurun_out/p2_$tag.log 2>&1 || { tail gpurun_out/p2_$tag.log; exit 1; }
  echo "== $tag"; grep query gpurun_out/p2_$tag.log | python3 -c "import sys,json; [print(d['query'][:50].ljust(50), d['scan_ms'], d['device_ms'], d['alg_GBps']) for d in map(json.loads, sys.stdin)]"
}
run base PHIP_X=1
run sf10 PHIP_X=1 --sf 10
run p1 PHIP_CONJ_P=1
run p2 PHIP_CONJ_P=2
run temporal PHIP_LIB=$PWD/pinot_amd/variants/lib_temporal.so
