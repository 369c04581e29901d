#!/bin/bash
# round 6: where C5's aggregation time goes -- the query with one part at a time (keys + COUNT, + the value expression,
# + the HLL, no group-by), each under both group-by walks
mkdir -p gpurun_out
W="from lineorder where C_REGION = 'AMERICA' and S_REGION = 'AMERICA'"
timeout -k 10 400 python -u tools/gb_ab.py --layout sorted --reps 15 --warmup 3 \
  --sql "C5cnt::select D_YEAR, C_NATION, count(*) $W group by D_YEAR, C_NATION limit 100000" \
  --sql "C5y::select D_YEAR, count(*) $W group by D_YEAR limit 100000" \
  --sql "C5rev::select D_YEAR, C_NATION, sum(LO_REVENUE) $W group by D_YEAR, C_NATION limit 100000" \
  --sql "C5sum::select D_YEAR, C_NATION, sum(LO_REVENUE - LO_SUPPLYCOST) $W group by D_YEAR, C_NATION limit 100000" \
  --sql "C5hll::select D_YEAR, C_NATION, DISTINCTCOUNTHLL(LO_CUSTKEY) $W group by D_YEAR, C_NATION limit 100000" \
  --sql "C5flat::select count(*), sum(LO_REVENUE - LO_SUPPLYCOST), DISTINCTCOUNTHLL(LO_CUSTKEY) $W" \
  --queries C5,C5cnt,C5y,C5rev,C5sum,C5hll,C5flat --set "" --set "PHIP_GB_BATCH=1" --set "PHIP_GB_BATCH=0" > gpurun_out/r06n_c5_parts.log 2>&1 || { tail -5 gpurun_out/r06n_c5_parts.log; exit 1; }
grep -v loaded_segments gpurun_out/r06n_c5_parts.log | cut -c1-120
