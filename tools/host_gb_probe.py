"""Host-side breakdown of SSB group-by queries (SF100, unsorted): per query the p50 of the library call
(GpuCombineOperator.run_raw: enqueue + device + the library's result assembly) and of the Python decode
(_block_from_result), beside the kernels' HIP-event times. PHIP_HOST_TRACE=1 adds the library's own phases.

    python tools/host_gb_probe.py --queries Q2.1,Q3.1,C5 [--reps 20]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", default="Q2.1,Q3.1,C5")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--layout", default="unsorted")
    args = ap.parse_args()
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuCombineOperator, GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    queries = args.queries.split(",")
    cols = ssb.columns_for(queries)
    gsegs = []
    for i in range(0, 100, 10):
        for r in ssb.make_segments(100, cols, seed=42, segments=range(i, i + 10), layout=args.layout):
            gsegs.append(GpuSegment(r))
    for q in queries:
        qc = parse(ssb.SSB_QUERIES[q])
        op = GpuInstancePlanMaker().make_instance_plan(qc, gsegs)
        inner = op
        while not isinstance(inner, GpuCombineOperator) and hasattr(inner, "inner"):
            inner = inner.inner
        ts = {"run_raw": [], "decode": [], "next_block": [], "kernels": []}
        for i in range(args.reps + 3):
            t0 = time.perf_counter()
            res = inner.run_raw()
            t1 = time.perf_counter()
            blk = inner._block_from_result(res)
            t2 = time.perf_counter()
            b2 = op.next_block()
            t3 = time.perf_counter()
            if i >= 3:
                ts["run_raw"].append((t1 - t0) * 1e3)
                ts["decode"].append((t2 - t1) * 1e3)
                ts["next_block"].append((t3 - t2) * 1e3)
                ts["kernels"].append((blk.filter_kernel_ms or 0) + (blk.agg_kernel_ms or 0))
        op.close()
        print(json.dumps({"query": q, "groups": len(blk.groups), **{k: round(float(np.median(v)), 4) for k, v in ts.items()},
                          "device_ms": round(float(blk.device_ms), 4)}), flush=True)
    for g in gsegs:
        g.destroy()


if __name__ == "__main__":
    main()
