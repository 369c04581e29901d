"""Where a query's wall time goes on the headline step (SSB SF100 sorted, Q1.1-Q1.3, bench.py's segments):
per query, the wall time of next_block(), of the phip_plan_execute call inside it (ctypes, GIL released), of the
result decode in Python, and the library's device time (events around the launches) and kernel times.

    python tools/host_probe.py [--segs 100] [--reps 50] [--layout sorted]
"""
import argparse
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=100)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--layout", default="sorted")
    args = ap.parse_args()
    import torch  # noqa: F401  (same import order as bench.py)
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    lib = _lib.load()
    _lib.check(lib.phip_init((ctypes.c_int32 * 1)(0), 1))
    qs = ["Q1.1", "Q1.2", "Q1.3"]
    cols = ssb.columns_for(qs)
    segs = []
    for i in range(0, args.segs, 10):
        for r in ssb.make_segments(100, cols, segments=list(range(i, min(i + 10, args.segs))), layout=args.layout):
            segs.append(GpuSegment(r))
    ops = {q: GpuInstancePlanMaker().make_instance_plan(parse(ssb.SSB_QUERIES[q]), segs) for q in qs}
    for q in qs:
        for _ in range(5):
            ops[q].next_block()
    rows = {q: [] for q in qs}
    step = []
    for _ in range(args.reps):
        t_step = time.perf_counter()
        for q in qs:
            op = ops[q]
            t0 = time.perf_counter()
            res = op.run_raw()
            t1 = time.perf_counter()
            r = res.contents
            dev, kf, ka = r.device_ms, r.filter_kernel_ms, r.agg_kernel_ms
            blk = op._block_from_result(res)
            t2 = time.perf_counter()
            rows[q].append(((t2 - t0) * 1e3, (t1 - t0) * 1e3, (t2 - t1) * 1e3, dev, kf, ka))
            del blk
        step.append((time.perf_counter() - t_step) * 1e3)
    print(f"layout {args.layout}, {len(segs)} segments; ms, median over {args.reps} reps")
    print(f"{'query':6s} {'wall':>7s} {'execute':>8s} {'decode':>7s} {'device':>7s} {'filter':>7s} {'agg':>7s}")
    for q in qs:
        m = np.median(np.array(rows[q]), axis=0)
        print(f"{q:6s} " + " ".join(f"{x:7.4f}" for x in m))
    print(f"step wall median {np.median(step):.4f} ms")
    for op in ops.values():
        op.close()


if __name__ == "__main__":
    main()
