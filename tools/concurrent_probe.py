"""Concurrent clients on one GPU: the SSB SF100 queries as 1..T client threads, each running its own prepared plan
back to back (its own execution lane), against the same queries run one after another. Prints one JSON line per
configuration: executions per second, mean wall per execution, mean kernel ms (HIP events).

usage: python tools/concurrent_probe.py [--queries Q1.1,Q1.2,Q1.3] [--layout sorted] [--reps 50]
       [--threads 1,2,3] [--raw]   (--raw: time the library call alone, run_raw, without the block decode)"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", default="Q1.1,Q1.2,Q1.3")
    ap.add_argument("--layout", default="sorted")
    ap.add_argument("--sf", type=int, default=100)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--threads", default="1,2,3")
    ap.add_argument("--raw", action="store_true")
    args = ap.parse_args()
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    lib = _lib.load()
    _lib.check(lib.phip_init((ctypes.c_int32 * 1)(0), 1))
    queries = args.queries.split(",")
    cols = ssb.columns_for(queries)
    nseg = (args.sf * ssb.ROWS_PER_SF) // ssb.SEGMENT_ROWS
    gsegs = []
    for i in range(0, nseg, 10):
        for r in ssb.make_segments(args.sf, cols, seed=42, segments=range(i, min(nseg, i + 10)), layout=args.layout):
            gsegs.append(GpuSegment(r))
            for ci in r.columns.values():
                if not ci.metadata.is_sorted:
                    ci.forward = b""
    pm = GpuInstancePlanMaker()

    def one(op):
        if args.raw:
            lib.phip_result_free(op.run_raw())
        else:
            op.next_block()

    # sequential reference: the queries one after another on one thread
    ops = [pm.make_instance_plan(parse(ssb.SSB_QUERIES[q]), gsegs) for q in queries]
    for _ in range(5):
        for op in ops:
            one(op)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        for op in ops:
            one(op)
    el = time.perf_counter() - t0
    n = args.reps * len(ops)
    print(json.dumps({"mode": "sequential", "queries": queries, "execs_per_s": round(n / el, 1),
                      "us_per_exec": round(el / n * 1e6, 2)}), flush=True)
    for op in ops:
        op.close()
    for nt in [int(x) for x in args.threads.split(",")]:
        # nt clients; client i runs queries[i % len(queries)]
        ops = [pm.make_instance_plan(parse(ssb.SSB_QUERIES[queries[i % len(queries)]]), gsegs) for i in range(nt)]
        for op in ops:
            for _ in range(5):
                one(op)
        barrier = threading.Barrier(nt + 1)
        walls = [[] for _ in range(nt)]

        def client(i, reps):
            barrier.wait()
            for _ in range(reps):
                ts = time.perf_counter()
                one(ops[i])
                walls[i].append(time.perf_counter() - ts)

        for reps in (5, args.reps):  # a concurrent warm-up first: the library creates lanes on demand (~10-20 ms)
            walls = [[] for _ in range(nt)]
            ths = [threading.Thread(target=client, args=(i, reps)) for i in range(nt)]
            for th in ths:
                th.start()
            barrier.wait()
            t0 = time.perf_counter()
            for th in ths:
                th.join()
            el = time.perf_counter() - t0
        n = args.reps * nt
        print(json.dumps({"mode": "threads", "threads": nt, "execs_per_s": round(n / el, 1),
                          "us_per_exec_wall": [round(float(np.mean(w)) * 1e6, 1) for w in walls],
                          "us_p50": [round(float(np.median(w)) * 1e6, 1) for w in walls]}), flush=True)
        for op in ops:
            op.close()
    for g in gsegs:
        g.destroy()


if __name__ == "__main__":
    main()
