"""A/B of library settings on the SSB group-by configs (C3 Q2.x-Q4.x, C5) inside ONE process: the SF100 segments
are generated and loaded once, then every query is planned and timed under each setting (environment variables
the library reads at plan creation, e.g. PHIP_GB_BATCH=0 / PHIP_GB_MODE=global). Prints one JSON line per
(query, setting): p50 wall, mean filter / aggregation kernel ms (HIP events), groups; and checks that every
setting returns the same groups and values (exact for integer results, 1e-9 relative for doubles).

usage: python tools/gb_ab.py --queries Q2.1,Q3.1,C5 --set "" --set PHIP_GB_BATCH=0 [--sf 100] [--reps 20]
       [--layout sorted]   (the Q1.x configs too: any SSB query name works; --sql NAME::SQL adds one)"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _same(a, b):
    if isinstance(a, (list, tuple)):
        return all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, np.ndarray):
        return np.array_equal(a, b)
    if isinstance(a, float) or isinstance(b, float):
        return a == b or abs(a - b) <= 1e-9 * max(abs(a), abs(b))
    return a == b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", default="Q2.1,Q2.2,Q2.3,Q3.1,Q3.2,Q3.3,Q3.4,Q4.1,Q4.2,Q4.3,C5")
    ap.add_argument("--set", action="append", default=None, help="space-separated NAME=VALUE settings ('' = none)")
    ap.add_argument("--sf", type=int, default=100)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--layout", default="unsorted")
    ap.add_argument("--sql", action="append", default=[],
                    help="NAME::SQL -- an extra query over the SSB columns (e.g. a C5 variant without its HLL), usable "
                         "in --queries by NAME")
    ap.add_argument("--hog-gib", type=float, default=0.0,
                    help="allocate (and zero) this many GiB of HBM beside the segments first: does resident memory the "
                         "queries never touch slow them (the group-by records' residency effect)?")
    ap.add_argument("--hog-chunk-mib", type=int, default=1024, help="size of each --hog-gib allocation")
    ap.add_argument("--gap", type=float, default=0.0,
                    help="seconds of idle GPU before each (query, setting): tools/trace_summary.py splits a rocprofv3 "
                         "kernel trace of this run into the queries at these gaps")
    args = ap.parse_args()
    sets = args.set if args.set is not None else [""]
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    for spec in args.sql:
        name, sql = spec.split("::", 1)
        ssb.SSB_QUERIES[name] = sql
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    queries = args.queries.split(",")
    cols = ssb.columns_for(queries)
    nseg = (args.sf * ssb.ROWS_PER_SF) // ssb.SEGMENT_ROWS
    gsegs = []
    t0 = time.time()
    for i in range(0, nseg, 10):
        for r in ssb.make_segments(args.sf, cols, seed=42, segments=range(i, min(nseg, i + 10)),
                                   layout=args.layout):
            gsegs.append(GpuSegment(r))
            for ci in r.columns.values():
                if not ci.metadata.is_sorted:
                    ci.forward = b""
    print(json.dumps({"loaded_segments": len(gsegs), "load_s": round(time.time() - t0, 1)}), flush=True)
    hogs = []
    if args.hog_gib > 0:
        hip = ctypes.CDLL("libamdhip64.so")
        left = int(args.hog_gib * (1 << 30))
        while left > 0:
            n = min(left, args.hog_chunk_mib << 20)
            p = ctypes.c_void_p()
            if hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) != 0:
                raise SystemExit("hipMalloc failed")
            hip.hipMemset(p, 0, ctypes.c_size_t(n))
            hogs.append(p)
            left -= n
        hip.hipDeviceSynchronize()
    base_env = dict(os.environ)
    for q in queries:
        qc = parse(ssb.SSB_QUERIES[q])
        ref = None
        for st in sets:
            os.environ.clear()
            os.environ.update(base_env)
            for kv in st.split():
                k, v = kv.split("=", 1)
                os.environ[k] = v
            op = GpuInstancePlanMaker().make_instance_plan(qc, gsegs)
            if args.gap:
                time.sleep(args.gap)
            wall, fk, ak = [], [], []
            blk = None
            for i in range(args.warmup + args.reps):
                ts = time.perf_counter()
                blk = op.next_block()
                te = time.perf_counter()
                if i >= args.warmup:
                    wall.append((te - ts) * 1e3)
                    fk.append(getattr(blk, "filter_kernel_ms", 0.0) or 0.0)
                    ak.append(getattr(blk, "agg_kernel_ms", 0.0) or 0.0)
            op.close()
            groups = getattr(blk, "groups", None)
            if groups is None:  # aggregation only: one row
                groups = {(): list(blk.results)}
            same = None
            if ref is None:
                ref = groups
            else:
                same = set(ref) == set(groups) and all(_same(ref[k], groups[k]) for k in ref)
            print(json.dumps({"query": q, "set": st, "p50_ms": round(float(np.median(wall)), 4),
                              "filter_ms": round(float(np.mean(fk)), 4), "agg_ms": round(float(np.mean(ak)), 4),
                              "groups": len(groups), "docs": blk.stats.num_docs_scanned,
                              "filter_bytes": getattr(blk, "filter_bytes", None), "agg_bytes": getattr(blk, "agg_bytes", None),
                              "fused": bool(getattr(blk, "fused", False)), "same_as_first": same}), flush=True)
    os.environ.clear()
    os.environ.update(base_env)
    for g in gsegs:
        g.destroy()


if __name__ == "__main__":
    main()
