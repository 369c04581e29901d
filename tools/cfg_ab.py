"""A/B of library settings on the BASELINE configs C1 (BenchmarkQueries, 10M rows, tools/bq.py) and C4 (inverted-index
sweep, 100 x 10M rows, tools/c4.py) inside ONE process: the segments are generated and loaded once, then every query is
planned and timed under each setting (environment variables the library reads at plan creation). Prints one JSON line
per (query, setting): p50 wall, mean filter / aggregation kernel ms (HIP events), and whether the block equals the first
setting's (exact for integers, 1e-9 relative for doubles).

usage: python tools/cfg_ab.py --configs c4 --set "" --set PHIP_AGG_LDS_DICT_MAX=1024 [--queries 'sel=0.5 SUM(M)']"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gb_ab import _same  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c4")
    ap.add_argument("--set", action="append", default=None)
    ap.add_argument("--queries", default="", help="comma-separated query names to keep ('' = all)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--c1-rows", type=int, default=10_000_000)
    ap.add_argument("--c4-distinct", type=int, default=10)
    ap.add_argument("--c4-copies", type=int, default=10)
    args = ap.parse_args()
    sets = args.set if args.set is not None else [""]
    keep = set(q for q in args.queries.split(",") if q)
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import bq, c4
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    base_env = dict(os.environ)
    for cfg in args.configs.split(","):
        if cfg == "c1":
            raws = bq.make_segments(args.c1_rows, 1, "EXP(0.001)")
            gsegs = [GpuSegment(r) for r in raws]
            named = dict(bq.QUERIES)
        else:
            distinct = [c4.make_segment(i) for i in range(args.c4_distinct)]
            gsegs = [GpuSegment(r) for _ in range(args.c4_copies) for r in distinct]
            named = {f"sel={s} {a}": c4.query(s, a) for s in c4.SELECTIVITIES for a in ("COUNT(*)", "SUM(M)")}
        for name, sql in named.items():
            if keep and name not in keep:
                continue
            qc = parse(sql)
            ref = None
            for st in sets:
                os.environ.clear()
                os.environ.update(base_env)
                for kv in st.split():
                    k, v = kv.split("=", 1)
                    os.environ[k] = v
                op = GpuInstancePlanMaker().make_instance_plan(qc, gsegs)
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
                if hasattr(op, "close"):
                    op.close()
                groups = getattr(blk, "groups", None)
                if groups is None:
                    groups = {(): list(blk.results)}
                same = None
                if ref is None:
                    ref = groups
                else:
                    same = set(ref) == set(groups) and all(_same(ref[k], groups[k]) for k in ref)
                print(json.dumps({"config": cfg, "query": name, "set": st, "p50_ms": round(float(np.median(wall)), 4),
                                  "filter_ms": round(float(np.mean(fk)), 4), "agg_ms": round(float(np.mean(ak)), 4),
                                  "docs": blk.stats.num_docs_scanned, "fused": bool(getattr(blk, "fused", False)),
                                  "same_as_first": same}), flush=True)
        os.environ.clear()
        os.environ.update(base_env)
        for g in gsegs:
            g.destroy()


if __name__ == "__main__":
    main()
