"""Kernel-time decomposition on synthetic SSB segments (a measurement aid, not part of the product).

Loads SF-`--sf` flattened lineorder segments once, then runs each query `--reps` times through the
GPU plan maker and prints, per query, the median scan-kernel and device time, the algorithmic bytes
 and the resulting HBM GB/s. Queries are SSB names (Q1.1 …) or raw SQL.

  python tools/explore.py --sf 100 Q1.1 "select count(*) from lineorder where LO_DISCOUNT between 1 and 3"
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("queries", nargs="+")
    ap.add_argument("--sf", type=int, default=100)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--seed", type=int, default=42)
    args = ap.parse_args()

    import ctypes

    from bench import algorithmic_bytes
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.context import columns_of
    from pinot_amd.query.sql import parse
    from tools import ssb

    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    sqls = [ssb.SSB_QUERIES.get(q, q) for q in args.queries]
    qcs = [parse(s) for s in sqls]
    cols = []
    for qc in qcs:
        need = list(qc.filter.columns()) if qc.filter else []
        for a in qc.aggregations:
            if a.argument is not None:
                need += columns_of(a.argument)
        for e in qc.group_by:
            need += columns_of(e)
        for c in need:
            if c not in cols:
                cols.append(c)
    nseg = (args.sf * ssb.ROWS_PER_SF) // ssb.SEGMENT_ROWS
    t0 = time.time()
    gsegs, metas = [], []
    for i in range(0, nseg, 10):
        for r in ssb.make_segments(args.sf, cols, seed=args.seed, segments=range(i, min(nseg, i + 10))):
            gsegs.append(GpuSegment(r))
            metas.append(r)
            for ci in r.columns.values():
                ci.forward = b""
    print(json.dumps({"loaded_segments": len(gsegs), "load_s": round(time.time() - t0, 1)}), flush=True)
    pm = GpuInstancePlanMaker()
    for name, qc in zip(args.queries, qcs):
        op = pm.make_instance_plan(qc, gsegs)
        op.next_block()
        kern, dev, wall = [], [], []
        for _ in range(args.reps):
            ts = time.perf_counter()
            blk = op.next_block()
            wall.append((time.perf_counter() - ts) * 1e3)
            kern.append(blk.scan_kernel_ms)
            dev.append(blk.device_ms)
        b = algorithmic_bytes(qc, metas)
        k = float(np.median(kern))
        print(json.dumps({"query": name, "scan_ms": round(k, 4), "device_ms": round(float(np.median(dev)), 4),
                          "wall_ms": round(float(np.median(wall)), 4), "alg_bytes": b,
                          "alg_GBps": round(b / (k * 1e-3) / 1e9, 1),
                          "docs_scanned": blk.stats.num_docs_scanned}), flush=True)
    for s in gsegs:
        s.destroy()


if __name__ == "__main__":
    main()
