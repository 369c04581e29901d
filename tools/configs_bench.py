"""Measurement of the BASELINE.json configs other than the headline (bench.py covers C2), one GPU.

Per query: p50 server-side latency (phip_plan_execute: the GPU work + result copy, plan prepared once,
as InstancePlanMakerImplV2's plan is built once per query), device time of the filter + aggregation
kernels (HIP events), rows scanned per second (numTotalDocs / p50 latency), algorithmic bytes
 per kernel time as a fraction of the 8 TB/s HBM peak, and the CPU oracle (one thread)
on a bounded sample of the same segments. Prints one JSON line per (config, query).

  python tools/configs_bench.py --configs C1,C3,C4,C5 [--c4-copies 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def inverted_bytes(qc, raw):
    """Referenced bitmap bytes + offsets of the inverted leaves of one segment."""
    from pinot_amd.query import predicate as predeval
    from pinot_amd.segment.dictionary import Dictionary
    total = 0
    cols = set()

    def walk(fc):
        nonlocal total
        if fc is None:
            return
        if fc.type == "PREDICATE":
            p = fc.predicate
            ci = raw.columns[p.column]
            if ci.inverted is None or p.type == "RANGE":
                return
            ev = predeval.evaluate(p, Dictionary(ci.dictionary, ci.metadata.data_type, ci.metadata.cardinality,
                                                 ci.metadata.string_width))
            card = ci.metadata.cardinality
            ids = ev.matching_dict_ids(card) if not ev.exclusive else np.asarray(ev.ids)
            offs = np.frombuffer(ci.inverted[:4 * (card + 1)], dtype=">u4").astype(np.int64)
            total += int(np.sum(offs[np.asarray(ids, dtype=np.int64) + 1] - offs[np.asarray(ids, dtype=np.int64)]))
            total += 4 * (len(ids) + 1)
            cols.add(p.column)
            return
        for c in fc.children:
            walk(c)
    walk(qc.filter)
    return total, cols


def alg_bytes(qc, raws):
    """Forward bytes of the scanned / projected columns + value dictionaries + inverted leaves."""
    from pinot_amd.query.context import columns_of
    filt = qc.filter.columns() if qc.filter else []
    vals = []
    for a in qc.aggregations:
        if a.argument is not None:
            vals += columns_of(a.argument)
    gb = [c for e in qc.group_by for c in columns_of(e)]
    total = 0
    for seg in raws:
        inv, inv_cols = inverted_bytes(qc, seg)
        total += inv
        for c in (set(filt) - inv_cols) | set(vals) | set(gb):
            m = seg.columns[c].metadata
            if not m.has_dictionary:
                total += seg.num_docs * (4 if m.data_type.name in ("INT", "FLOAT") else 8)
            elif m.is_sorted:
                total += 8 * m.cardinality
            else:
                total += (seg.num_docs * m.bits_per_element + 7) // 8
        for c in set(vals):
            m = seg.columns[c].metadata
            if m.has_dictionary:
                total += m.cardinality * (8 if m.data_type.name in ("LONG", "DOUBLE") else 4)
    return total


def time_gpu(qc, gsegs, reps, warmup):
    """p50 wall (ms), and per-kernel device time + library-reported algorithmic bytes (phip_result filter_* /
    agg_*; SURVEY.md §8d restated per launch, as bench.py reports them)."""
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    lib = _lib.load()
    # the reference's default numGroupsLimit (100,000, InstancePlanMakerImplV2.java): a query with more groups
    # takes the limit pass (limit.hip), as the reference's per-segment generators stop at the limit
    op = GpuInstancePlanMaker().make_instance_plan(qc, gsegs)
    if hasattr(op, "inner") and hasattr(op.inner, "run_raw"):
        op = op.inner  # star-tree: the traversal is plan-time; time the prepared plan over the star-tree docs
    wall, kern, dev, fk, ak = [], [], [], [], []
    fb = ab = 0
    ngroups = None
    if not hasattr(op, "run_raw"):  # FILTER / CASE / star-tree operators: several plans per block
        for i in range(warmup + reps):
            t0 = time.perf_counter()
            blk = op.next_block()
            t1 = time.perf_counter()
            if i >= warmup:
                wall.append((t1 - t0) * 1e3)
                kern.append(getattr(blk, "scan_kernel_ms", 0.0) or 0.0)
                dev.append(getattr(blk, "device_ms", 0.0) or 0.0)
                fk.append(getattr(blk, "filter_kernel_ms", 0.0) or 0.0)
                ak.append(getattr(blk, "agg_kernel_ms", 0.0) or 0.0)
        fb, ab = int(getattr(blk, "filter_bytes", 0) or 0), int(getattr(blk, "agg_bytes", 0) or 0)
        op.close()
        ng = len(blk.groups) if hasattr(blk, "groups") else None
        per = {}
        for name, ms, b in (("filter_kernel", float(np.mean(fk)), fb), ("agg_kernel", float(np.mean(ak)), ab)):
            if ms > 0:
                per[name] = {"ms": round(ms, 4), "alg_bytes": b, "GBps": round(b / (ms * 1e-3) / 1e9, 1),
                             "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        return (float(np.median(wall)), float(np.median(kern)), float(np.median(dev)), blk.stats.num_docs_scanned,
                ng, per)
    for i in range(warmup + reps):
        t0 = time.perf_counter()
        res = op.run_raw()
        t1 = time.perf_counter()
        r = res.contents
        if i >= warmup:
            wall.append((t1 - t0) * 1e3)
            kern.append(r.scan_kernel_ms)
            dev.append(r.device_ms)
            fk.append(r.filter_kernel_ms)
            ak.append(r.agg_kernel_ms)
        fb, ab = int(r.filter_bytes), int(r.agg_bytes)
        ngroups = r.num_groups
        docs = r.num_docs_scanned
        lib.phip_result_free(res)
    op.close()
    per = {}
    for name, ms, b in (("filter_kernel", float(np.mean(fk)), fb), ("agg_kernel", float(np.mean(ak)), ab)):
        if ms > 0:
            per[name] = {"ms": round(ms, 4), "alg_bytes": b, "GBps": round(b / (ms * 1e-3) / 1e9, 1),
                         "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    return float(np.median(wall)), float(np.median(kern)), float(np.median(dev)), docs, ngroups, per


def time_cpu(qc, raws, budget_s=10.0):
    from oracle import executor
    t = 0.0
    rows = 0
    runs = 0
    while t < budget_s and runs < 3:
        t0 = time.perf_counter()
        executor.execute(qc, raws)
        t += time.perf_counter() - t0
        rows += sum(r.num_docs for r in raws)
        runs += 1
    return rows / t / 1e9, t / runs * 1e3


def emit(cfg, name, qc, raws_meta, gsegs, args, cpu_raws=None, note=None):
    total_docs = sum(s.num_docs for s in gsegs)
    wall, kern, dev, docs, ng, per = time_gpu(qc, gsegs, args.reps, args.warmup)
    b = alg_bytes(qc, raws_meta)
    # roofline: the dominant kernel's own algorithmic bytes over its time (never above 1 by construction of the
    # per-launch bytes); the whole-query figure is kept as query_alg_bytes for reference
    dom = max(per, key=lambda k: per[k]["ms"]) if per else None
    out = {"config": cfg, "query": name, "rows": total_docs, "p50_ms": round(wall, 4), "kernel_ms": round(kern, 4),
           "device_ms": round(dev, 4), "G_rows_per_s": round(total_docs / (wall * 1e-3) / 1e9, 2),
           "docs_matched": int(docs), "groups": int(ng) if qc.group_by and ng is not None else None,
           "star_tree": bool(getattr(gsegs[0], "star_trees", None)) and name.startswith("STARTREE"),
           "query_alg_bytes": int(b), "kernels": per, "dominant_kernel": dom,
           "hbm_frac": per[dom]["frac"] if dom else None}
    if cpu_raws is not None and not args.no_cpu:
        v, ms = time_cpu(qc, cpu_raws)
        out["cpu_oracle"] = {"G_rows_per_s": round(v, 4), "ms_per_query": round(ms, 1), "cores": 1,
                             "rows": sum(r.num_docs for r in cpu_raws)}
    if note:
        out["note"] = note
    print(json.dumps(out), flush=True)


def strip_host(raw):
    for ci in raw.columns.values():
        ci.forward = b""


def run_c1(args):
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import bq
    raws = bq.make_segments(args.c1_rows, 1, args.c1_scenario, star_tree=True)  # the reference table config
    gsegs = [GpuSegment(r) for r in raws]
    for name, sql in bq.QUERIES.items():
        qc = parse(sql)
        heavy = name == "STARTREE_SUM_QUERY"
        cpu = None if heavy else raws  # the oracle's 10M-group merge is Python-bound: not a baseline
        emit("C1", name, qc, raws, gsegs, args, cpu_raws=cpu,
             note=f"{args.c1_scenario}, {args.c1_rows} rows, 1 segment")
    for g in gsegs:
        g.destroy()


def _ssb(args, queries, cfg):
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    cols = ssb.columns_for(queries)
    nseg = (args.sf * ssb.ROWS_PER_SF) // ssb.SEGMENT_ROWS
    gsegs, metas = [], []
    for i in range(0, nseg, 10):
        for r in ssb.make_segments(args.sf, cols, seed=42, segments=range(i, min(nseg, i + 10))):
            gsegs.append(GpuSegment(r))
            metas.append(r)
            if len(metas) > 1:
                strip_host(r)
    sample = [metas[0]]
    for q in queries:
        emit(cfg, q, parse(ssb.SSB_QUERIES[q]), metas, gsegs, args, cpu_raws=sample,
             note=f"SSB SF{args.sf}: {nseg} x 6M-row segments; CPU oracle on 1 segment")
    for g in gsegs:
        g.destroy()


def run_c4(args):
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import c4
    distinct = [c4.make_segment(i) for i in range(args.c4_distinct)]
    gsegs = []
    for _ in range(args.c4_copies):
        for r in distinct:
            gsegs.append(GpuSegment(r))
    metas = [distinct[i % len(distinct)] for i in range(len(gsegs))]
    for sel in c4.SELECTIVITIES:
        for agg in ("COUNT(*)", "SUM(M)"):
            emit("C4", f"sel={sel} {agg}", parse(c4.query(sel, agg)), metas, gsegs, args, cpu_raws=[distinct[0]],
                 note=f"{len(gsegs)} x 10M-row segments ({args.c4_distinct} distinct, each loaded "
                      f"{args.c4_copies}x); CPU oracle on 1 segment")
    for g in gsegs:
        g.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C3,C4,C5")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--sf", type=int, default=100)
    ap.add_argument("--c1-rows", type=int, default=10_000_000)
    ap.add_argument("--c1-scenario", default="EXP(0.001)")
    ap.add_argument("--c4-distinct", type=int, default=10)
    ap.add_argument("--c4-copies", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import ctypes

    from pinot_amd import _lib
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    cfgs = args.configs.split(",")
    if "C1" in cfgs:
        run_c1(args)
    if "C3" in cfgs:
        _ssb(args, ["Q2.1", "Q2.2", "Q2.3", "Q3.1", "Q3.2", "Q3.3", "Q3.4", "Q4.1", "Q4.2", "Q4.3"], "C3")
    if "C5" in cfgs:
        _ssb(args, ["C5"], "C5 (1 GPU slice: SF100 of SF1000/8)")
    if "C4" in cfgs:
        run_c4(args)


if __name__ == "__main__":
    main()
