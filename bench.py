"""Headline benchmark: SSB SF100 flattened lineorder, Q1.1-Q1.3 (scan filter + SUM), per GPU.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; N>1 is launched by
torch.distributed.run with one rank per GPU. A step = Q1.1 + Q1.2 + Q1.3, each one phip_query over
every segment resident on the rank (SF100 = 100 segments x 6M rows per GPU, weak scaling: rank r owns
segments [100r, 100r+100) of an SF(100N) table). Partial aggregates of each query are merged across
ranks with an RCCL all-reduce (the CombineOperator replacement's exchange step). value = rows
scanned per second over the whole job (3 x 600M x N rows per step / max-over-ranks step time).

Also reported: p50 latency per query, the fused scan kernel's HBM roofline fraction (algorithmic
bytes per SURVEY.md §8(d) / scan-kernel time from HIP events recorded by libpinot_hip on the stream
the kernel runs on), and the CPU oracle timed on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(qc, segments):
    """sum over referenced columns of ceil(N*b/8) + value-lookup dictionaries card*w."""
    from pinot_amd.query.context import columns_of
    filt = qc.filter.columns() if qc.filter else []
    vals = []
    for a in qc.aggregations:
        if a.argument is not None:
            vals += columns_of(a.argument)
    for e in qc.group_by:
        vals += columns_of(e)
    total = 0
    for seg in segments:
        for c in set(filt) | set(vals):
            m = seg.columns[c].metadata
            total += (seg.num_docs * m.bits_per_element + 7) // 8
        for c in set(vals):
            m = seg.columns[c].metadata
            if c not in [e.name for e in qc.group_by]:
                total += m.cardinality * 4
    return total


def cpu_baseline(queries, sf, seed, target_s=15.0):
    """The oracle ('port', scalar C + numpy, 1 thread) on a bounded sample of the same segments."""
    from oracle import executor
    from pinot_amd.query.sql import parse
    from tools import ssb
    cols = ssb.columns_for(queries)
    qcs = [parse(ssb.SSB_QUERIES[q]) for q in queries]
    rows = 0
    t_total = 0.0
    nseg = 0
    while t_total < target_s and nseg < 48:
        seg = ssb.make_segments(sf, cols, seed=seed, segments=[nseg])[0]
        t0 = time.perf_counter()
        for qc in qcs:
            executor.execute(qc, [seg])
            rows += seg.num_docs
        t_total += time.perf_counter() - t0
        nseg += 1
    return {"value": rows / t_total / 1e9, "unit": "G rows/s", "cores": 1, "kind": "port",
            "sample": f"{'+'.join(queries)} over {nseg} x 6M-row SF{sf} segments ({rows} rows scanned, "
                      f"{t_total:.1f} s, oracle/executor.py single thread)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sf", type=int, default=100, help="scale factor per GPU (SF100 = 600M rows)")
    ap.add_argument("--queries", default="Q1.1,Q1.2,Q1.3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01_traffic.json"),
                    help="HBM bytes per scan launch from a rocprofv3 --pmc pass (see profiles/)")
    ap.add_argument("--seed", type=int, default=42)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    from pinot_amd import _lib
    import ctypes
    dev = (ctypes.c_int32 * 1)(local_rank if world > 1 else 0)
    _lib.check(_lib.load().phip_init(dev, 1))

    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb

    queries = args.queries.split(",")
    cols = ssb.columns_for(queries)
    seg_per_gpu = (args.sf * ssb.ROWS_PER_SF) // ssb.SEGMENT_ROWS
    my_segs = list(range(rank * seg_per_gpu, (rank + 1) * seg_per_gpu))
    t0 = time.time()
    gsegs, raw_meta = [], []
    chunk = 10
    for i in range(0, len(my_segs), chunk):  # generate + load in chunks to bound host memory
        raws = ssb.make_segments(args.sf * world, cols, seed=args.seed, segments=my_segs[i:i + chunk])
        for r in raws:
            gsegs.append(GpuSegment(r))
            raw_meta.append(r)
            for ci in r.columns.values():  # free host copies of the (large) index bytes
                ci.forward = b""
    load_s = time.time() - t0
    rows_per_rank = sum(s.num_docs for s in gsegs)

    pm = GpuInstancePlanMaker()
    qcs = {q: parse(ssb.SSB_QUERIES[q]) for q in queries}
    ops = {q: pm.make_instance_plan(qcs[q], gsegs) for q in queries}
    alg_bytes = {q: algorithmic_bytes(qcs[q], raw_meta) for q in queries}

    from pinot_amd.engine.distributed import allreduce_block

    def run_query(q):
        blk = ops[q].next_block()
        if dist is not None:
            # the exchange step: RCCL all-reduce of the partial blocks (exact int64 / f64 / HLL-max slots)
            merged = allreduce_block(blk, dist)
            merged.scan_kernel_ms = blk.scan_kernel_ms
            return merged
        return blk

    for _ in range(args.warmup):
        for q in queries:
            run_query(q)
    lat = {q: [] for q in queries}
    kern = {q: [] for q in queries}
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        for q in queries:
            ts = time.perf_counter()
            blk = run_query(q)
            lat[q].append((time.perf_counter() - ts) * 1e3)
            kern[q].append(blk.scan_kernel_ms)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank != 0:
        dist.destroy_process_group()
        return
    total_rows = rows_per_rank * world * len(queries) * args.steps
    value = total_rows / elapsed / 1e9
    ms_per_step = elapsed * 1e3 / args.steps
    kern_ms = sum(np.mean(kern[q]) for q in queries)
    bytes_per_step = sum(alg_bytes[q] for q in queries)
    achieved = bytes_per_step / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("queries") == queries and tj.get("sf") == args.sf:
                traffic = tj.get("hbm_bytes_per_step")
        except Exception:
            traffic = None
    out = {
        "metric": "rows scanned/s (G) + p50 query latency, SSB flattened SF100, Q1.1-Q1.3",
        "value": round(value, 3),
        "unit": "G rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 dict ids / int64 sums",
        "data": "synthetic SSB-shaped (tools/ssbgen.c, seeded), Pinot segment encodings",
        "config": {"workload": f"SSB SF{args.sf} flattened lineorder per GPU, {len(gsegs)} segments x "
                               f"{ssb.SEGMENT_ROWS} rows, queries {'+'.join(queries)}",
                   "rows_per_gpu": rows_per_rank, "parallelism": f"segment-sharded x{world}, RCCL all-reduce"},
        "p50_latency_ms": {q: round(float(np.median(lat[q])), 3) for q in queries},
        "scan_kernel_ms": {q: round(float(np.mean(kern[q])), 3) for q in queries},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_step": bytes_per_step,
                     "kernels": "filter_kernel + agg_kernel per query (HIP events around both, on the library's stream)",
                     "kernel_ms_per_step": round(kern_ms, 4)},
        "load_s": round(load_s, 1),
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(queries, args.sf * world, args.seed)
    print(json.dumps(out), flush=True)
    for s in gsegs:
        s.destroy()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
