"""Headline benchmark: SSB SF100 flattened lineorder, Q1.1-Q1.3 (scan filter + SUM), per GPU.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; N>1 is launched by
torch.distributed.run with one rank per GPU, or, without it, by this script itself (spawn_ranks: N rank processes
started before any GPU call, rank 0's line printed). A step = Q1.1 + Q1.2 + Q1.3, each one query over 100 segments
x 6M rows per GPU (SF100 per GPU, weak scaling). At N = 1 the rank holds exactly those 100 (BASELINE C2); at
N > 1 each rank holds 125 segments of an SF(125N) table (N = 8: SF1000, BASELINE C5) and the step runs over
the first 100 of them, while the C5 query (DISTINCTCOUNTHLL + GROUP BY) runs over all 125 per rank and is
reported under "c5". Partial aggregates of each query are merged across ranks (the CombineOperator
replacement's exchange step, engine/distributed.distributed_block: each GPU's one-group partial table -- rows and
statistics in device memory -- all-reduced in place over RCCL, one int64 SUM collective for Q1.x). value = rows
scanned per second over the whole job (3 x 600M x N rows per step / max-over-ranks wall time of the K timed
steps).

Layout: rows sorted by LO_ORDERDATE, so D_YEAR / D_YEARMONTHNUM / D_WEEKNUMINYEAR carry
sorted forward indexes and their predicates are doc ranges (SortedIndexBasedFilterOperator), exactly as
Pinot's CPU path would use them. The same queries over the unsorted layout (every row scanned: the
scan-bound case) are measured in the same run and reported under "unsorted_layout".

Roofline (per kernel, from the library's own HIP events on the stream the kernels run on -- recorded by each launch's
dispatch packet in a repeat of the timed executions, so they time the kernel itself): achieved = the kernel's
algorithmic bytes per launch (phip_result.filter_bytes / agg_bytes, SURVEY.md §8d, computed by libpinot_hip from the
tiles it must stream and the docs it must project) / its mean launch time; the dominant kernel (largest time share)
is the headline `roofline`. `traffic` = HBM bytes per launch of that
kernel from this round's rocprofv3 --pmc FETCH_SIZE (x2, gfx950) / WRITE_SIZE passes
(profiles/<round>_traffic.json, tools/traffic.py), or null.

cpu_baseline: oracle/cpu_scan.c, an OpenMP C restatement of Pinot's CPU server path ("restatement, not
Pinot": no JVM here), over the SAME segments and queries, one worker per usable CPU (the affinity mask capped
by the cgroup quota: oracle/cpu_baseline.usable_cpus).
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
ROUND = "r06"


def latest_profile(kind):
    """profiles/<round>_<kind>.json of this round, else the newest earlier round's (rNN sorts by name)."""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{kind}.json")))
    mine = os.path.join(ROOT, "profiles", f"{ROUND}_{kind}.json")
    return mine if os.path.exists(mine) else (cands[-1] if cands else mine)


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def load_layout(ssb, seg_per_gpu, world, rank, cols, seed, layout, keep_host):
    """This rank's segments [seg_per_gpu * rank, seg_per_gpu * (rank + 1)) of an SF(seg_per_gpu x world) table."""
    from pinot_amd.engine.segment import GpuSegment
    table_sf = seg_per_gpu * world * ssb.SEGMENT_ROWS // ssb.ROWS_PER_SF
    my_segs = list(range(rank * seg_per_gpu, (rank + 1) * seg_per_gpu))
    gsegs, raws = [], []
    for i in range(0, len(my_segs), 10):  # generate + load in chunks to bound host memory
        for r in ssb.make_segments(table_sf, cols, seed=seed, segments=my_segs[i:i + 10], layout=layout):
            gsegs.append(GpuSegment(r))
            if keep_host:
                raws.append(r)
            else:
                for ci in r.columns.values():  # free host copies of the (large) fixed-bit index bytes; the plan
                    if not ci.metadata.is_sorted:  # reads sorted columns' doc ranges on the host (tiny)
                        ci.forward = b""
    return gsegs, raws


def run_c5(args, dist, qc, gsegs, torch):
    """BASELINE config C5: DISTINCTCOUNTHLL + GROUP BY over every segment of every rank, merged
    across GPUs by distributed_block (node-global dictionaries registered once at load, the dense partial
    tables all-reduced in place over RCCL, one collective per reduce operator and type). Returns wall seconds of
    the K timed queries (max over ranks), per-query latencies and the merged block of the last query."""
    from pinot_amd.engine.distributed import distributed_block, register_global_dictionaries
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    register_global_dictionaries(gsegs, [e.name for e in qc.group_by], dist)
    op = GpuInstancePlanMaker().make_instance_plan(qc, gsegs)
    fb = GpuInstancePlanMaker(device_trim=False).make_instance_plan(qc, gsegs)
    for _ in range(args.warmup):
        distributed_block(op, dist, fallback_op=fb)
    lat = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    blk = None
    for _ in range(args.steps):
        ts = time.perf_counter()
        blk = distributed_block(op, dist, fallback_op=fb)
        lat.append((time.perf_counter() - ts) * 1e3)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    op.close()
    fb.close()
    return el, lat, blk


def run_layout(args, dist, queries, qcs, gsegs, torch):
    """Warm-up, then exactly args.steps timed steps bracketed by barrier + synchronize on both sides."""
    from pinot_amd.engine.distributed import distributed_block
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    pm = GpuInstancePlanMaker()
    ops = {q: pm.make_instance_plan(qcs[q], gsegs) for q in queries}

    def run_query(q):
        if dist is not None:  # the exchange step: the partial tables all-reduced in place on the GPUs (RCCL)
            return distributed_block(ops[q], dist)  # (the merged block carries this GPU's kernel times)
        return ops[q].next_block()

    # The warm-up and timed steps run as a server would: without the library's per-kernel timing markers
    # (PHIP_KERNEL_TIMING=0 -- two barrier packets per query the command processor waits on; --timed-markers keeps
    # them); the kernel durations of the roofline come from the pass after the timed region.
    markers_env = os.environ.get("PHIP_KERNEL_TIMING")
    if not args.timed_markers:
        os.environ["PHIP_KERNEL_TIMING"] = "0"
    try:
        for _ in range(args.warmup):
            for q in queries:
                run_query(q)
        lat = {q: [] for q in queries}
        kstats = {q: [] for q in queries}
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            for q in queries:
                ts = time.perf_counter()
                blk = run_query(q)
                lat[q].append((time.perf_counter() - ts) * 1e3)
                kstats[q].append((blk.filter_kernel_ms, blk.agg_kernel_ms, blk.filter_bytes, blk.agg_bytes,
                                   bool(getattr(blk, "fused", False)), int(getattr(blk, "stream_bytes", 0) or 0)))
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
    finally:
        if markers_env is None:
            os.environ.pop("PHIP_KERNEL_TIMING", None)
        else:
            os.environ["PHIP_KERNEL_TIMING"] = markers_env
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # one more execution per query, outside the timed region: this rank's answers, checked against the CPU
    # restatement on the same segments (check_parity)
    answers = {q: ops[q].next_block() for q in queries}
    # Kernel durations for the roofline, outside the timed region: the same executions again with each one-kernel
    # plan's HIP events recorded by its dispatch packet (PHIP_EXT_EVENTS=1: hipExtLaunchKernel on the library's
    # stream), which time the kernel itself; the timed steps' barrier-marker events also hold the ~5 us dispatch
    # latency of the kernel behind the first marker (sorted Q1.x: 131.8 / 35.3 / 21.4 us vs rocprofv3's 126.3 / 30.0 /
    # 16.0, profiles/r06f_trace_sorted.json). The extra dispatch work is why the timed steps do not use it
    # (profiles/r04p_host_ab.log: step 0.286 -> 0.304 ms).
    kstats_ext = {q: [] for q in queries}
    os.environ["PHIP_EXT_EVENTS"] = "1"
    try:
        for _ in range(args.steps):
            for q in queries:
                blk = ops[q].next_block()
                kstats_ext[q].append((blk.filter_kernel_ms, blk.agg_kernel_ms, blk.filter_bytes, blk.agg_bytes,
                                      bool(getattr(blk, "fused", False)), int(getattr(blk, "stream_bytes", 0) or 0)))
    finally:
        del os.environ["PHIP_EXT_EVENTS"]
    concurrent = None
    if dist is None and not args.no_concurrent:
        # Outside the headline: the same queries as concurrent clients (one thread per query, each running its
        # prepared plan `steps` times back to back on its own execution lane -- a server's worker threads, DESIGN.md
        # §7); reported beside `value`, which stays the sequential step.
        # The warm-up runs concurrently too: the library creates an execution lane (stream + scratch, ~10-20 ms) the
        # first time a query finds every lane busy.
        import threading
        barrier = threading.Barrier(len(queries) + 1)

        def client(q, n):
            barrier.wait()
            for _ in range(n):
                ops[q].next_block()

        for n in (max(args.warmup, 1), args.steps):
            threads = [threading.Thread(target=client, args=(q, n)) for q in queries]
            for th in threads:
                th.start()
            torch.cuda.synchronize()
            barrier.wait()
            t0 = time.perf_counter()
            for th in threads:
                th.join()
            torch.cuda.synchronize()
            concurrent = time.perf_counter() - t0
    for op in ops.values():
        op.close()
    return elapsed, lat, kstats, answers, concurrent, kstats_ext


def check_parity(queries, qcs, answers, raws, dist, torch):
    """Every query's GPU answer on this rank (exact int64 SUM, numDocsScanned) against oracle/cpu_scan.c over the
    same segments (its SUM is a double sum of integer products, exact below 2^53), outside the timed region; the
    ranks agree on the verdict with one MIN all-reduce. Returns (ok, per-query detail)."""
    from oracle import cpu_baseline
    detail = {}
    ok = True
    threads = cpu_baseline.usable_cpus()[0]
    for q in queries:
        total, matched = cpu_baseline.Prepared(qcs[q], raws).run(threads)
        blk = answers[q]
        got = blk.results[0]
        good = (isinstance(got, int) and abs(total) < 2 ** 53 and got == int(total)
                and blk.stats.num_docs_scanned == matched)
        ok &= good
        detail[q] = {"sum": got, "cpu_sum": int(total), "docs": blk.stats.num_docs_scanned, "cpu_docs": matched,
                     "equal": good}
    if dist is not None:
        t = torch.tensor([1 if ok else 0], dtype=torch.int64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item())
    return ok, detail


GROUP_BY_LEGS = {"c3": ["Q2.1", "Q2.2", "Q2.3", "Q3.1", "Q3.2", "Q3.3", "Q3.4", "Q4.1", "Q4.2", "Q4.3"],
                 "c5": ["C5"]}


def _same_value(got, want):
    """An exact int64 SUM intermediate (int) against the CPU's exact sum; a double one must equal it exactly too
    (the sums here are integral and below 2^53, where the reference's double holder is exact)."""
    if isinstance(got, (int, np.integer)):
        return int(got) == want
    return abs(want) < 2 ** 53 and float(got) == float(want)


def compare_groups(blk, cpu_groups, sum_agg, hll_agg):
    """A GPU GroupByResultsBlock against cpu_baseline.PreparedGroupBy.groups: the same key tuples, every SUM equal,
    every HLL register equal. Returns (equal, first mismatch or None)."""
    if set(blk.groups) != set(cpu_groups):
        extra = sorted(set(blk.groups) - set(cpu_groups), key=str)[:2]
        miss = sorted(set(cpu_groups) - set(blk.groups), key=str)[:2]
        return False, f"group sets differ: {len(blk.groups)} vs {len(cpu_groups)}, gpu-only {extra}, cpu-only {miss}"
    for k, (s, _, regs) in cpu_groups.items():
        g = blk.groups[k]
        if sum_agg is not None and not _same_value(g[sum_agg], s):
            return False, f"SUM of {k}: {g[sum_agg]} vs {s}"
        if hll_agg is not None and not np.array_equal(np.asarray(g[hll_agg], dtype=np.uint8), regs):
            return False, f"HLL registers of {k} differ"
    return True, None


def check_merged_group_by(qc, blk, raws, dist):
    """The cross-GPU merged group-by block (every rank holds it) against oracle/cpu_scan.c over ALL ranks'
    segments: each rank runs the CPU group-by over its own segments, the value-keyed groups are gathered and merged
    (sums and counts added, registers max-ed: the reference's combine merge), and each rank compares. Returns
    "checked" when every rank's block equals the merged CPU answer (one MIN all-reduce), else the first mismatch."""
    import torch
    from oracle import cpu_baseline
    p = cpu_baseline.PreparedGroupBy(qc, raws)
    out = p.run(cpu_baseline.usable_cpus()[0])
    mine = (p.groups(out), out[3])
    parts = [mine]
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, mine)
    merged, docs = {}, 0
    for groups, d in parts:
        docs += d
        for k, (s, c, regs) in groups.items():
            if k in merged:
                s0, c0, r0 = merged[k]
                merged[k] = (None if s is None else s0 + s, c0 + c, None if regs is None else np.maximum(r0, regs))
            else:
                merged[k] = (s, c, regs)
    good, why = compare_groups(blk, merged, p.sum_agg, p.hll_agg)
    if good and blk.stats.num_docs_scanned != docs:
        good, why = False, f"numDocsScanned {blk.stats.num_docs_scanned} vs {docs}"
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([1 if good else 0], dtype=torch.int64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if good and not bool(t.item()):
            good, why = False, "another rank's merged block differs"
    return "checked" if good else f"MISMATCH: {why}"


def run_group_by(args, dist, leg, gsegs, raws, torch, want_cpu):
    """BASELINE C3 (SSB Q2.x-Q4.x, multi-column GROUP BY) / the C5 query over this rank's resident segments, each
    query prepared once and run warmup + steps times; then one more execution per query, outside the timed region,
    checked bit-exactly against oracle/cpu_scan.c's group-by over the same segments (group set, exact SUMs, HLL
    registers, numDocsScanned). Per query: p50 latency, kernel times and each kernel's algorithmic-byte frac.
    At N > 1 the queries run over the rank's own segments (the merged C5 is "c5_merged")."""
    from oracle import cpu_baseline
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.query.sql import parse
    from tools import ssb
    queries = GROUP_BY_LEGS[leg]
    qcs = {q: parse(ssb.SSB_QUERIES[q]) for q in queries}
    pm = GpuInstancePlanMaker()
    ops = {q: pm.make_instance_plan(qcs[q], gsegs) for q in queries}
    for _ in range(args.warmup):
        for q in queries:
            ops[q].next_block()
    lat = {q: [] for q in queries}
    ks = {q: [] for q in queries}
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for q in queries:
            ts = time.perf_counter()
            blk = ops[q].next_block()
            lat[q].append((time.perf_counter() - ts) * 1e3)
            ks[q].append((blk.filter_kernel_ms, blk.agg_kernel_ms, blk.filter_bytes, blk.agg_bytes))
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    answers = {q: ops[q].next_block() for q in queries}
    for op in ops.values():
        op.close()
    rows = sum(s.num_docs for s in gsegs)
    threads = cpu_baseline.usable_cpus()[0]
    per_q = {}
    ok = True
    for q in queries:
        k = np.asarray(ks[q], dtype=np.float64)
        fms, ams = float(k[:, 0].mean()), float(k[:, 1].mean())
        fb, ab = float(k[:, 2].mean()), float(k[:, 3].mean())
        blk = answers[q]
        d = {"p50_ms": round(float(np.median(lat[q])), 4), "groups": len(blk.groups),
             "docs_scanned": blk.stats.num_docs_scanned,
             "filter_ms": round(fms, 4), "agg_ms": round(ams, 4),
             "filter_frac": round(fb / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if fms > 0 else None,
             "agg_frac": round(ab / (ams * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if ams > 0 else None,
             "filter_bytes": int(fb), "agg_bytes": int(ab)}
        if not args.no_parity:
            p = cpu_baseline.PreparedGroupBy(qcs[q], raws)
            out = p.run(threads)
            good, why = compare_groups(blk, p.groups(out), p.sum_agg, p.hll_agg)
            good = good and out[3] == blk.stats.num_docs_scanned
            if why is None and not good:
                why = f"numDocsScanned {blk.stats.num_docs_scanned} vs {out[3]}"
            d["parity"] = "equal" if good else f"MISMATCH: {why}"
            ok &= good
        per_q[q] = d
    res = {"queries": {q: ssb.SSB_QUERIES[q] for q in queries},
           "rows_per_query": rows, "segments": len(gsegs),
           "value": round(rows * len(queries) * args.steps / elapsed / 1e9, 3), "unit": "G rows/s",
           "ms_per_pass": round(elapsed * 1e3 / args.steps, 4), "per_query": per_q}
    if not args.no_parity:
        if dist is not None:
            t = torch.tensor([1 if ok else 0], dtype=torch.int64,
                             device="cuda" if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = bool(t.item())
        res["parity"] = "checked" if ok else "MISMATCH"
    if want_cpu:
        v, th, reps, el = cpu_baseline.time_group_by([qcs[q] for q in queries], raws, threads,
                                                     min_seconds=args.cpu_seconds)
        res["cpu_baseline"] = {"value": round(v / 1e9, 4), "unit": "G rows/s", "cores": th, "kind": "port",
                               "sample": f"restatement, not Pinot: oracle/cpu_scan.c cg_run (OpenMP dense group-by, "
                                         f"{th} threads) running {'+'.join(queries)} over the same {len(raws)} "
                                         f"segments, {reps} reps in {el:.1f} s"}
    return res


def _intermediate_equal(ag, g, o, ex):
    """One function's GPU intermediate against the oracle's (exact integers; doubles 1e-9 relative, the north star's
    DOUBLE tolerance; HLL registers bit-exact)."""
    rel = 1e-9
    f = ag.function
    if f in ("distinctcounthll", "distinctcountrawhll"):
        return np.array_equal(np.asarray(g), np.asarray(o))
    if f == "count":
        return g == o
    if f == "sum":
        if ex is not None and isinstance(g, (int, np.integer)):
            return int(g) == ex
        ref = ex if ex is not None else o
        return g == o or abs(g - ref) <= rel * max(abs(ref), 1.0)
    if f in ("min", "max"):
        return g == o
    if f == "avg":
        return g[1] == o[1] and (float(g[0]) == o[0] or abs(g[0] - o[0]) <= rel * abs(o[0]))
    if f == "minmaxrange":
        return tuple(map(float, g)) == tuple(o)
    return g == o


def compare_blocks(qc, gblk, oblk, exact, scale=1):
    """A GPU results block against oracle/executor.py's over the same segments (`scale` copies of them: counts, sums
    and docs multiply; MIN / MAX / HLL do not change). Returns None when equal, else the first difference."""
    from pinot_amd.engine.reduce import trim_groups
    if gblk.stats.num_docs_scanned != oblk.stats.num_docs_scanned * scale:
        return f"numDocsScanned {gblk.stats.num_docs_scanned} vs {oblk.stats.num_docs_scanned * scale}"

    def scaled(ag, v, ex):
        if scale == 1 or ag.function not in ("count", "sum"):
            return v, ex
        return v * scale, (ex * scale if ex is not None else None)

    if not qc.group_by:
        for ag, g, o, ex in zip(qc.aggregations, gblk.results, oblk.results, exact):
            o, ex = scaled(ag, o, ex)
            if not _intermediate_equal(ag, g, o, ex):
                return f"{ag.function}: {g} vs {o} (exact {ex})"
        return None
    if getattr(gblk, "num_groups_trimmed", False):
        oblk = trim_groups(qc, oblk)
    if gblk.num_groups_limit_reached != oblk.num_groups_limit_reached:
        return "numGroupsLimitReached differs"
    if set(gblk.groups) != set(oblk.groups):
        return f"group sets differ: {len(gblk.groups)} vs {len(oblk.groups)}"
    for k, v in oblk.groups.items():
        for ag, g, o, ex in zip(qc.aggregations, gblk.groups[k], v, exact[k]):
            o, ex = scaled(ag, o, ex)
            if not _intermediate_equal(ag, g, o, ex):
                return f"group {k} {ag.function}: {g} vs {o}"
    return None


def time_config_queries(args, named, gsegs, oracle_segs, scale, rows_label):
    """The queries of one config over its resident segments: each prepared once, `warmup` + `steps` executions (p50
    wall, kernel times and algorithmic bytes per kernel from the library's HIP events), then the last block checked
    against oracle/executor.py over `oracle_segs` (x `scale` copies) outside the timed region; the oracle's own run
    time is the config's CPU baseline (numpy restatement, one thread)."""
    from oracle import executor
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.query.sql import parse
    pm = GpuInstancePlanMaker()
    rows = sum(s.num_docs for s in gsegs)
    per_q, ok, t_total, cpu_rows, cpu_s = {}, True, 0.0, 0, 0.0
    for name, sql in named.items():
        qc = parse(sql)
        op = pm.make_instance_plan(qc, gsegs)
        for _ in range(args.warmup):
            op.next_block()
        lat, fk, ak = [], [], []
        blk = None
        for _ in range(args.steps):
            ts = time.perf_counter()
            blk = op.next_block()
            lat.append((time.perf_counter() - ts) * 1e3)
            fk.append(getattr(blk, "filter_kernel_ms", 0.0) or 0.0)
            ak.append(getattr(blk, "agg_kernel_ms", 0.0) or 0.0)
        if hasattr(op, "close"):
            op.close()
        p50 = float(np.median(lat))
        t_total += float(np.sum(lat)) / 1e3
        fms, ams = float(np.mean(fk)), float(np.mean(ak))
        fb, ab = int(getattr(blk, "filter_bytes", 0) or 0), int(getattr(blk, "agg_bytes", 0) or 0)
        d = {"p50_ms": round(p50, 4), "G_rows_per_s": round(rows / (p50 * 1e-3) / 1e9, 2),
             "docs_scanned": blk.stats.num_docs_scanned, "filter_ms": round(fms, 4), "agg_ms": round(ams, 4),
             "filter_bytes": fb, "agg_bytes": ab,
             "filter_frac": round(fb / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if fms > 0 else None,
             "agg_frac": round(ab / (ams * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if ams > 0 else None,
             "fused": bool(getattr(blk, "fused", False))}
        if qc.group_by:
            d["groups"] = len(blk.groups)
        if not args.no_parity:
            t0 = time.perf_counter()
            oblk, exact = executor.execute(qc, oracle_segs)
            cpu_s += time.perf_counter() - t0
            cpu_rows += sum(s.num_docs for s in oracle_segs)
            why = compare_blocks(qc, blk, oblk, exact, scale)
            d["parity"] = "equal" if why is None else f"MISMATCH: {why}"
            ok &= why is None
        per_q[name] = d
    res = {"rows_per_query": rows, "segments": len(gsegs), "unit": "G rows/s",
           "value": round(rows * len(named) * args.steps / t_total / 1e9, 3) if t_total else None,
           "ms_per_pass": round(t_total * 1e3 / args.steps, 4), "per_query": per_q, "layout": rows_label}
    if not args.no_parity:
        res["parity"] = "checked" if ok else "MISMATCH"
        res["cpu_baseline"] = {"value": round(cpu_rows / cpu_s / 1e9, 4) if cpu_s else None, "unit": "G rows/s",
                               "cores": 1, "kind": "port",
                               "sample": f"oracle/executor.py (numpy restatement of the CPU server path, one thread): "
                                         f"each query once over {len(oracle_segs)} segment(s) of the same data "
                                         f"({cpu_rows // max(len(named), 1)} rows per query), {cpu_s:.1f} s"}
    return res


def run_c1(args):
    """BASELINE configs[0]: the BenchmarkQueries segment (P/BenchmarkQueries.java:81-137; 10M rows,
    EXP(0.001), tools/bq.py), every query of the GPU subset, one GPU; parity against oracle/executor.py on the segment."""
    from pinot_amd.engine.segment import GpuSegment
    from tools import bq
    raws = bq.make_segments(args.c1_rows, 1, "EXP(0.001)")
    gsegs = [GpuSegment(r) for r in raws]
    try:
        res = time_config_queries(args, bq.QUERIES, gsegs, raws, 1, f"{args.c1_rows} rows, 1 segment, EXP(0.001)")
    finally:
        for g in gsegs:
            g.destroy()
    return res


def run_c4(args):
    """BASELINE configs[3]: 5-predicate AND / OR / NOT over Roaring inverted indexes, 100 x 10M = 1B
    rows (10 distinct generated segments each resident 10 times), selectivity 0.01 %-50 %, COUNT(*) and SUM(M);
    parity against oracle/executor.py over the 10 distinct segments (counts, sums and docs x 10)."""
    from pinot_amd.engine.segment import GpuSegment
    from tools import c4
    distinct = [c4.make_segment(i, num_rows=args.c4_rows) for i in range(args.c4_distinct)]
    gsegs = [GpuSegment(r) for _ in range(args.c4_copies) for r in distinct]
    named = {f"sel={sel} {agg}": c4.query(sel, agg) for sel in c4.SELECTIVITIES for agg in ("COUNT(*)", "SUM(M)")}
    try:
        res = time_config_queries(args, named, gsegs, distinct, args.c4_copies,
                                  f"{len(gsegs)} x {args.c4_rows} rows ({args.c4_distinct} distinct x {args.c4_copies})")
    finally:
        for g in gsegs:
            g.destroy()
    return res


# kernel families of one query execution: a plain filter launch, a filter launch that aggregated its own tiles
# (fused), and a separate aggregation launch.
#
# Traffic (MI355X_MICROARCH.md §HBM: FETCH_SIZE tallies a wide stream's 128-B requests at 64 B; other shapes are to be
# calibrated in the kernel's own access pattern). profiles/<round>_traffic.json holds each family's raw FETCH_SIZE
# and WRITE_SIZE per launch and `stream_factor` = the streamed bytes / FETCH_SIZE of the SAME filter kernel run as a
# stream-only probe (PHIP_FILTER_PROBE=1 PHIP_FUSE=0: its bytes are known exactly). A launch's traffic is then its
# streamed bytes (exact) + the rest of its FETCH at face value (gathers: 64-B requests) + WRITE -- never below the
# bytes it must stream. `touched` (profiles/<round>_touched.json, tools/touched_lines.py) is the floor of a gathering
# launch at 64-B line granularity: the streamed bytes + every line holding a matched doc's id or value.
def roofline(kstats, queries, traffic, touched, layout, steps):
    """Per-kernel achieved bandwidth on algorithmic bytes; headline = the kernel with the most time per step
    (launches per step x mean launch time)."""
    kernels = {}
    fams = {"filter_kernel": lambda s: (s[0] if not s[4] else 0.0, s[2], s[5], False),
            "fused_filter_agg": lambda s: (s[0] if s[4] else 0.0, s[2], s[5], True),
            "agg_kernel": lambda s: (s[1], s[3], 0, True)}
    tj = (traffic or {}).get("per_launch", {}).get(layout) or {}
    factor = (traffic or {}).get("stream_factor")
    tq = ((touched or {}).get("per_query") or {}).get(layout) or {}
    for name, pick in fams.items():
        ms, by, sb, per_q, floor = [], [], [], {}, []
        for q in queries:
            xs = [pick(s) for s in kstats[q]]
            for t, b, st, gathers in xs:
                if t > 0:
                    ms.append(t)
                    by.append(b)
                    sb.append(st)
                    if q in tq:
                        floor.append(st + (tq[q]["touched_bytes"] if gathers else 0))
            per_q[q] = round(float(np.mean([x[0] for x in xs])), 4)
        if not ms:
            continue
        launches = len(ms)
        mean_ms = sum(ms) / launches
        mean_b = sum(by) / launches
        mean_stream = sum(sb) / launches
        ach = mean_b / (mean_ms * 1e-3) / 1e9 if mean_ms > 0 else 0.0
        tr = tj.get(name)
        tsel, method = None, None
        if isinstance(tr, dict):
            if factor:
                gather_fetch = max(0.0, tr["fetch_raw"] - mean_stream / factor)
                tsel = int(mean_stream + gather_fetch + tr["write"])
                method = f"streamed bytes (exact) + FETCH beyond stream/{factor:.3f} (calibrated) + WRITE"
            else:
                tsel = tr["x2"] if name == "filter_kernel" else tr["raw"]
                method = "uncalibrated: FETCH x2 + WRITE (streaming) / FETCH + WRITE (gathering)"
        fl = int(sum(floor) / len(floor)) if len(floor) == launches else None

        def frac(b):
            return round(b / (mean_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if b else None
        kernels[name] = {"ms_per_launch": round(mean_ms, 4), "launches_per_step": round(launches / steps, 3),
                         "ms_per_step": round(mean_ms * launches / steps, 4),
                         "alg_bytes_per_launch": int(mean_b), "stream_bytes_per_launch": int(mean_stream),
                         "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                         "traffic_per_launch": tsel, "traffic_frac": frac(tsel), "traffic_method": method,
                         "traffic_fetch_raw": tr.get("fetch_raw") if isinstance(tr, dict) else None,
                         "touched_floor_per_launch": fl, "touched_frac": frac(fl),
                         "time_share": None, "per_query_ms": per_q}
    tot = sum(k["ms_per_step"] for k in kernels.values()) or 1.0
    for k in kernels.values():
        k["time_share"] = round(k["ms_per_step"] / tot, 3)
    if not kernels:  # every tile of this rank's segments pruned (a sorted-layout shard outside the dates): no launch
        return {"bound": "hbm", "kernel": None, "achieved": 0.0, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": 0.0,
                "traffic": None, "kernels": {}, "bytes": "no kernel launched on this rank: its segments' tiles were "
                                                         "all pruned by the sorted index"}
    dom = max(kernels, key=lambda k: kernels[k]["ms_per_step"])
    d = kernels[dom]
    return {"bound": "hbm", "kernel": dom, "achieved": d["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": d["frac"], "traffic": d["traffic_per_launch"], "kernels": kernels,
            "bytes": "algorithmic bytes per launch (phip_result.filter_bytes / agg_bytes, SURVEY.md §8d) / mean "
                     "launch time from HIP events on the library's stream; dominant = most device time per step "
                     "(launches x mean); traffic = PMC HBM bytes per launch, calibrated (traffic_method); "
                     "touched_floor = streamed bytes + the 64-B lines a launch's gathers must move"}


def spawn_ranks(n):
    """`bench.py --gpus N` without torchrun: N rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set as torch.distributed.run sets them, rendezvous on 127.0.0.1), started before this process touches
    the GPU. Rank 0's stdout (the JSON line) passes through; every rank's stderr is inherited. Returns the exit
    code: the first non-zero one (the other ranks are then stopped), else 0."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr, start_new_session=False))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log(f"rank {procs.index(p)} exited with {code}: stopping the other ranks")
                for q in live:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = ranks. Under torchrun it must equal WORLD_SIZE; without torchrun, N > 1 starts N rank "
                         "processes here (one per GPU, before any GPU call) and prints rank 0's line")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--segs-per-gpu", type=int, default=0,
                    help="segments (6M rows each) per GPU: default 100 at one GPU (C2: SF100), 125 at N > 1 "
                         "(N = 8: SF1000, BASELINE C5); Q1.x always runs over 100 of them per GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--c5", default="auto", choices=["auto", "on", "off"],
                    help="also time the C5 query over all segments of all ranks (auto: at N > 1)")
    ap.add_argument("--queries", default="Q1.1,Q1.2,Q1.3")
    ap.add_argument("--group-by", default="c3,c5",
                    help="group-by legs over the headline layout's segments (BASELINE C3 = SSB Q2.x-Q4.x, C5's "
                         "query), each parity-checked against oracle/cpu_scan.c; '' = none")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline time per leg")
    ap.add_argument("--configs", default="c1,c4",
                    help="the other BASELINE configs as legs at N = 1 (c1: BenchmarkQueries 10M rows; c4: 1B-row "
                         "inverted-index sweep), each parity-checked against oracle/executor.py; '' = none")
    ap.add_argument("--c1-rows", type=int, default=10_000_000)
    ap.add_argument("--c4-rows", type=int, default=10_000_000)
    ap.add_argument("--c4-distinct", type=int, default=10)
    ap.add_argument("--c4-copies", type=int, default=10)
    ap.add_argument("--layout", default="both", choices=["sorted", "unsorted", "both"],
                    help="headline = sorted (SURVEY.md §8d C2); both also measures the unsorted layout")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the check of every query's answer against oracle/cpu_scan.c on the same segments")
    ap.add_argument("--timed-markers", action="store_true",
                    help="keep the library's per-kernel timing markers in the timed steps (default: off, as a server "
                         "runs; the roofline's kernel durations come from a separate pass either way)")
    ap.add_argument("--no-concurrent", action="store_true",
                    help="skip the concurrent-client leg (profiling runs: every kernel launch is then sequential, so "
                         "rocprof averages equal the timed leg's)")
    ap.add_argument("--traffic-json", default=latest_profile("traffic"),
                    help="HBM bytes per launch per kernel and layout from rocprofv3 --pmc passes (tools/traffic.py)")
    ap.add_argument("--touched-json", default=latest_profile("touched"),
                    help="64-B lines the gathers touch per query and layout (tools/touched_lines.py)")
    ap.add_argument("--seed", type=int, default=42)
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        raise SystemExit(spawn_ranks(args.gpus))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        # (--dist-backend gloo with more ranks than GPUs rehearses the N > 1 path on a one-GPU box: ranks share a
        # device and the merges stage through the host; the driver's runs use RCCL, one rank per GPU)
        local_rank = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank)
        dist.init_process_group(args.dist_backend)
    from pinot_amd import _lib
    import ctypes
    dev = (ctypes.c_int32 * 1)(local_rank)
    _lib.check(_lib.load().phip_init(dev, 1))

    from pinot_amd.query.sql import parse
    from tools import ssb

    queries = args.queries.split(",")
    seg_per_gpu = args.segs_per_gpu or (100 if world == 1 else 125)
    head_segs = min(100, seg_per_gpu)  # C2's SF100 per GPU: weak scaling of the headline at exactly 100 per rank
    want_c5 = args.c5 == "on" or (args.c5 == "auto" and world > 1)
    gb_legs = [g for g in args.group_by.split(",") if g]
    for g in gb_legs:
        if g not in GROUP_BY_LEGS:
            raise SystemExit(f"unknown group-by leg {g}")
    cols = ssb.columns_for(queries + (["C5"] if want_c5 else []))
    gb_cols = ssb.columns_for(queries + (["C5"] if want_c5 else []) + [q for g in gb_legs for q in GROUP_BY_LEGS[g]])
    qcs = {q: parse(ssb.SSB_QUERIES[q]) for q in queries}
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("queries") == queries and tj.get("sf") == 100:
                traffic = tj
        except Exception:
            traffic = None
    touched = None
    if os.path.exists(args.touched_json):
        try:
            with open(args.touched_json) as f:
                tj = json.load(f)
            if tj.get("queries") == queries and tj.get("sf") == 100:
                touched = tj
        except Exception:
            touched = None
    layouts = (["sorted", "unsorted"] if world == 1 else ["sorted"]) if args.layout == "both" else [args.layout]
    want_cpu = not args.no_cpu_baseline and rank == 0 and world == 1
    results = {}
    for li, layout in enumerate(layouts):
        t0 = time.time()
        gsegs, all_raws = load_layout(ssb, seg_per_gpu, world, rank, gb_cols if li == 0 else cols, args.seed, layout,
                                      keep_host=not args.no_parity or (want_cpu and li == 0))
        load_s = time.time() - t0
        log(f"rank {rank}: {layout} layout loaded ({len(gsegs)} segments, {len(gb_cols if li == 0 else cols)} "
            f"columns) in {load_s:.1f} s")
        head = gsegs[:head_segs]
        raws = all_raws[:head_segs]
        rows_per_rank = sum(s.num_docs for s in head)
        elapsed, lat, kstats, answers, concurrent, kstats_ext = run_layout(args, dist, queries, qcs, head, torch)
        rf = roofline(kstats_ext, queries, traffic, touched, layout, args.steps)
        rf["timing"] = ("kernel durations from HIP events recorded by each launch's dispatch packet (PHIP_EXT_EVENTS=1, "
                        "the timed steps' executions repeated outside the timed region, whose own steps ran without "
                        "timing markers)")
        rb = roofline(kstats, queries, traffic, touched, layout, args.steps) if args.timed_markers else None
        if rb and rb["kernel"]:
            rf["bracket_events"] = {"kernel": rb["kernel"], "frac": rb["frac"],
                                    "ms_per_launch": rb["kernels"][rb["kernel"]]["ms_per_launch"],
                                    "note": "the timed steps' own barrier-marker events"}
        res = {"elapsed": elapsed, "rows_per_rank": rows_per_rank, "load_s": load_s, "nseg": len(head),
               "lat": lat, "roofline": rf}
        if concurrent:
            res["concurrent"] = {"value": round(rows_per_rank * len(queries) * args.steps / concurrent / 1e9, 3),
                                 "unit": "G rows/s", "ms_per_step": round(concurrent * 1e3 / args.steps, 4),
                                 "note": f"{'+'.join(queries)} as {len(queries)} concurrent client threads (one per "
                                         f"query, own execution lane each), {args.steps} executions each; not `value`"}
        if not args.no_parity:
            res["parity"] = check_parity(queries, qcs, answers, raws, dist, torch)
        log(f"rank {rank}: {layout} Q1.x timed, parity {res.get('parity', (None,))[0]}")
        if li == 0:
            for g in gb_legs:  # C3 / C5 over this rank's resident segments, parity-checked, own cpu_baseline
                res[g] = run_group_by(args, dist, g, gsegs, all_raws, torch, want_cpu)
                log(f"rank {rank}: group-by leg {g}: {res[g]['value']} G rows/s, parity {res[g].get('parity')}")
        if want_c5 and li == 0:
            qc5 = parse(ssb.SSB_QUERIES["C5"])
            el5, lat5, blk5 = run_c5(args, dist, qc5, gsegs, torch)
            rows5 = sum(s.num_docs for s in gsegs) * world
            res["c5_merged"] = {"query": ssb.SSB_QUERIES["C5"], "rows": rows5, "segments": len(gsegs) * world,
                         "value": round(rows5 * args.steps / el5 / 1e9, 3), "unit": "G rows/s",
                         "ms_per_query": round(el5 * 1e3 / args.steps, 3),
                         "p50_latency_ms": round(float(np.median(lat5)), 3), "groups": len(blk5.groups),
                         "merge": ("distributed_block: node-global dictionaries, dense partial tables all-reduced "
                                   f"in place over {'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} "
                                   "(int64 SUM + uint8 MAX for this query)") if dist is not None
                         else "one GPU: no exchange"}
            if not args.no_parity:
                res["c5_merged"]["parity"] = check_merged_group_by(qc5, blk5, all_raws, dist)
        for s in gsegs:
            s.destroy()
        del all_raws
        if not (want_cpu and li == 0):
            del raws
        if want_cpu and li == 0:
            from oracle import cpu_baseline
            v, threads, reps, el, _ = cpu_baseline.time_queries([qcs[q] for q in queries], raws, min_seconds=10.0)
            res["cpu"] = {"value": round(v / 1e9, 4), "unit": "G rows/s", "cores": threads, "kind": "port",
                          "sample": f"restatement, not Pinot: oracle/cpu_scan.c (OpenMP C restatement of the CPU "
                                    f"server path, {threads} threads = the usable CPUs: "
                                    f"{cpu_baseline.usable_cpus()[1]}) running "
                                    f"{'+'.join(queries)} over the same {len(raws)} x {ssb.SEGMENT_ROWS}-row "
                                    f"SF{head_segs} {layout} segments, {reps} reps in {el:.1f} s"}
            del raws
        results[layout] = res

    cfg_legs = {}
    if world == 1:
        for leg in [c for c in args.configs.split(",") if c]:
            t0 = time.time()
            cfg_legs[leg] = {"c1": run_c1, "c4": run_c4}[leg](args)
            log(f"config leg {leg}: {cfg_legs[leg]['value']} G rows/s, parity {cfg_legs[leg].get('parity')} "
                f"({time.time() - t0:.0f} s)")
    if rank != 0:
        dist.destroy_process_group()
        return
    head = results[layouts[0]]

    def summary(r):
        total_rows = r["rows_per_rank"] * world * len(queries) * args.steps
        return total_rows / r["elapsed"] / 1e9, r["elapsed"] * 1e3 / args.steps

    value, ms_per_step = summary(head)
    out = {
        "metric": "rows scanned/s (G) + p50 query latency, SSB flattened SF100/SF1000, 1-8 GPU",
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
        "config": {"workload": f"SSB SF{head['nseg']} flattened lineorder per GPU, {head['nseg']} segments x "
                               f"{ssb.SEGMENT_ROWS} rows, queries {'+'.join(queries)}"
                               + (f" (each rank holds {seg_per_gpu} segments of an SF{seg_per_gpu * world} table; "
                                  f"C5 runs over all of them)" if want_c5 else ""),
                   "layout": f"{layouts[0]}" + (" by LO_ORDERDATE (SURVEY.md §8d C2)" if layouts[0] == "sorted" else ""),
                   "rows_per_gpu": head["rows_per_rank"],
                   "parallelism": (f"segment-sharded x{world}, partial tables all-reduced over "
                                   f"{'RCCL' if args.dist_backend == 'nccl' else args.dist_backend}") if world > 1
                   else "one GPU (no collective)"},
        "p50_latency_ms": {q: round(float(np.median(head["lat"][q])), 3) for q in queries},
        "roofline": head["roofline"],
        "load_s": round(head["load_s"], 1),
    }
    if "cpu" in head:
        out["cpu_baseline"] = head["cpu"]
    if "concurrent" in head:
        out["concurrent_clients"] = head["concurrent"]
    if not args.no_parity:
        ok = all(results[l]["parity"][0] for l in layouts) and all(head[g].get("parity") == "checked" for g in gb_legs) \
            and head.get("c5_merged", {}).get("parity", "checked") == "checked"
        out["parity"] = "checked" if ok else "MISMATCH"
        out["parity_detail"] = {
            "against": "oracle/cpu_scan.c on the same segments, every rank, outside the timed region: exact int64 "
                       "SUM == the CPU's (integer-valued) double SUM, numDocsScanned == its matched docs; group-by "
                       "legs (c3, c5): the same group keys, exact SUMs and HLL registers as cpu_scan.c's dense "
                       "group-by (per-query detail under each leg)",
            **{l: results[l]["parity"][1] for l in layouts}}
    for g in gb_legs:
        out[g] = head[g]
    for leg, r in cfg_legs.items():
        out[leg] = r
        if not args.no_parity and r.get("parity") != "checked":
            out["parity"] = "MISMATCH"
    if "c5_merged" in head:  # the C5 query over every rank's segments, merged across ranks (N > 1 / --c5 on)
        out["c5_merged"] = head["c5_merged"]
    if len(layouts) > 1:
        r = results[layouts[1]]
        v2, ms2 = summary(r)
        out["unsorted_layout"] = {"value": round(v2, 3), "unit": "G rows/s", "ms_per_step": round(ms2, 3),
                                  "p50_latency_ms": {q: round(float(np.median(r["lat"][q])), 3) for q in queries},
                                  "roofline": r["roofline"]}
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
