"""Multi-GPU server path on the GPU: node-global dictionaries, dense partial tables handed out by
phip_plan_execute_partial, merged across ranks (engine/distributed.allreduce_partial_table) and finished by
phip_plan_finish. The box has one GPU, so the two "ranks" are two processes on cuda:0 over gloo (tensors
staged through the host); the in-place RCCL path on the library's device buffers runs at world size 1
below. Every merged block must equal the oracle over all segments."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-9
QUERIES = [
    "SELECT g, h, COUNT(*), SUM(m), SUM(d), MIN(d), MAX(m), AVG(h), DISTINCTCOUNTHLL(h) FROM t WHERE m > -500000000 "
    "GROUP BY g, h ORDER BY g, h LIMIT 100000",
    "SELECT g, SUM(big), COUNT(*) FROM t GROUP BY g ORDER BY g LIMIT 100000",  # int64 on one rank, double on the other
    "SELECT h, MINMAXRANGE(d), SUM(m * h) FROM t WHERE h < 4 GROUP BY h ORDER BY h LIMIT 100000",
    "SELECT g, h, SUM(m) FROM t GROUP BY g, h ORDER BY SUM(m) DESC LIMIT 3",  # trim after the merge
    # FILTER + GROUP BY: the infos are programs of one plan, its partial table merges like any other
    "SELECT g, COUNT(*) FILTER(WHERE h = 1), SUM(m) FILTER(WHERE d > 0), MAX(d), COUNT(*) FROM t "
    "GROUP BY g ORDER BY g LIMIT 100000",
]


def _segments():
    from pinot_amd.segment.creator import SegmentCreator
    from pinot_amd.spi import DataType
    rng = np.random.default_rng(23)
    out = []
    for k in range(4):
        n = 30000 + 7000 * k
        c = SegmentCreator(f"d{k}")
        c.add_column("g", DataType.STRING, np.array([f"key{x:03d}" for x in rng.integers(5 * k, 40 + 6 * k, n)]))
        c.add_column("h", DataType.INT, rng.integers(0, 7 + k, n))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.normal(0, 100, n), 4))
        big = rng.integers(2 ** 60, 2 ** 61, n) if k % 2 == 1 else rng.integers(0, 1000, n)
        c.add_column("big", DataType.LONG, big)
        out.append(c.build())
    return out


def _close(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return np.array_equal(np.asarray(a), np.asarray(b))
    if isinstance(a, tuple):
        return all(_close(x, y) for x, y in zip(a, b))
    if isinstance(a, float) or isinstance(b, float):
        a, b = float(a), float(b)
        return a == b or abs(a - b) <= REL * max(abs(a), abs(b))
    return a == b


def _compare(merged, whole, qc):
    assert merged.stats.num_docs_scanned == whole.stats.num_docs_scanned
    assert merged.stats.num_total_docs == whole.stats.num_total_docs
    assert merged.stats.num_segments_processed == whole.stats.num_segments_processed
    assert set(merged.groups) == set(whole.groups), (len(merged.groups), len(whole.groups))
    for k, v in whole.groups.items():
        for x, y in zip(merged.groups[k], v):
            assert _close(x, y), (k, x, y)


def _worker(rank, world, port, q, limit, errs):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import executor
        from pinot_amd.engine.distributed import distributed_block, register_global_dictionaries
        from pinot_amd.engine.plan import GpuInstancePlanMaker
        from pinot_amd.engine.reduce import trim_groups
        from pinot_amd.engine.segment import GpuSegment
        from pinot_amd.query.sql import parse
        raws = _segments()
        mine = [GpuSegment(s) for i, s in enumerate(raws) if i % world == rank]
        qc = parse(q)
        qc.options["minServerGroupTrimSize"] = 20
        register_global_dictionaries(mine, [e.name for e in qc.group_by], dist)
        op = GpuInstancePlanMaker(num_groups_limit=limit).make_instance_plan(qc, mine)
        fb = GpuInstancePlanMaker(num_groups_limit=limit, device_trim=False).make_instance_plan(qc, mine)
        part = op.execute_partial()
        assert (part is None) == (limit < 1000), "dense partial expected unless numGroupsLimit is hit"
        if part is not None:
            # the table is the caller's until finish / abandon: another execution of the plan is refused
            from pinot_amd._lib import PhipError
            with pytest.raises(PhipError):
                op.execute_partial()
            op.abandon_partial()
        merged = trim_groups(qc, distributed_block(op, dist, fallback_op=fb))
        whole = trim_groups(qc, executor.execute(qc, raws, num_groups_limit=limit)[0])
        if "DESC LIMIT 3" in q:
            assert len(merged.groups) == 20 and len(whole.groups) == 20
        _compare(merged, whole, qc)
        op.close()
        fb.close()
        for s in mine:
            s.destroy()
    except Exception as e:  # surfaced to the parent
        import traceback
        errs.put(f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("limit", [100_000, 50], ids=["dense", "limit-fallback"])
@pytest.mark.parametrize("q", QUERIES)
def test_gpu_distributed_world2(q, limit, gpu_lib):
    import torch.multiprocessing as mp
    if limit < 1000 and "h, MINMAXRANGE" in q:
        pytest.skip("fewer groups than the limit")
    ctx = mp.get_context("spawn")
    errs = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, limit, errs)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not errs.empty():
        msgs.append(errs.get())
    assert not msgs, msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_gpu_partial_inplace_rccl_world1(gpu_lib):
    """RCCL all-reduce directly on the library's partial-table buffers (torch tensors aliasing them through
    __cuda_array_interface__), then phip_plan_finish: equals phip_plan_execute on the same plan."""
    import torch
    import torch.distributed as dist
    from pinot_amd.engine.distributed import (allreduce_partial_table, partial_tensors, register_global_dictionaries,
                                              unregister_global_dictionaries)
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    raws = _segments()
    segs = [GpuSegment(s) for s in raws]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        qc = parse(QUERIES[0])
        register_global_dictionaries(segs, ["g", "h"], dist)
        op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
        ref = op.next_block()
        part = op.execute_partial()
        assert part is not None and part.global_keys == 1
        table, hll = partial_tensors(part)
        assert table.is_cuda and table.data_ptr() == part.table
        kinds = [part.row_kinds[r] for r in range(part.num_rows)]
        kinds2, stats = allreduce_partial_table(table, hll, kinds, list(part.stats), dist)
        torch.cuda.synchronize()
        assert kinds2 == kinds
        for i, x in enumerate(stats):
            part.stats[i] = x
        blk = op.finish(part)
        assert blk.stats.num_docs_scanned == ref.stats.num_docs_scanned
        assert set(blk.groups) == set(ref.groups)
        for k, v in ref.groups.items():
            for x, y in zip(blk.groups[k], v):
                assert _close(x, y), (k, x, y)
        op.close()
    finally:
        unregister_global_dictionaries(["g", "h"])
        dist.destroy_process_group()
        for s in segs:
            s.destroy()


# ---- BASELINE config C5 through the sharded path ---------------------------------------------------------------
def _c5_worker(rank, world, port, errs):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import executor
        from pinot_amd.engine.distributed import distributed_block, register_global_dictionaries
        from pinot_amd.engine.plan import GpuInstancePlanMaker
        from pinot_amd.engine.segment import GpuSegment
        from pinot_amd.query.sql import parse
        from tools import ssb
        qc = parse(ssb.SSB_QUERIES["C5"])
        raws = ssb.make_segments(1, ssb.columns_for(["C5"]), segment_rows=1_000_000)  # SSB SF1, 6 segments
        mine = [GpuSegment(s) for i, s in enumerate(raws) if i % world == rank]
        register_global_dictionaries(mine, [e.name for e in qc.group_by], dist)
        op = GpuInstancePlanMaker().make_instance_plan(qc, mine)
        fb = GpuInstancePlanMaker(device_trim=False).make_instance_plan(qc, mine)
        calls = []
        orig = dist.all_reduce

        def counted(t, op=None, group=None, **kw):
            calls.append((str(op), str(t.dtype)))
            return orig(t, op=op if op is not None else dist.ReduceOp.SUM, group=group, **kw)
        dist.all_reduce = counted
        merged = distributed_block(op, dist, fallback_op=fb)
        dist.all_reduce = orig
        # the device path: the shape check (int64 MAX), then the table -- counts + exact SUM + statistics as one
        # int64 SUM, the HLL registers as one uint8 MAX
        assert len(calls) == 3 and sorted(c[1] for c in calls) == ["torch.int64", "torch.int64", "torch.uint8"], calls
        whole, _ = executor.execute(qc, raws)
        assert len(whole.groups) == 35  # 7 years x the 5 nations of AMERICA
        _compare(merged, whole, qc)
        op.close()
        fb.close()
        for s in mine:
            s.destroy()
    except Exception as e:  # surfaced to the parent
        import traceback
        errs.put(f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


def test_gpu_c5_sharded_world2(gpu_lib):
    """BASELINE C5 (DISTINCTCOUNTHLL(LO_CUSTKEY) + SUM(LO_REVENUE - LO_SUPPLYCOST) GROUP BY D_YEAR, C_NATION) over
    SSB SF1 split across two ranks: global dictionaries -> dense partial tables -> merge -> finish equals the
    oracle over all six segments (registers and integer sums bit-exact)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errs = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c5_worker, args=(r, 2, port, errs)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=110)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not errs.empty():
        msgs.append(errs.get())
    assert not msgs, msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


# ---- aggregation-only queries: the one-group partial table merged on the device ---------------------------------
AGG_QUERIES = [
    "SELECT COUNT(*), SUM(m), SUM(h) FROM t WHERE h < 5",  # every row an int64 sum: one SUM collective
    "SELECT MIN(d), MAX(m), SUM(d), AVG(h), DISTINCTCOUNTHLL(h), MINMAXRANGE(d), COUNT(*) FROM t WHERE m > 0",
    "SELECT SUM(big), COUNT(*) FROM t",  # int64 on one rank, double on the other (the overflow bound is per GPU)
]


def _agg_worker(rank, world, port, q, errs):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import executor
        from pinot_amd.engine.distributed import distributed_block
        from pinot_amd.engine.plan import GpuInstancePlanMaker
        from pinot_amd.engine.segment import GpuSegment
        from pinot_amd.query.sql import parse
        raws = _segments()
        mine = [GpuSegment(s) for i, s in enumerate(raws) if i % world == rank]
        qc = parse(q)
        op = GpuInstancePlanMaker().make_instance_plan(qc, mine)
        for _ in range(2):  # (the plan executes again after a merge)
            merged = distributed_block(op, dist)
            whole, _ = executor.execute(qc, raws)
            assert merged.stats.num_docs_scanned == whole.stats.num_docs_scanned
            assert merged.stats.num_total_docs == whole.stats.num_total_docs
            assert merged.stats.num_segments_matched == whole.stats.num_segments_matched
            for x, y in zip(merged.results, whole.results):
                assert _close(x, y), (q, x, y)
        op.close()
        for s in mine:
            s.destroy()
    except Exception as e:  # surfaced to the parent
        import traceback
        errs.put(f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("q", AGG_QUERIES)
def test_gpu_distributed_aggregation_world2(q, gpu_lib):
    """Aggregation-only queries over two ranks through phip_plan_execute_partial's one-group table (rows, statistics,
    u8 HLL registers) -> merge -> phip_plan_finish: equal to the oracle over all segments (AggregationResultsBlockMerger
    semantics: sums add, MIN / MAX / registers take the extreme, statistics add)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errs = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agg_worker, args=(r, 2, port, q, errs)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not errs.empty():
        msgs.append(errs.get())
    assert not msgs, msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.mark.parametrize("q", AGG_QUERIES[:2])
def test_gpu_aggregation_partial_inplace_rccl_world1(q, gpu_lib):
    """RCCL all-reduces directly on an aggregation plan's device partial (rows + statistics, u8 registers), then
    phip_plan_finish: equals phip_plan_execute on the same plan; an all-int64 query is ONE collective."""
    import torch.distributed as dist
    from pinot_amd.engine.distributed import allreduce_aggregation_partial
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    raws = _segments()
    segs = [GpuSegment(s) for s in raws]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        qc = parse(q)
        op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
        ref = op.next_block()
        part = op.execute_partial()
        assert part is not None and part.num_groups == 1 and part.stats_dev and part.hll_u8 == 1
        calls = []
        orig = dist.all_reduce

        def counted(t, op=None, group=None, **kw):
            calls.append(str(t.dtype))
            return orig(t, op=op if op is not None else dist.ReduceOp.SUM, group=group, **kw)
        dist.all_reduce = counted
        allreduce_aggregation_partial(part, dist)
        dist.all_reduce = orig
        if q == AGG_QUERIES[0]:
            assert calls == ["torch.int64"], calls
        blk = op.finish(part)
        assert blk.stats.num_docs_scanned == ref.stats.num_docs_scanned
        assert blk.stats.num_segments_matched == ref.stats.num_segments_matched
        for x, y in zip(blk.results, ref.results):
            assert _close(x, y), (x, y)
        op.close()
    finally:
        dist.destroy_process_group()
        for s in segs:
            s.destroy()
