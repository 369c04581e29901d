"""World-size-2 gloo tests of the cross-GPU exchange step (pinot_amd/engine/distributed.py).

Each rank owns half of the segments (the multi-GPU sharding of bench.py), computes its partial block
(here with the CPU oracle: these tests run without a GPU) and merges it with allreduce_block; the
merged block must equal the block over all segments computed in one process, exactly for counts,
integer sums, min/max, group keys and HLL registers, and within 1e-9 relative for DOUBLE sums.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

QUERIES = [
    "SELECT COUNT(*), SUM(m), MIN(d), MAX(m), AVG(d), DISTINCTCOUNTHLL(m), MINMAXRANGE(h) FROM t WHERE h <> 3",
    "SELECT g, h, COUNT(*), SUM(m), SUM(d), MIN(d), MAX(m), DISTINCTCOUNTHLL(g) FROM t WHERE m > 0 "
    "GROUP BY g, h ORDER BY g, h LIMIT 100000",
    "SELECT g, COUNT(*) FROM t WHERE h = 5 GROUP BY g ORDER BY g LIMIT 100000",
    # server-level trim AFTER the cross-GPU merge (reduce.trim_groups; minServerGroupTrimSize = 20 below)
    "SELECT g, h, SUM(m), COUNT(*) FROM t GROUP BY g, h ORDER BY SUM(m) DESC LIMIT 4",
]
REL = 1e-9


def _segments():
    from pinot_amd.segment.creator import SegmentCreator
    from pinot_amd.spi import DataType
    rng = np.random.default_rng(11)
    out = []
    for k in range(4):
        n = 5000 + 700 * k
        c = SegmentCreator(f"s{k}")
        # key domains differ per segment, so the per-rank key sets differ
        c.add_column("g", DataType.STRING, np.array([f"k{x}" for x in rng.integers(3 * k, 20 + 4 * k, n)]))
        c.add_column("h", DataType.INT, rng.integers(0, 6 + k, n))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        c.add_column("d", DataType.DOUBLE, rng.random(n) * 100)
        out.append(c.build())
    return out


def _close(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return np.array_equal(np.asarray(a), np.asarray(b))
    if isinstance(a, tuple):
        return all(_close(x, y) for x, y in zip(a, b))
    if isinstance(a, float) or isinstance(b, float):
        return a == b or abs(a - b) <= REL * max(abs(a), abs(b))
    return a == b


def _worker(rank, world, port, q, errs):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import executor
        from pinot_amd.engine.distributed import allreduce_block
        from pinot_amd.query.sql import parse
        segs = _segments()
        from pinot_amd.engine.reduce import trim_groups
        qc = parse(q)
        qc.options["minServerGroupTrimSize"] = 20
        mine = [s for i, s in enumerate(segs) if i % world == rank]
        part, _ = executor.execute(qc, mine)
        calls = _count_collectives(dist)
        merged = trim_groups(qc, allreduce_block(part, dist))
        # one float64 SUM + one int64 MAX per merge, whatever the functions (DISTINCTCOUNTHLL, MIN, AVG ...), and for a
        # group-by one int64 SUM of the key-space bound that picks the dense merge over the record merge
        want = [("max", "torch.int64"), ("sum", "torch.float64")] + ([("sum", "torch.int64")] if qc.group_by else [])
        assert sorted(calls) == sorted(want), calls
        whole = trim_groups(qc, executor.execute(qc, segs)[0])
        if "DESC LIMIT 4" in q:
            assert len(whole.groups) == 20 and getattr(merged, "num_groups_trimmed", False)
        assert merged.stats.num_docs_scanned == whole.stats.num_docs_scanned
        assert merged.stats.num_total_docs == whole.stats.num_total_docs
        if qc.group_by:
            assert set(merged.groups) == set(whole.groups), "group keys differ"
            for k, v in whole.groups.items():
                for x, y in zip(merged.groups[k], v):
                    assert _close(x, y), (k, x, y)
        else:
            for x, y in zip(merged.results, whole.results):
                assert _close(x, y), (x, y)
    except Exception as e:  # surfaced to the parent
        errs.put(f"rank {rank}: {type(e).__name__}: {e}")
    finally:
        dist.destroy_process_group()


def _count_collectives(dist):
    """Records (op, dtype) of every all_reduce the merge issues from here on."""
    calls = []
    orig = dist.all_reduce

    def counted(t, op=None, group=None, **kw):
        calls.append(("max" if op == dist.ReduceOp.MAX else ("sum" if op in (None, dist.ReduceOp.SUM) else str(op)),
                      str(t.dtype)))
        return orig(t, op=op if op is not None else dist.ReduceOp.SUM, group=group, **kw)
    dist.all_reduce = counted
    return calls


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("q", QUERIES)
def test_allreduce_block_world2_gloo(q):
    ctx = mp.get_context("spawn")
    errs = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, errs)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not errs.empty():
        msgs.append(errs.get())
    assert not msgs, msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_allreduce_block_single_process_is_identity():
    from oracle import executor
    from pinot_amd.engine.distributed import allreduce_block
    from pinot_amd.query.sql import parse
    qc = parse(QUERIES[0])
    blk, _ = executor.execute(qc, _segments()[:1])
    assert allreduce_block(blk) is blk


# ---- device-resident merge: node-global dictionaries + dense partial tables (engine/distributed.py) --------
# CPU restatement of the library's partial-table encoding (pinot_amd/csrc/dev_common.h f64_ordered; row layout
# of include/pinot_hip.h phip_partial), used to feed the product's all-reduce with oracle partials.
def _ordered(d):
    u = int(np.array([d], "<f8").view(np.uint64)[0])
    return (~u & (2 ** 64 - 1)) if u >> 63 else u | (1 << 63)


def _unordered(u):
    u &= 2 ** 64 - 1
    v = (u & ((1 << 63) - 1)) if u >> 63 else (~u & (2 ** 64 - 1))
    return float(np.array([v], np.uint64).view("<f8")[0])


def _s64(u):
    return u - (1 << 64) if u >= (1 << 63) else u


PARTIAL_Q = ("SELECT g, h, COUNT(*), SUM(m), SUM(d), MIN(d), MAX(m), DISTINCTCOUNTHLL(h) FROM t WHERE m > -500000000 "
             "GROUP BY g, h ORDER BY g, h LIMIT 100000")


def _partial_worker(rank, world, port, f64_rank, errs):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import executor
        from pinot_amd import _lib
        from pinot_amd.engine.distributed import allreduce_partial_table, global_dictionary
        from pinot_amd.query.sql import parse
        segs = _segments()
        mine = [s for i, s in enumerate(segs) if i % world == rank]
        qc = parse(PARTIAL_Q)
        gd = {}
        for col in ("g", "h"):
            dt, vals = global_dictionary(mine, col, dist)
            whole_vals = sorted({v.item() if hasattr(v, "item") else v
                                 for s in segs for v in executor.OracleSegment(s).dictionary(col)})
            if col == "g":
                got = [bytes(r).rstrip(b"\0").decode() for r in vals]
            else:
                got = [int(x) for x in vals]
            assert got == whole_vals, (col, got[:5], whole_vals[:5])
            gd[col] = got
        cg, ch = len(gd["g"]), len(gd["h"])
        G = cg * ch
        ig = {v: i for i, v in enumerate(gd["g"])}
        ih = {v: i for i, v in enumerate(gd["h"])}
        part, _ = executor.execute(qc, mine)
        m = 1 << qc.aggregations[5].log2m
        kinds = [_lib.ROW_COUNT, _lib.ROW_COUNT, _lib.ROW_SUM_I64, _lib.ROW_SUM_F64, _lib.ROW_MIN, _lib.ROW_MAX,
                 _lib.ROW_HLL]
        if rank == f64_rank:
            kinds[2] = _lib.ROW_SUM_F64  # this GPU's overflow bound chose double for SUM(m)
        table = np.zeros((7, G), np.int64)
        table[4, :] = _s64(2 ** 64 - 1)  # MIN identity (atomicMin from the top)
        hll = np.zeros((G, m), np.int32)
        for (g, h), v in part.groups.items():
            k = ig[g] + cg * ih[h]  # mixed radix, column 0 least significant
            table[0, k] = v[0]
            if kinds[2] == _lib.ROW_SUM_F64:
                table[2, k] = np.array([float(v[1])], "<f8").view(np.int64)[0]
            else:
                table[2, k] = v[1]
            table[3, k] = np.array([v[2]], "<f8").view(np.int64)[0]
            table[4, k] = _s64(_ordered(v[3]))
            table[5, k] = _s64(_ordered(float(v[4])))
            hll[k] = np.asarray(v[5], np.int32)
        s = part.stats
        stats = [s.num_docs_scanned, s.num_entries_scanned_in_filter, s.num_entries_scanned_post_filter,
                 s.num_total_docs, s.num_segments_processed, s.num_segments_matched]
        t, th = torch.from_numpy(table), torch.from_numpy(hll.reshape(-1))
        # the SUM_F64 flags as distributed_block exchanges them with its shape check
        f = torch.tensor([1 if k == _lib.ROW_SUM_F64 else 0 for k in kinds], dtype=torch.int64)
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        calls = _count_collectives(dist)
        kinds2, stats2 = allreduce_partial_table(t, th, kinds, stats, dist, any_f64=f.tolist())
        # one collective per (reduce operator, type): int64 SUM (counts, exact sums, statistics), float64 SUM,
        # int64 MAX (MIN rows reversed), uint8 MAX (HLL registers)
        assert sorted(calls) == sorted([("sum", "torch.int64"), ("sum", "torch.float64"), ("max", "torch.int64"),
                                        ("max", "torch.uint8")]), calls
        whole, _ = executor.execute(qc, segs)
        assert stats2[0] == whole.stats.num_docs_scanned and stats2[3] == whole.stats.num_total_docs
        want_f64 = f64_rank is not None
        assert kinds2[2] == (_lib.ROW_SUM_F64 if want_f64 else _lib.ROW_SUM_I64), kinds2
        table, hll = t.numpy(), th.numpy().reshape(G, m)
        present = {int(k) for k in np.nonzero(table[0])[0]}
        assert len(present) == len(whole.groups)
        for (g, h), v in whole.groups.items():
            k = ig[g] + cg * ih[h]
            assert k in present
            assert table[0, k] == v[0]
            s_m = float(table[2:3, k].view("<f8")[0]) if want_f64 else int(table[2, k])
            assert _close(s_m, v[1] if not want_f64 else float(v[1])), (s_m, v[1])
            assert _close(float(table[3:4, k].view("<f8")[0]), v[2])
            assert _unordered(int(table[4, k])) == v[3]
            assert _unordered(int(table[5, k])) == float(v[4])
            assert np.array_equal(hll[k].astype(np.uint8), np.asarray(v[5]))
    except Exception as e:  # surfaced to the parent
        import traceback
        errs.put(f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("f64_rank", [None, 1], ids=["int64", "mixed-sum-kinds"])
def test_allreduce_partial_table_world2_gloo(f64_rank):
    """The product's device-table merge (allreduce_partial_table) over the library's row encodings: counts,
    exact and double sums, MIN / MAX on the order-preserving u64 image, HLL registers, statistics, and the
    per-GPU int64/double disagreement of a SUM row; keys in node-global dictionaries (global_dictionary)."""
    ctx = mp.get_context("spawn")
    errs = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_partial_worker, args=(r, 2, port, f64_rank, errs)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not errs.empty():
        msgs.append(errs.get())
    assert not msgs, msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_float_order_keys_round_trip():
    """Node-global FLOAT / DOUBLE dictionaries sort in Double.compare order (-0.0 < 0.0, NaN last)."""
    from pinot_amd.engine.distributed import _order_keys, _values_of_keys
    from pinot_amd.spi import DataType
    for dt, code in ((DataType.DOUBLE, "<f8"), (DataType.FLOAT, "<f4")):
        v = np.array([3.5, -0.0, 0.0, -2.25, np.inf, -np.inf, np.nan, 1e-30], code)
        k = _order_keys(v, dt)
        order = np.argsort(k, kind="stable")
        got = _values_of_keys(k[order], dt)
        want = np.array([-np.inf, -2.25, -0.0, 0.0, 1e-30, 3.5, np.inf, np.nan], code)
        assert np.array_equal(got.view(np.uint64 if code == "<f8" else np.uint32),
                              want.view(np.uint64 if code == "<f8" else np.uint32))


class _StubPlan:
    """A group-by operator's partial-table protocol without a GPU: execute_partial hands out a table (or raises on
    the failing rank), and while one is pending the plan refuses to run, as libpinot_hip.so does
    (runtime.cpp: PHIP_ERR_INVALID until phip_plan_finish / phip_plan_abandon_partial)."""

    def __init__(self, fail_partial=False, fail_block=False):
        from types import SimpleNamespace
        self.query = SimpleNamespace(group_by=["g"])
        self.fail_partial, self.fail_block = fail_partial, fail_block
        self.pending = False
        self.abandoned = 0

    def execute_partial(self):
        if self.pending:
            raise RuntimeError("pending partial table")
        if self.fail_partial:
            raise ValueError("execution failed on this rank")
        self.pending = True
        from types import SimpleNamespace
        return SimpleNamespace(global_keys=0, num_groups=0, num_rows=0)  # (local key order: records merge)

    def abandon_partial(self):
        self.pending = False
        self.abandoned += 1

    def next_block(self):
        if self.pending:
            raise RuntimeError("pending partial table")
        if self.fail_block:
            raise ValueError("record path failed on this rank")
        from pinot_amd.engine.results import ExecutionStatistics, GroupByResultsBlock
        return GroupByResultsBlock([], ["g"], {}, ExecutionStatistics(), False)


def _failure_worker(rank, world, port, where, errs):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pinot_amd import _lib
        from pinot_amd.engine.distributed import distributed_block
        _lib.load = lambda *a, **k: None  # (no library on a CPU host: the protocol is what is tested)
        op = _StubPlan(fail_partial=(where == "partial" and rank == 0), fail_block=(where == "records" and rank == 0))
        try:
            distributed_block(op, dist)
            raise AssertionError("every rank must raise when one rank fails")
        except (ValueError, RuntimeError) as e:
            assert (rank == 0) == isinstance(e, ValueError), repr(e)
        assert not op.pending, "a surviving rank's plan must not stay blocked behind its partial table"
        if rank != 0 or where == "records":
            assert op.abandoned == 1
        op.fail_partial = op.fail_block = False
        distributed_block(op, dist)  # the plans execute again afterwards, on every rank
    except Exception as e:  # surfaced to the parent
        import traceback
        errs.put(f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("where", ["partial", "records"])
def test_distributed_block_rank_failure_world2_gloo(where):
    """when one rank's execution raises (its partial table, or the record-merge fallback), every rank
    raises instead of waiting in a collective, and every surviving rank hands its pending partial table back, so
    its plan runs again afterwards."""
    ctx = mp.get_context("spawn")
    errs = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failure_worker, args=(r, 2, port, where, errs)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not errs.empty():
        msgs.append(errs.get())
    assert not msgs, msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _null_worker(rank, world, port, errs):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pinot_amd.engine.distributed import allreduce_block
        from pinot_amd.engine.results import AggregationResultsBlock, ExecutionStatistics
        from pinot_amd.query.sql import parse
        q = parse("SET enableNullHandling = true; SELECT SUM(a), MIN(a), AVG(a), COUNT(a), MAX(b), SUM(c) FROM t")
        # rank 0 aggregated no non-null value of a / b; rank 1 has values; c is null everywhere
        if rank == 0:
            res = [None, None, None, 0, None, None]
        else:
            res = [7, -2.5, (7, 2), 2, 11.0, None]
        blk = AggregationResultsBlock(q.aggregations, res, ExecutionStatistics(3, 0, 3, 10, 1, 1))
        out = allreduce_block(blk, dist)
        assert out.results == [7, -2.5, (7, 2), 2, 11.0, None], out.results
        assert out.stats.num_docs_scanned == 6 and out.stats.num_total_docs == 20
    except Exception as e:  # surfaced to the parent
        import traceback
        errs.put(f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


def test_allreduce_block_null_intermediates_world2_gloo():
    """enableNullHandling across ranks: a rank's null intermediate adds nothing (the nullable functions' merge keeps
    the other side), and a function null on every rank stays null."""
    ctx = mp.get_context("spawn")
    errs = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_null_worker, args=(r, 2, port, errs)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not errs.empty():
        msgs.append(errs.get())
    assert not msgs, msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
