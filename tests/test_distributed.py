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
        merged = trim_groups(qc, allreduce_block(part, dist))
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
