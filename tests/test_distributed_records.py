"""World-size-2 gloo tests of the columnar record merge (distributed._merge_records_columnar): the exchange a large
key space takes instead of the dense table -- key / value / register matrices all-gathered over the communicator and
merged by key in rank order -- and of the dense record merge (the node-global dictionaries' table). Each rank computes
its partial block with the CPU oracle over its half of the segments; the merged block must equal the oracle's block
over all segments (exact keys, counts, integer sums, min / max, HLL registers, null keys and null intermediates under
enableNullHandling; doubles within 1e-9 relative). Raw DOUBLE keys -0.0 and 0.0 are two groups on both paths (the
reference keys reals by their bits), and DISTINCTCOUNTHLL functions of different log2m merge on both paths and in an
aggregation-only block."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.test_distributed import _close, _free_port

QUERIES = [
    "SELECT h, l, COUNT(*), SUM(m), SUM(d), MIN(d), MAX(m), AVG(d), MINMAXRANGE(m), DISTINCTCOUNTHLL(m) FROM t "
    "WHERE m > -500000000 GROUP BY h, l LIMIT 1000000",
    "SELECT d2, COUNT(*), DISTINCTCOUNTHLL(h, 8), DISTINCTCOUNTHLL(l, 10) FROM t GROUP BY d2 LIMIT 1000000",
    "SET enableNullHandling = true; SELECT n, h, COUNT(*), SUM(x), MIN(x), COUNT(x), AVG(x) FROM t "
    "GROUP BY n, h LIMIT 1000000",
    "SELECT g, h, COUNT(*), SUM(m) FROM t GROUP BY g, h LIMIT 1000000",   # STRING key: the object merge
    "SELECT z, h, COUNT(*), SUM(m), MAX(d) FROM t GROUP BY z, h LIMIT 1000000",  # raw DOUBLE key with -0.0 and 0.0
]
AGG_QUERIES = ["SELECT COUNT(*), DISTINCTCOUNTHLL(h, 8), DISTINCTCOUNTHLL(l, 10), SUM(m) FROM t"]


def _segments():
    from pinot_amd.segment.creator import SegmentCreator
    from pinot_amd.spi import DataType
    rng = np.random.default_rng(23)
    out = []
    for k in range(4):
        n = 3000 + 500 * k
        c = SegmentCreator(f"r{k}", no_dictionary_columns=["z"])
        c.add_column("g", DataType.STRING, np.array([f"k{x}" for x in rng.integers(2 * k, 15 + 3 * k, n)]))
        c.add_column("h", DataType.INT, rng.integers(0, 40 + 10 * k, n))
        c.add_column("l", DataType.LONG, rng.integers(-30, 30, n) * 10 ** 10)
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.random(n) * 100, 3))
        c.add_column("d2", DataType.DOUBLE, np.round(rng.normal(0, 3, n), 1))
        c.add_column("n", DataType.INT, rng.integers(0, 25, n), nulls=rng.random(n) < 0.2)
        c.add_column("x", DataType.LONG, rng.integers(0, 1000, n), nulls=rng.random(n) < (0.5 if k % 2 else 0.05))
        c.add_column("z", DataType.DOUBLE, np.array([-0.0, 0.0, 1.25, -3.5])[rng.integers(0, 4, n)])
        out.append(c.build())
    return out


def _worker(rank, world, port, q, errs, max_dense=8):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import executor
        from pinot_amd.engine.distributed import allreduce_block
        from pinot_amd.query.sql import parse
        segs = _segments()
        qc = parse(q)
        mine = [s for i, s in enumerate(segs) if i % world == rank]
        part, _ = executor.execute(qc, mine)
        objs = []
        orig = dist.all_gather_object
        dist.all_gather_object = lambda *a, **kw: (objs.append(1), orig(*a, **kw))[1]
        merged = allreduce_block(part, dist, max_dense_groups=max_dense)  # 8: every query's key space is larger
        dist.all_gather_object = orig
        if max_dense == 8 and qc.group_by:
            # numeric keys merge as columns (no Python objects over the wire); the STRING key keeps the object merge
            assert (len(objs) > 0) == ("SELECT g," in q), objs
        whole, _ = executor.execute(qc, segs)
        if "GROUP BY z" in q:
            zs = {k[0] for k in whole.groups}
            assert len(zs) == 4 and 0.0 in zs and any(np.signbit(float(z)) and float(z) == 0 for z in zs), zs
        if not qc.group_by:
            assert len(merged.results) == len(whole.results)
            for x, y in zip(merged.results, whole.results):
                assert _close(x, y), (x, y)
            return
        assert merged.stats.num_docs_scanned == whole.stats.num_docs_scanned
        assert merged.num_groups_limit_reached == whole.num_groups_limit_reached
        assert set(merged.groups) == set(whole.groups), "group keys differ"
        for k, v in whole.groups.items():
            for x, y in zip(merged.groups[k], v):
                assert (x is None) == (y is None), (k, x, y)
                if y is not None:
                    assert _close(x, y), (k, x, y)
    except Exception as e:  # surfaced to the parent
        import traceback
        errs.put(f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


CASES = [pytest.param(q, 8, id=f"columnar-{i}") for i, q in enumerate(QUERIES)] + \
    [pytest.param(q, 1 << 22, id=f"dense-{i}") for i, q in enumerate(QUERIES + AGG_QUERIES)]


@pytest.mark.parametrize("q,max_dense", CASES)
def test_record_merge_world2_gloo(q, max_dense):
    ctx = mp.get_context("spawn")
    errs = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, errs, max_dense)) for r in range(2)]
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
