"""Group-by results in one round trip (runtime.cpp one_trip / aggregate.hip group_gather_mapped_kernel): when neither
numGroupsLimit nor the trim can apply and the key space's rows fit the mapped landing area, the group count, keys,
values, exact sums and HLL registers come back through mapped host memory without a wait for the count. Both paths
(PHIP_GB_ONE_TRIP_MAX=0 forces the two-trip one, PHIP_GB_ONE_TRIP_HLL=0 for plans with registers) must give the
oracle's groups: every aggregation kind, registers bit-exact, several keys,
an empty result, a key space right at the landing area's size limit, and a plan executed repeatedly (the landing
area is reused)."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.query.sql import parse
from pinot_amd.spi import DataType

pytestmark = pytest.mark.gpu

QUERIES = [
    "SELECT g, COUNT(*), SUM(v), MIN(d), MAX(v), AVG(d), MINMAXRANGE(v) FROM t WHERE f < 40 GROUP BY g LIMIT 1000",
    "SELECT g, s, SUM(v), COUNT(*) FROM t GROUP BY g, s LIMIT 100000",
    "SELECT s, SUM(d) FROM t WHERE f > 1000 GROUP BY s LIMIT 100",                     # nothing matches
    "SELECT g, SUM(v) FILTER (WHERE f < 10), COUNT(*) FROM t GROUP BY g LIMIT 1000",
    "SELECT g, s, MAX(d) FROM t WHERE s <> 'b3' GROUP BY g, s ORDER BY g, s DESC LIMIT 5",
    "SELECT g, DISTINCTCOUNTHLL(v), SUM(d) FROM t WHERE f < 70 GROUP BY g LIMIT 1000",   # registers packed 4 a word
    "SELECT g, s, DISTINCTCOUNTHLL(f, 4), DISTINCTCOUNTHLL(s, 4), COUNT(*) FROM t GROUP BY g, s LIMIT 100000",
]


@pytest.fixture(scope="module")
def segs(gpu_lib):
    from pinot_amd.engine.segment import GpuSegment
    rng = np.random.default_rng(5)
    raws = []
    for k, n in enumerate((40_000, 2048 * 3 + 1)):
        c = SegmentCreator(f"ot{k}")
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        c.add_column("g", DataType.INT, rng.integers(0, 30, n))
        c.add_column("s", DataType.STRING, np.array([f"b{x}" for x in rng.integers(0, 12, n)]))
        c.add_column("v", DataType.LONG, rng.integers(-10 ** 12, 10 ** 12, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.normal(0, 100, n), 3))
        raws.append(c.build())
    gs = [GpuSegment(r) for r in raws]
    yield raws, gs
    for g in gs:
        g.destroy()


def _run(sql, segs, monkeypatch, max_bytes, reps=1):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    monkeypatch.delenv("PHIP_GB_ONE_TRIP_HLL", raising=False)
    if max_bytes is None:
        monkeypatch.delenv("PHIP_GB_ONE_TRIP_MAX", raising=False)
    elif max_bytes == "no-hll":
        monkeypatch.delenv("PHIP_GB_ONE_TRIP_MAX", raising=False)
        monkeypatch.setenv("PHIP_GB_ONE_TRIP_HLL", "0")
    else:
        monkeypatch.setenv("PHIP_GB_ONE_TRIP_MAX", str(max_bytes))
    raws, gs = segs
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, gs)
    blks = [op.next_block() for _ in range(reps)]
    op.close()
    return qc, blks, executor.execute(qc, raws)


@pytest.mark.parametrize("max_bytes", [None, 0, "no-hll"])
@pytest.mark.parametrize("sql", QUERIES)
def test_gpu_group_one_trip(sql, max_bytes, segs, monkeypatch):
    from pinot_amd.engine.reduce import reduce_blocks
    from tests import fixtures
    from tests.test_gpu_limits import _check
    qc, blks, (oblk, exact) = _run(sql, segs, monkeypatch, max_bytes, reps=3)
    for blk in blks:
        if not qc.order_by:
            _check(qc, blk, oblk, exact)
        assert fixtures.rows_match(sorted(reduce_blocks(qc, [blk]).rows) if not qc.order_by else
                                   reduce_blocks(qc, [blk]).rows,
                                   sorted(reduce_blocks(qc, [oblk]).rows) if not qc.order_by else
                                   reduce_blocks(qc, [oblk]).rows)


@pytest.mark.parametrize("slack", [-1, 0])
def test_gpu_group_one_trip_size_limit(slack, segs, monkeypatch):
    """The landing area holds 64 + key space x (8 + 16 x aggregations) bytes (key space g x s = 30 x 12 = 360, two
    aggregations): at that size and one byte below it (the one-trip and the two-trip path) the oracle's groups."""
    from tests.test_gpu_limits import _check
    need = 64 + 30 * 12 * (8 + 16 * 2)
    sql = "SELECT g, s, SUM(v), COUNT(*) FROM t GROUP BY g, s LIMIT 100000"
    qc, blks, (oblk, exact) = _run(sql, segs, monkeypatch, need + slack)
    _check(qc, blks[0], oblk, exact)


@pytest.fixture(scope="module")
def wide(gpu_lib):
    from pinot_amd.engine.segment import GpuSegment
    rng = np.random.default_rng(17)
    n = 120_000
    c = SegmentCreator("otw")
    c.add_column("a", DataType.INT, rng.integers(0, 20_000, n))   # ~20K groups: above trimSize 5000, below 100K
    c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
    c.add_column("f", DataType.INT, rng.integers(0, 100, n))
    raw = c.build()
    g = GpuSegment(raw)
    yield [raw], [g]
    g.destroy()


@pytest.mark.parametrize("max_bytes", [None, 0])
@pytest.mark.parametrize("sql", ["SELECT a, SUM(m) FROM t WHERE f < 90 GROUP BY a ORDER BY SUM(m) DESC LIMIT 10",
                                 "SELECT a, COUNT(*) FROM t GROUP BY a ORDER BY a DESC LIMIT 7"])
def test_gpu_group_one_trip_trim_fallback(sql, max_bytes, wide, monkeypatch):
    """A plan whose trim can apply goes one trip speculatively; with more groups than trimSize the compaction and
    gather run again into device buffers and the device trim keeps its top 5000: the oracle's rows either way."""
    from pinot_amd.engine.reduce import reduce_blocks, trim_groups
    from tests import fixtures
    qc, blks, (oblk, exact) = _run(sql, wide, monkeypatch, max_bytes, reps=2)
    for blk in blks:
        assert blk.num_groups_trimmed
        o = trim_groups(qc, oblk)
        assert fixtures.rows_match(reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [o]).rows)
