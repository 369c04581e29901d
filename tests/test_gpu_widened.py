"""Shapes the GPU path widened to in round 5, each against the oracle:

  * GROUP BY of more than four columns (DictionaryBasedGroupKeyGenerator has no column cap,
    pinot-core/.../groupby/DictionaryBasedGroupKeyGenerator.java:105-186): up to eight columns in the mixed-radix
    key, dense and hash tables, with the device trim and numGroupsLimit;
  * DISTINCTCOUNTHLL functions of different log2m in one query (each DistinctCountHLLAggregationFunction keeps its
    own log2m, DistinctCountHLLAggregationFunction.java:105-145): aggregation-only, group-by, filtered;
  * the shapes the library still refuses reach the configured CPU plan maker (GpuPlanWithCpuFallback) instead of
    failing the query.
"""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker, UnsupportedOnGpu
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wide_segments(gpu_lib):
    from pinot_amd.engine.segment import GpuSegment
    rng = np.random.default_rng(2024)
    raws = []
    for k, n in enumerate((20_000, 33_333, 7_001)):
        c = SegmentCreator(f"wide{k}", inverted_index_columns=["c3"])
        for j, card in enumerate((3, 4, 5, 2, 6, 3, 7, 2)):
            c.add_column(f"c{j}", DataType.INT, rng.integers(0, card, n) * 10 + j)
        c.add_column("s", DataType.STRING, np.array([f"s{x}" for x in rng.integers(0, 9, n)]))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        c.add_column("u", DataType.INT, rng.integers(0, 50_000, n))
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        raws.append(c.build())
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


def _check_groups(qc, blk, oblk, ex):
    from tests.test_gpu_parity import _assert_intermediates_equal
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert set(blk.groups) == set(oblk.groups)
    for k, v in oblk.groups.items():
        _assert_intermediates_equal(qc.aggregations, blk.groups[k], v, ex[k])


WIDE = [
    "SELECT c0, c1, c2, c3, c4, COUNT(*), SUM(m) FROM t GROUP BY c0, c1, c2, c3, c4 LIMIT 100000",
    "SELECT c0, c1, c2, c3, c4, c5, c6, c7, SUM(m), MAX(u) FROM t WHERE f < 60 "
    "GROUP BY c0, c1, c2, c3, c4, c5, c6, c7 LIMIT 100000",
    "SELECT s, c1, c2, c4, c6, COUNT(*), DISTINCTCOUNTHLL(u) FROM t WHERE c3 = 13 "
    "GROUP BY s, c1, c2, c4, c6 LIMIT 100000",
    "SELECT s, c1, c2, c4, c6, COUNT(*), DISTINCTCOUNTHLL(u) FROM t WHERE c3 = 33 "  # no doc matches: no group
    "GROUP BY s, c1, c2, c4, c6 LIMIT 100000",
    "SELECT c0, c1, c2, c3, c4, u, SUM(m) FROM t WHERE f < 5 GROUP BY c0, c1, c2, c3, c4, u LIMIT 100000",  # hash
    "SELECT c0, c1, c2, c3, c4, c5, SUM(m) FROM t GROUP BY c0, c1, c2, c3, c4, c5 ORDER BY SUM(m) DESC LIMIT 10",
]


@pytest.mark.parametrize("sql", WIDE)
def test_gpu_group_by_more_than_four_columns(sql, wide_segments):
    raws, segs = wide_segments
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
    try:
        blk = op.next_block()
    finally:
        op.close()
    oblk, ex = executor.execute(qc, raws)
    if qc.order_by:
        from pinot_amd.engine.reduce import reduce_blocks
        from tests import fixtures
        assert fixtures.rows_match(reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [oblk]).rows)
    else:
        _check_groups(qc, blk, oblk, ex)


def test_gpu_group_by_five_columns_num_groups_limit(wide_segments):
    """numGroupsLimit cuts the five-column key per segment in first-seen order, as the oracle does."""
    from tests.test_gpu_limits import _check
    raws, segs = wide_segments
    qc = parse("SELECT c0, c1, c2, c4, u, COUNT(*), SUM(m) FROM t GROUP BY c0, c1, c2, c4, u LIMIT 100000")
    gblk = GpuInstancePlanMaker(num_groups_limit=500).make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws, num_groups_limit=500)
    assert oblk.num_groups_limit_reached
    _check(qc, gblk, oblk, exact)


MIXED = [
    "SELECT DISTINCTCOUNTHLL(u, 10), DISTINCTCOUNTHLL(m), DISTINCTCOUNTHLL(s, 5), COUNT(*) FROM t WHERE f < 70",
    "SELECT c1, DISTINCTCOUNTHLL(u, 12), DISTINCTCOUNTHLL(m, 6), SUM(m) FROM t GROUP BY c1 LIMIT 100",
    "SELECT c1, c2, DISTINCTCOUNTHLL(u), DISTINCTCOUNTHLL(m, 11) FROM t WHERE f >= 10 GROUP BY c1, c2 LIMIT 100",
    "SELECT DISTINCTCOUNTHLL(u, 9) FILTER (WHERE f < 30), DISTINCTCOUNTHLL(m) FROM t",
]


@pytest.mark.parametrize("sql", MIXED)
def test_gpu_mixed_log2m_hll(sql, wide_segments):
    from tests.test_gpu_parity import _assert_intermediates_equal
    raws, segs = wide_segments
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
    try:
        blk = op.next_block()
    finally:
        op.close()
    oblk, ex = executor.execute(qc, raws)
    if qc.group_by:
        _check_groups(qc, blk, oblk, ex)
        for v in blk.groups.values():
            for ag, x in zip(qc.aggregations, v):
                if ag.function == "distinctcounthll":
                    assert len(x) == 1 << ag.log2m
    else:
        assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
        _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
        for ag, x in zip(qc.aggregations, blk.results):  # registers of each function's own size
            if ag.function == "distinctcounthll":
                assert len(x) == 1 << ag.log2m


class _Cpu:
    def __init__(self):
        self.calls = 0

    def make_instance_plan(self, query, segments):
        self.calls += 1
        return type("P", (), {"next_block": lambda s: "cpu", "close": lambda s: None})()


@pytest.mark.parametrize("sql", [
    "SELECT DISTINCTCOUNTHLL(u, 10), DISTINCTCOUNTHLL(u, 8) FROM t WHERE f < 50",  # one column, two log2m
    "SELECT c0, c1, c2, c3, c4, c5, c6, c7, s, COUNT(*) FROM t GROUP BY c0, c1, c2, c3, c4, c5, c6, c7, s LIMIT 10",
])
def test_gpu_refusals_reach_the_cpu_plan_maker(sql, wide_segments):
    """A shape the library refuses (PHIP_ERR_UNSUPPORTED) raises UnsupportedOnGpu without a CPU plan maker and is
    answered by the configured one with it -- never a failed query (the Java plan maker keeps its CPU operator)."""
    raws, segs = wide_segments
    qc = parse(sql)
    with pytest.raises(UnsupportedOnGpu):
        op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
        try:
            op.next_block()
        finally:
            op.close()
    cpu = _Cpu()
    op = GpuInstancePlanMaker(cpu_plan_maker=cpu).make_instance_plan(qc, segs)
    assert op.next_block() == "cpu" and cpu.calls == 1
    op.close()


def test_gpu_plan_deadline_and_cancel(wide_segments):
    """phip_plan_set_deadline / phip_plan_cancel (QueryContext.getEndTimeMs, BaseSingleBlockCombineOperator.java:
    133-144): a past deadline fails the execution with PHIP_ERR_TIMEOUT, a far one runs it, a cancel is sticky; the
    query option timeoutMs runs a query with time left."""
    import ctypes
    import time

    from pinot_amd import _lib
    from pinot_amd.engine.plan import QueryCancelledError, QueryTimeoutError
    raws, segs = wide_segments
    lib = _lib.load()
    for sql in ("SELECT SUM(m), COUNT(*) FROM t WHERE f < 40", "SELECT c1, c2, SUM(m) FROM t GROUP BY c1, c2 LIMIT 100"):
        op = GpuInstancePlanMaker().make_instance_plan(parse(sql), segs)
        op.run_raw(prepare_only=True)
        res = ctypes.POINTER(_lib.Result)()
        _lib.check(lib.phip_plan_set_deadline(op._plan, 1))  # 1 ms after the epoch: long past
        with pytest.raises(QueryTimeoutError):
            _lib.check(lib.phip_plan_execute(op._plan, ctypes.byref(res)))
        _lib.check(lib.phip_plan_set_deadline(op._plan, int(time.time() * 1000) + 60_000))
        _lib.check(lib.phip_plan_execute(op._plan, ctypes.byref(res)))
        lib.phip_result_free(res)
        _lib.check(lib.phip_plan_cancel(op._plan))
        with pytest.raises(QueryCancelledError):
            _lib.check(lib.phip_plan_execute(op._plan, ctypes.byref(res)))
        op.close()
    qc = parse("SET timeoutMs = 60000; SELECT c1, SUM(m) FROM t WHERE f < 40 GROUP BY c1 LIMIT 100")
    blk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
    oblk, ex = executor.execute(qc, raws)
    _check_groups(qc, blk, oblk, ex)
