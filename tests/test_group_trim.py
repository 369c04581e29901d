"""Server-level group trim: ORDER BY <aggregation> keeps max(5 * limit, 5000) groups.

Reference: GroupByUtils.createIndexedTableForCombineOperator (pinot-core/.../util/GroupByUtils.java:96-140)
sizes the combine's IndexedTable with trimSize = getTableCapacity(limit, minServerGroupTrimSize) (:55-58);
IndexedTable.finish keeps the top trimSize records by the ORDER BY (TableResizer.getTopRecords). The
records tied at the trim boundary are heap-order dependent in the reference; the device keeps the lowest
group key, so the tests below assert the boundary property (every kept value orders before every dropped
one) plus exact values, and exact top-k sets where the order values are distinct.
"""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuCombineOperator, plan_aggregations
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType


def _spec(sql, **options):
    qc = parse(sql)
    qc.options.update(options)
    op = object.__new__(GpuCombineOperator)
    op.query = qc
    op.prims, op.mapping = plan_aggregations(qc.aggregations)
    return op._trim_spec(), op


def test_trim_spec_rules():
    from pinot_amd import _lib
    (agg, desc, trim, _k, _t), op = _spec("SELECT k, SUM(m) FROM t GROUP BY k ORDER BY SUM(m) DESC LIMIT 10")
    assert agg >= 0 and (desc, trim) == (1, 5000)
    (agg, desc, trim, keys, _t), _ = _spec("SELECT a, b, SUM(m) FROM t GROUP BY a, b ORDER BY b, a DESC LIMIT 10")
    assert (agg, trim, keys) == (-1, 5000, [2, -1])
    (agg, desc, trim, _k, _t), _ = _spec("SELECT k, COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) LIMIT 2000")
    assert (agg >= 0, desc, trim) == (True, 0, 10000)
    (agg, desc, trim, _k, _t), _ = _spec("SELECT k, MAX(m) FROM t GROUP BY k ORDER BY MAX(m) DESC LIMIT 10",
                                         minServerGroupTrimSize=100)
    assert trim == 100
    # mixed ORDER BY: general terms (TableResizer extractors), least significant last
    (agg, _d, trim, keys, terms), op = _spec("SELECT k, SUM(m), AVG(m) FROM t GROUP BY k ORDER BY SUM(m), k DESC, "
                                             "AVG(m) DESC LIMIT 10")
    s_sum = op.mapping[0][1]
    s_avg = op.mapping[1][1]
    assert (agg, trim, keys) == (-1, 5000, [])
    assert terms == [(_lib.ORDER_VALUE, s_sum, 0, 0), (_lib.ORDER_GROUP_KEY, 0, 0, 1),
                     (_lib.ORDER_AVG, s_avg[0], s_avg[1], 1)]
    (_a, _d, _t, _k, terms), op = _spec("SELECT k, MINMAXRANGE(m) FROM t GROUP BY k ORDER BY MINMAXRANGE(m) LIMIT 10")
    assert terms == [(_lib.ORDER_RANGE, op.mapping[0][1][0], op.mapping[0][1][1], 0)]
    # DISTINCTCOUNTHLL: its cardinality estimate, computed from the registers on the device
    (_a, _d, _t, _k, terms), op = _spec("SELECT k, DISTINCTCOUNTHLL(m) FROM t GROUP BY k ORDER BY DISTINCTCOUNTHLL(m), "
                                        "k LIMIT 10")
    assert terms == [(_lib.ORDER_HLL, op.mapping[0][1], 0, 0), (_lib.ORDER_GROUP_KEY, 0, 0, 0)]
    # no trim: disabled, a serialized HLL (DISTINCTCOUNTRAWHLL), no ORDER BY
    for sql, opts in (("SELECT k, SUM(m) FROM t GROUP BY k ORDER BY SUM(m) DESC LIMIT 10", {"minServerGroupTrimSize": 0}),
                      ("SELECT k, DISTINCTCOUNTRAWHLL(m) FROM t GROUP BY k ORDER BY DISTINCTCOUNTRAWHLL(m), k LIMIT 10",
                       {}),
                      ("SELECT k, SUM(m) FROM t GROUP BY k LIMIT 10", {})):
        assert _spec(sql, **opts)[0] == (-1, 0, 0, [], []), sql


def _segments(n_segs=2, n=200_003, card=60_000, seed=4):
    rng = np.random.default_rng(seed)
    out = []
    for s in range(n_segs):
        c = SegmentCreator(f"trim{s}")
        c.add_column("k", DataType.INT, rng.integers(0, card, n))
        c.add_column("k2", DataType.INT, rng.integers(0, 40_000, n))
        c.add_column("m", DataType.LONG, rng.integers(0, 2 ** 40, n))
        c.add_column("q", DataType.INT, rng.integers(0, 50, n))
        out.append(c.build())
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("sql,exact_set", [
    ("SELECT k, SUM(m) FROM t GROUP BY k ORDER BY SUM(m) DESC LIMIT 10", True),
    ("SELECT k, MIN(m), COUNT(*) FROM t WHERE q < 40 GROUP BY k ORDER BY MIN(m) LIMIT 1500", True),
    ("SELECT k, COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) DESC LIMIT 20", False),  # many ties
    ("SELECT k, k2, SUM(m) FROM t GROUP BY k, k2 ORDER BY SUM(m) DESC LIMIT 100", True),  # > 2^26 keys: hash table
])
def test_gpu_device_trim(gpu_lib, sql, exact_set):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    raws = _segments()
    segs = [GpuSegment(r) for r in raws]
    try:
        qc = parse(sql)
        blk = GpuInstancePlanMaker(num_groups_limit=10 ** 9).make_instance_plan(qc, segs).next_block()
        oblk, _ = executor.execute(qc, raws, num_groups_limit=10 ** 9)
        trim = max(5 * qc.limit, 5000)
        assert len(oblk.groups) > trim
        assert blk.num_groups_trimmed and len(blk.groups) == trim
        # every kept group carries the oracle's exact intermediates
        for k, v in blk.groups.items():
            assert k in oblk.groups
            for a, (g, o) in enumerate(zip(v, oblk.groups[k])):
                assert g == o or abs(g - o) <= 1e-9 * max(abs(g), abs(o)), (k, a, g, o)
        from pinot_amd.engine.reduce import _agg_index
        ai = _agg_index(qc, qc.order_by[0].expression)
        desc = not qc.order_by[0].ascending
        kept = np.array([v[ai] for v in blk.groups.values()], dtype=np.float64)
        dropped = np.array([v[ai] for k, v in oblk.groups.items() if k not in blk.groups], dtype=np.float64)
        if desc:
            assert kept.min() >= dropped.max()
        else:
            assert kept.max() <= dropped.min()
        if exact_set:
            allv = sorted(oblk.groups.items(), key=lambda kv: kv[1][ai], reverse=desc)
            assert set(blk.groups) == {k for k, _ in allv[:trim]}
        # the broker's final rows are those of the untrimmed oracle
        got = reduce_blocks(qc, [blk]).rows
        want = reduce_blocks(qc, [oblk]).rows
        if exact_set:
            assert got == want
        else:
            assert [r[1:] for r in got] == [r[1:] for r in want]
    finally:
        for s in segs:
            s.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("sql", [
    "SELECT k, COUNT(*), SUM(m) FROM t GROUP BY k ORDER BY COUNT(*) DESC, k LIMIT 10",
    "SELECT k, k2, AVG(m) FROM t WHERE q < 45 GROUP BY k, k2 ORDER BY AVG(m) DESC, k2 LIMIT 100",  # hash table
    "SELECT q, k, SUM(m), MIN(m) FROM t GROUP BY q, k ORDER BY q DESC, SUM(m) LIMIT 1200",
    "SELECT k, MINMAXRANGE(m), MAX(m) FROM t GROUP BY k ORDER BY MINMAXRANGE(m), MAX(m) DESC, k LIMIT 10",
    # the registers' cardinality estimate (clearspring HyperLogLog.cardinality) on the device
    "SELECT k, DISTINCTCOUNTHLL(k2), COUNT(*) FROM t GROUP BY k ORDER BY DISTINCTCOUNTHLL(k2) DESC, k LIMIT 10",
    "SELECT k, DISTINCTCOUNTHLL(m, 5), SUM(m) FROM t WHERE q < 30 GROUP BY k ORDER BY DISTINCTCOUNTHLL(m, 5), k DESC "
    "LIMIT 1100",
])
def test_gpu_device_trim_mixed_order(gpu_lib, sql):
    """Mixed ORDER BY (GroupByUtils.java:108,161 -> TableResizer over group values and final results): the kept
    groups are exactly the first trimSize of the untrimmed oracle's groups by the whole ORDER BY (a total order
    here), each with the oracle's values, and the broker's rows match."""
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.reduce import final_result, _agg_index
    from pinot_amd.engine.segment import GpuSegment
    raws = _segments()
    segs = [GpuSegment(r) for r in raws]
    try:
        qc = parse(sql)
        op = GpuInstancePlanMaker(num_groups_limit=10 ** 9).make_instance_plan(qc, segs)
        assert op._trim_spec()[4], "expected the general ORDER BY terms"
        blk = op.next_block()
        oblk, _ = executor.execute(qc, raws, num_groups_limit=10 ** 9)
        trim = max(5 * qc.limit, 5000)
        assert len(oblk.groups) > trim
        assert blk.num_groups_trimmed and len(blk.groups) == trim
        gb = [str(e) for e in qc.group_by]

        def val(k, v, e):
            if str(e) in gb:
                return k[gb.index(str(e))]
            i = _agg_index(qc, e)
            return final_result(qc.aggregations[i].function, v[i])

        recs = sorted(oblk.groups.items())
        for ob in reversed(qc.order_by):
            recs.sort(key=lambda kv: val(kv[0], kv[1], ob.expression), reverse=not ob.ascending)
        assert set(blk.groups) == {k for k, _ in recs[:trim]}
        for k, v in blk.groups.items():
            for g, o in zip(v, oblk.groups[k]):
                if isinstance(o, np.ndarray):
                    assert np.array_equal(g, o)
                elif isinstance(o, tuple):
                    assert all(x == y or abs(x - y) <= 1e-9 * max(abs(x), abs(y)) for x, y in zip(g, o))
                else:
                    assert g == o or abs(g - o) <= 1e-9 * max(abs(g), abs(o))
        assert reduce_blocks(qc, [blk]).rows == reduce_blocks(qc, [oblk]).rows
    finally:
        for s in segs:
            s.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("sql", [
    "SELECT k, SUM(m) FROM t GROUP BY k ORDER BY k DESC LIMIT 10",
    "SELECT q, k, COUNT(*), MAX(m) FROM t WHERE q >= 3 GROUP BY q, k ORDER BY k, q DESC LIMIT 2000",
    "SELECT k, k2 FROM t GROUP BY k, k2 ORDER BY k2 DESC, k LIMIT 50",  # > 2^26 keys: hash table, no aggregation
])
def test_gpu_device_trim_by_group_keys(gpu_lib, sql):
    """ORDER BY group-by columns (BenchmarkQueries STARTREE_SUM_QUERY's shape): the kept groups are exactly
    the first trimSize by the key order, since group keys are distinct."""
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    raws = _segments()
    segs = [GpuSegment(r) for r in raws]
    try:
        qc = parse(sql)
        blk = GpuInstancePlanMaker(num_groups_limit=10 ** 9).make_instance_plan(qc, segs).next_block()
        oblk, _ = executor.execute(qc, raws, num_groups_limit=10 ** 9)
        trim = max(5 * qc.limit, 5000)
        assert len(oblk.groups) > trim
        assert blk.num_groups_trimmed and len(blk.groups) == trim
        gb = [str(e) for e in qc.group_by]
        keys = list(oblk.groups)
        for ob in reversed(qc.order_by):
            j = gb.index(str(ob.expression))
            keys.sort(key=lambda t: t[j], reverse=not ob.ascending)
        assert set(blk.groups) == set(keys[:trim])
        for k, v in blk.groups.items():
            for g, o in zip(v, oblk.groups[k]):
                assert g == o or abs(g - o) <= 1e-9 * max(abs(g), abs(o))
        assert reduce_blocks(qc, [blk]).rows == reduce_blocks(qc, [oblk]).rows
    finally:
        for s in segs:
            s.destroy()
