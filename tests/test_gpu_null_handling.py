"""Null value vectors on the GPU (PHIP_LEAF_NULL over the resident null doc words) and enableNullHandling: three-valued
filters (the plan's trees, plan._three_valued), null-skipping aggregations with null results
(GpuNullHandlingAggregationOperator), COUNT(col), IS [NOT] NULL with and without null handling, and the shapes that
stay on the CPU; GROUP BY with null keys and per-group null results (GpuNullHandlingGroupByOperator,
phip_query_desc.null_group_by) -- every block against the oracle (eval_filter3, the oracle's null-skipping
_agg_segment and null-aware _group_segment), including numDocsScanned and the post-filter entries."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker, UnsupportedOnGpu
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def null_segments(gpu_lib):
    """Three ragged segments. d / l / f / s / r carry nulls at different rates (segment 1's d has none: no null
    vector there), z is null everywhere, g / k / t never are; s has an inverted index, t is sorted, r is raw."""
    from pinot_amd.engine.segment import GpuSegment
    rng = np.random.default_rng(91)
    raws = []
    for k, n in enumerate((30_001, 70_000, 4_097)):
        c = SegmentCreator(f"nz{k}", inverted_index_columns=["s"], no_dictionary_columns=["r"])
        c.add_column("d", DataType.INT, rng.integers(0, 200, n), nulls=(rng.random(n) < 0.1) if k != 1 else None)
        c.add_column("l", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n), nulls=rng.random(n) < 0.3)
        c.add_column("f", DataType.DOUBLE, np.round(rng.normal(0, 100, n), 2), nulls=rng.random(n) < 0.05)
        c.add_column("s", DataType.STRING, np.array([f"v{x}" for x in rng.integers(0, 6, n)]),
                     nulls=rng.random(n) < 0.2)
        c.add_column("r", DataType.LONG, rng.integers(0, 1_000_000, n), nulls=rng.random(n) < 0.15)
        c.add_column("z", DataType.INT, rng.integers(0, 9, n), nulls=np.ones(n, dtype=bool))
        c.add_column("g", DataType.INT, rng.integers(0, 8, n))
        c.add_column("k", DataType.INT, rng.integers(-50, 50, n))
        c.add_column("t", DataType.INT, np.sort(rng.integers(0, 30, n)))
        raws.append(c.build())
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


NH = "SET enableNullHandling = true; "
AGG = [
    "SELECT SUM(d), MIN(d), MAX(d), COUNT(d), COUNT(*), AVG(d) FROM t",
    "SELECT SUM(l), MIN(f), MAX(r), COUNT(r) FROM t WHERE g < 5",
    "SELECT SUM(d * k), SUM(l - r), MINMAXRANGE(f) FROM t WHERE s = 'v3' OR d > 100",
    "SELECT COUNT(*), SUM(k) FROM t WHERE NOT (d > 50 AND s IN ('v1', 'v2'))",
    "SELECT SUM(d), COUNT(*) FROM t WHERE d IS NULL",
    "SELECT SUM(d), COUNT(d) FROM t WHERE d IS NOT NULL AND NOT (l < 0)",
    "SELECT SUM(k) FILTER (WHERE d > 10), MAX(l) FILTER (WHERE s IS NULL), COUNT(*) FROM t WHERE g <> 3",
    "SELECT SUM(z), COUNT(z), MIN(z), COUNT(*) FROM t",
    "SELECT SUM(d), MIN(l), COUNT(*) FROM t WHERE k = -999",
    "SELECT DISTINCTCOUNTHLL(d), COUNT(*) FROM t WHERE NOT (s = 'v1')",
    "SELECT COUNT(*), SUM(k) FROM t WHERE NOT (r BETWEEN 10 AND 500000)",
    "SELECT COUNT(*), MAX(f) FROM t WHERE NOT (t BETWEEN 3 AND 20) AND NOT (d <> 12345)",
    "SELECT SUM(k), COUNT(*) FROM t WHERE NOT (NOT (d = 7 OR l > 0) AND s <> 'v4')",
    # raw column leaves that fold to a constant keep the null bitmap (BaseRawValueBasedPredicateEvaluator: never
    # always-true / always-false): an empty range and a NOT IN left without integral values
    "SELECT COUNT(*), SUM(k) FROM t WHERE NOT (r BETWEEN 500 AND 100)",
    "SELECT COUNT(*), SUM(k) FROM t WHERE NOT (r NOT IN (1.5, 2.5))",
    "SELECT COUNT(*), MAX(l) FROM t WHERE NOT (r IN (2.5) AND g < 4) OR k = 3",
]


def _run(sql, mat):
    raws, segs = mat
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
    blk = op.next_block()
    op.close()
    oblk, ex = executor.execute(qc, raws)
    return qc, blk, oblk, ex


@pytest.mark.parametrize("sql", AGG)
def test_gpu_null_handling_aggregations(sql, null_segments):
    from tests.test_gpu_parity import _assert_intermediates_equal
    qc, blk, oblk, ex = _run(NH + sql, null_segments)
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert blk.stats.num_entries_scanned_post_filter == oblk.stats.num_entries_scanned_post_filter
    for ag, g, o, e in zip(qc.aggregations, blk.results, oblk.results, ex):
        assert (g is None) == (o is None), (ag, g, o)
        if o is not None:
            _assert_intermediates_equal([ag], [g], [o], [e])
    got, want = reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [oblk]).rows
    assert fixtures.rows_match(got, want) if all(v is not None for v in want[0]) else \
        [v is None for v in got[0]] == [v is None for v in want[0]]


@pytest.mark.parametrize("sql", [
    "SELECT COUNT(*), SUM(k) FROM t WHERE d IS NULL OR s IS NOT NULL",
    "SELECT COUNT(*), MIN(k) FROM t WHERE NOT (z IS NULL) OR (g = 2 AND l IS NULL)",
    "SELECT SUM(d), COUNT(*) FROM t WHERE NOT (d = 5)",  # two-valued: null docs hold Integer.MIN_VALUE
])
def test_gpu_is_null_without_null_handling(sql, null_segments):
    from tests.test_gpu_parity import _assert_intermediates_equal
    qc, blk, oblk, ex = _run(sql, null_segments)
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)


@pytest.mark.parametrize("sql", [
    "SELECT g, SUM(k), COUNT(*) FROM t WHERE NOT (d > 50) GROUP BY g LIMIT 100",
    "SELECT g, t, MAX(k), COUNT(*) FROM t WHERE s IS NULL OR NOT (l > 0) GROUP BY g, t LIMIT 1000",
])
def test_gpu_null_handling_group_by_over_null_free_columns(sql, null_segments):
    from tests.test_gpu_limits import _check
    qc, blk, oblk, ex = _run(NH + sql, null_segments)
    _check(qc, blk, oblk, ex)


@pytest.mark.parametrize("sql", [
    # nine primitive slots once the non-null counts are added (device kMaxAggs = 8): the CPU plan maker's
    "SELECT g, SUM(d), MIN(l), MAX(f), COUNT(*), AVG(r) FROM t GROUP BY g LIMIT 10",
    "SELECT d, k FROM t WHERE g = 1 LIMIT 10",                  # selected null values
])
def test_gpu_null_handling_refusals(sql, null_segments):
    raws, segs = null_segments
    with pytest.raises(UnsupportedOnGpu):
        GpuInstancePlanMaker().make_instance_plan(parse(NH + sql), segs)


def test_gpu_null_handling_selection_of_null_free_columns(null_segments):
    raws, segs = null_segments
    qc = parse(NH + "SELECT g, k FROM t WHERE NOT (d = 5 OR s = 'v2') LIMIT 200")
    blk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
    oblk, _ = executor.execute(qc, raws)
    assert blk.rows == oblk.rows


@pytest.mark.parametrize("dt,base", [(DataType.INT, 7), (DataType.DOUBLE, -1.25)])
def test_gpu_null_enabled_known_answers(dt, base, gpu_lib):
    """NullEnabledQueriesTest (pinot-core/src/test/.../queries/NullEnabledQueriesTest.java:93-122,473-495): four
    copies of 1000 records, the odd ones null: COUNT(col) 2000, MIN base, MAX base + 998, AVG / SUM of the evens."""
    from pinot_amd.engine.segment import GpuSegment
    vals = np.array([base + i for i in range(1000)])
    c = SegmentCreator("ne")
    c.add_column("col", dt, vals, nulls=np.arange(1000) % 2 == 1)
    raw = c.build()
    segs = [GpuSegment(raw) for _ in range(4)]
    try:
        q = parse(NH + "SELECT COUNT(col) AS count, MIN(col) AS min, MAX(col) AS max, AVG(col) AS avg, "
                       "SUM(col) AS sum FROM testTable LIMIT 1000")
        rt = reduce_blocks(q, [GpuInstancePlanMaker().make_instance_plan(q, segs).next_block()])
        row = rt.rows[0]
        s = float(sum(base + i for i in range(0, 1000, 2)))
        assert rt.columns == ["count", "min", "max", "avg", "sum"]
        assert row[0] == 2000 and abs(row[1] - base) < 1e-1 and abs(row[2] - (base + 998)) < 1e-1
        assert abs(row[3] - s / 500) < 1e-1 and abs(row[4] - 4 * s) < 1e-1
    finally:
        for g in segs:
            g.destroy()


# ---- GROUP BY under enableNullHandling: null keys, per-group null results -----------------------------------------
GB = [
    "SELECT s, COUNT(*) FROM t GROUP BY s LIMIT 100",                                    # a null STRING key
    "SELECT d, g, COUNT(*), SUM(k) FROM t WHERE g < 6 GROUP BY d, g LIMIT 100000",      # INT key, nulls in 2 segments
    "SELECT r, COUNT(*) FROM t WHERE k > 40 GROUP BY r LIMIT 100000",                   # a raw LONG key with nulls
    "SELECT g, SUM(d), MIN(l), COUNT(d), COUNT(*), AVG(r) FROM t GROUP BY g LIMIT 100",  # null results
    "SELECT s, g, SUM(d * k), MINMAXRANGE(f), COUNT(l) FROM t WHERE NOT (d > 150) GROUP BY s, g LIMIT 1000",
    "SELECT z, SUM(z), COUNT(z), COUNT(*) FROM t GROUP BY z LIMIT 10",                  # all-null key and values
    "SELECT t, s, DISTINCTCOUNTHLL(d), SUM(l) FROM t WHERE s IS NOT NULL OR d IS NULL GROUP BY t, s LIMIT 10000",
    "SELECT k, s, SUM(f), COUNT(*) FROM t WHERE k = -999 GROUP BY k, s LIMIT 10",       # nothing matches
]


def _check_nullable_groups(qc, blk, oblk, ex):
    from tests.test_gpu_parity import _assert_intermediates_equal
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert blk.stats.num_entries_scanned_post_filter == oblk.stats.num_entries_scanned_post_filter
    assert blk.num_groups_limit_reached == oblk.num_groups_limit_reached
    assert set(blk.groups) == set(oblk.groups)
    for key, ov in oblk.groups.items():
        gv = blk.groups[key]
        for ag, g, o, e in zip(qc.aggregations, gv, ov, ex[key]):
            assert (g is None) == (o is None), (key, ag, g, o)
            if o is not None:
                _assert_intermediates_equal([ag], [g], [o], [e])


@pytest.mark.parametrize("sql", GB)
def test_gpu_null_handling_group_by(sql, null_segments):
    """Null keys (the library's null key id) and per-group null results (IS NOT NULL programs beside the query's
    own) against the oracle's null-aware GroupByOperator: keys, every intermediate, numDocsScanned, post-filter
    entries."""
    qc, blk, oblk, ex = _run(NH + sql, null_segments)
    _check_nullable_groups(qc, blk, oblk, ex)


@pytest.mark.parametrize("mode", ["hash", "fused_xcd", "fused_hbm", "tuple"])
@pytest.mark.parametrize("sql", [GB[1], GB[3], GB[4]])
def test_gpu_null_handling_group_by_table_modes(sql, mode, null_segments, monkeypatch):
    """The same null keys / null results through the hash table, fused into the filter (XCD copies, one HBM
    table) where the program is conjunctive, and as tuple keys (a null key's id inside the packed tuple)."""
    monkeypatch.setenv(*{"hash": ("PHIP_GB_HASH", "1"), "fused_xcd": ("PHIP_FUSED_GB", "3"),
                         "fused_hbm": ("PHIP_FUSED_GB", "2"), "tuple": ("PHIP_TUPLE_KEYS", "1")}[mode])
    qc, blk, oblk, ex = _run(NH + sql, null_segments)
    _check_nullable_groups(qc, blk, oblk, ex)


NH_FILTER_GB = [
    "SELECT g, SUM(k) FILTER (WHERE d > 3), COUNT(*) FROM t GROUP BY g LIMIT 100",
    "SELECT d, g, SUM(l) FILTER (WHERE k > 40), MIN(f) FILTER (WHERE s IS NULL), COUNT(d) FILTER (WHERE g < 3), "
    "AVG(r) FROM t WHERE g < 6 GROUP BY d, g LIMIT 100000",
    # every function filtered: the main info still generates the groups (functions none of whose docs reached a group
    # are null, COUNT 0)
    "SELECT s, MAX(f) FILTER (WHERE d IS NOT NULL), COUNT(*) FILTER (WHERE d > 190) FROM t GROUP BY s LIMIT 100",
    "SELECT z, SUM(z) FILTER (WHERE g = 1), COUNT(*) FROM t GROUP BY z LIMIT 10",
    "SET filteredAggregationsSkipEmptyGroups = true; SELECT g, t, SUM(k) FILTER (WHERE d > 150), "
    "MINMAXRANGE(l) FILTER (WHERE d > 150) FROM t GROUP BY g, t LIMIT 100000",
]


@pytest.mark.parametrize("sql", NH_FILTER_GB)
def test_gpu_null_handling_filtered_group_by(sql, null_segments):
    """FILTER + GROUP BY under enableNullHandling (FilteredGroupByOperator's infos over the null-aware generator):
    programs = the infos, then their IS NOT NULL sets; a nullable function is null where its own program's docs
    never reached the group (ObjectGroupByResultHolder). Keys, every intermediate and the summed statistics equal the
    oracle's."""
    qc, blk, oblk, ex = _run(NH + sql, null_segments)
    _check_nullable_groups(qc, blk, oblk, ex)


@pytest.mark.parametrize("limit", [40, 150])
def test_gpu_null_handling_group_by_num_groups_limit(limit, null_segments):
    """numGroupsLimit counts the null key in first-seen order (getKeyForNullValue) over the query's matched docs --
    program 0 -- per segment; the kept groups and their null results equal the oracle's."""
    raws, segs = null_segments
    for sql in ("SELECT d, COUNT(*), SUM(l) FROM t GROUP BY d LIMIT 100000",
                "SELECT d, g, COUNT(d), MAX(f) FROM t WHERE k > 0 GROUP BY d, g LIMIT 100000"):
        qc = parse(NH + sql)
        op = GpuInstancePlanMaker(num_groups_limit=limit).make_instance_plan(qc, segs)
        blk = op.next_block()
        op.close()
        oblk, ex = executor.execute(qc, raws, num_groups_limit=limit)
        assert oblk.num_groups_limit_reached
        _check_nullable_groups(qc, blk, oblk, ex)


@pytest.mark.parametrize("order", ["d ASC", "d DESC", "d ASC NULLS FIRST", "d DESC NULLS LAST", "SUM(l) DESC",
                                   "SUM(l) ASC NULLS FIRST"])
def test_gpu_null_handling_group_by_order_by(order, null_segments):
    """Broker rows ordered with the reference's null placement (OrderByExpressionContext.isNullsLast: nulls as the
    largest value unless NULLS FIRST / LAST says otherwise), for keys and null results alike; trimmed on the device
    or the host, the rows equal the oracle's."""
    raws, segs = null_segments
    qc = parse(NH + f"SELECT d, SUM(l), COUNT(*) FROM t WHERE g < 3 GROUP BY d ORDER BY {order} LIMIT 30")
    blk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
    oblk, _ = executor.execute(qc, raws)
    got, want = reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [oblk]).rows
    assert [r[0] for r in got] == [r[0] for r in want]
    for a, b in zip(got, want):
        assert (a[1] is None) == (b[1] is None) and a[2] == b[2]
        if b[1] is not None:
            assert abs(a[1] - b[1]) <= 1e-9 * max(1.0, abs(b[1]))


NULL_GB_KATS = [
    ("SELECT column1, COUNT(*) FROM testTable GROUP BY column1",
     {"column1": [None, None, None, 1, 2, 2]}, {(2,): [8], (1,): [4], (None,): [12]}),
    ("SELECT column1, COUNT(column2) FROM testTable GROUP BY column1",
     {"column1": [1, None, None], "column2": [1, 1, 1]}, {(None,): [8], (1,): [4]}),
    ("SELECT count(*), column1, column2 FROM testTable GROUP BY column1, column2",
     {"column1": [None, None, None, 1, 1, 1], "column2": [None, 1, 1, 1, None, -2 ** 31]},
     {(None, None): [4], (None, 1): [8], (1, 1): [4], (1, None): [4], (1, -2 ** 31): [4]}),
    ("SELECT count(*), column1 FROM testTable GROUP BY column1",
     {"column1": [None, 1, 1, 2, 3]}, {(1,): [8], (2,): [4], (3,): [4], (None,): [4]}),
]


@pytest.mark.parametrize("sql,cols,expect", NULL_GB_KATS, ids=[k[0][:48] for k in NULL_GB_KATS])
def test_gpu_null_group_keys_known_answers(sql, cols, expect, gpu_lib):
    """NullHandlingEnabledQueriesTest's GROUP BY cases (testGroupByOrderByNullsLastUsingOrdinal :153-176,
    testHavingFilterIsNull :178-199, testMultiColumnGroupBy :778-806, testGroupByOrderBy :834-858): one segment
    queried as 2 servers x 2 segments, every count x 4; a stored Integer.MIN_VALUE is a value, a null doc the null
    key."""
    from pinot_amd.engine.results import merge_intermediate
    from pinot_amd.engine.segment import GpuSegment
    c = SegmentCreator("kat")
    for name, vals in cols.items():
        nulls = [v is None for v in vals]
        c.add_column(name, DataType.INT, [0 if v is None else v for v in vals], nulls=nulls if any(nulls) else None)
    seg = GpuSegment(c.build())
    try:
        qc = parse(NH + sql)
        blk = GpuInstancePlanMaker().make_instance_plan(qc, [seg, seg]).next_block()
        merged = {}
        for _ in range(2):
            for k, v in blk.groups.items():
                merged[k] = [merge_intermediate(a.function, x, y) for a, x, y in zip(qc.aggregations, merged[k], v)] \
                    if k in merged else list(v)
        assert merged == expect
        if sql.startswith("SELECT column1, COUNT(*)"):  # the test's own ORDER BY 1 DESC NULLS LAST: 2, 1, null
            q2 = parse(NH + sql + " ORDER BY column1 DESC NULLS LAST")
            b2 = GpuInstancePlanMaker().make_instance_plan(q2, [seg, seg]).next_block()
            assert reduce_blocks(q2, [b2, b2]).rows == [[2, 8], [1, 4], [None, 12]]
    finally:
        seg.destroy()
