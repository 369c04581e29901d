"""Null value vectors on the GPU (PHIP_LEAF_NULL over the resident null doc words) and enableNullHandling: three-valued
filters (the plan's trees, plan._three_valued), null-skipping aggregations with null results
(GpuNullHandlingAggregationOperator), COUNT(col), IS [NOT] NULL with and without null handling, and the shapes that
stay on the CPU (null group keys, per-group nulls) -- every block against the oracle (eval_filter3, the oracle's
null-skipping _agg_segment), including numDocsScanned and the post-filter entries."""
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
    "SELECT g, SUM(d) FROM t GROUP BY g LIMIT 10",              # per-group null results
    "SELECT s, COUNT(*) FROM t GROUP BY s LIMIT 10",            # a null group key
    "SELECT g, SUM(k) FILTER (WHERE d > 3) FROM t GROUP BY g LIMIT 10",
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
