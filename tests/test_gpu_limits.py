"""Result-parity edges of group-by and integer sums.

numGroupsLimit: the reference keeps, per segment, the first numGroupsLimit distinct keys in doc order
(IntGroupIdMap.getGroupId returns INVALID_ID past groupIdUpperBound, DictionaryBasedGroupKeyGenerator.java:
153-174,1023-1048) and flags numGroupsLimitReached when a segment's group count reaches the limit
(GroupByOperator.java:116, OR-ed by GroupByCombineOperator.java:123-124). Known answer:
InterSegmentAggregationSingleValueQueriesTest.testNumGroupsLimit (:763-775).

int64 overflow: SumAggregationFunction accumulates in double (:76-101) and never wraps; the library keeps
an exact int64 sum while sum |value| over all docs stays below 2^62 and otherwise sums in double.
"""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.reduce import reduce_blocks, trim_groups
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures


# ---------------------------------------------------------------------------------------------- CPU: oracle
def test_oracle_first_seen_group_limit():
    """Per segment the first `limit` keys in doc order survive; later keys' docs are dropped."""
    c = SegmentCreator("fs")
    c.add_column("k", DataType.INT, [5, 3, 5, 7, 3, 9, 7, 5])
    c.add_column("m", DataType.LONG, [1, 10, 100, 1000, 10000, 100000, 1000000, 10000000])
    raw = c.build()
    qc = parse("SELECT k, COUNT(*), SUM(m) FROM t GROUP BY k")
    blk, ex = executor.execute(qc, [raw], num_groups_limit=2)
    assert blk.num_groups_limit_reached
    assert set(blk.groups) == {(5,), (3,)}
    assert blk.groups[(5,)][0] == 3 and ex[(5,)][1] == 10000101
    assert blk.groups[(3,)][0] == 2 and ex[(3,)][1] == 10010
    blk, _ = executor.execute(qc, [raw], num_groups_limit=4)
    assert blk.num_groups_limit_reached and len(blk.groups) == 4  # numGroups >= limit
    blk, _ = executor.execute(qc, [raw], num_groups_limit=5)
    assert not blk.num_groups_limit_reached and len(blk.groups) == 4


def test_oracle_num_groups_limit_known_answer():
    """InterSegmentAggregationSingleValueQueriesTest.testNumGroupsLimit (:763-775)."""
    seg = fixtures.segment_for("test_data_sv")
    qc = parse("SELECT COUNT(*) FROM testTable GROUP BY column1")
    blk, _ = executor.execute(qc, [seg, seg])
    assert not blk.num_groups_limit_reached
    blk, _ = executor.execute(qc, [seg, seg], num_groups_limit=1000)
    assert blk.num_groups_limit_reached and len(blk.groups) == 1000
    assert reduce_blocks(qc, [blk, blk]).num_groups_limit_reached


def test_oracle_exact_sums_beyond_int64():
    c = SegmentCreator("big")
    c.add_column("a", DataType.LONG, [2 ** 62 + 5, 2 ** 62 + 7, 2 ** 62 - 1])
    c.add_column("b", DataType.LONG, [2 ** 40, -3, 2 ** 41])
    raw = c.build()
    qc = parse("SELECT SUM(a), SUM(a * b) FROM t")
    blk, ex = executor.execute(qc, [raw])
    assert ex[0] == 3 * 2 ** 62 + 11
    assert ex[1] == (2 ** 62 + 5) * 2 ** 40 - 3 * (2 ** 62 + 7) + (2 ** 62 - 1) * 2 ** 41
    assert abs(blk.results[1] - ex[1]) <= 1e-12 * abs(ex[1])


# ---------------------------------------------------------------------------------------------- GPU
def _gpu(*a, **k):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    return GpuInstancePlanMaker(*a, **k)


def _segs(raws):
    from pinot_amd.engine.segment import GpuSegment
    return [GpuSegment(r) for r in raws]


def _check(qc, gblk, oblk, exact):
    from tests.test_gpu_parity import _assert_intermediates_equal
    assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert gblk.num_groups_limit_reached == oblk.num_groups_limit_reached
    assert set(gblk.groups) == set(oblk.groups)
    for k, v in oblk.groups.items():
        _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])


@pytest.mark.gpu
@pytest.mark.parametrize("limit", [None, 1000, 6582, 6583])
def test_gpu_num_groups_limit_known_answer(gpu_lib, limit):
    """testNumGroupsLimit: default limit -> not reached; 1000 -> reached, and the kept groups are each
    segment's first 1000 column1 values in doc order (column1 has 6582 distinct values, so 6582 reaches
    the limit and 6583 does not)."""
    seg = _segs([fixtures.segment_for("test_data_sv")])[0]
    try:
        kw = {} if limit is None else {"num_groups_limit": limit}
        qc = parse("SELECT column1, COUNT(*), SUM(column3), MAX(column9) FROM testTable GROUP BY column1 LIMIT 100000")
        gblk = _gpu(**kw).make_instance_plan(qc, [seg, seg]).next_block()
        oblk, exact = executor.execute(qc, [seg.segment, seg.segment], **kw)
        assert oblk.num_groups_limit_reached == (limit is not None and limit <= 6582)
        _check(qc, gblk, oblk, exact)
        assert reduce_blocks(qc, [gblk, gblk]).num_groups_limit_reached == oblk.num_groups_limit_reached
    finally:
        seg.destroy()


@pytest.fixture(scope="module")
def many_groups(gpu_lib):
    """3 segments x ~180K docs, ~145K distinct keys each (> the default limit of 100,000), keys in random
    doc order so the first-seen sets differ per segment; the dictionaries differ per segment too."""
    rng = np.random.default_rng(101)
    raws = []
    for s in range(3):
        n = 180_000 + 1111 * s
        c = SegmentCreator(f"mg{s}")
        c.add_column("a", DataType.INT, rng.integers(0, 400_000, n))
        c.add_column("s", DataType.STRING, np.array([f"s{x}" for x in rng.integers(0, 7, n)]))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.random(n) * 100, 2))
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        raws.append(c.build())
    segs = _segs(raws)
    yield raws, segs
    for g in segs:
        g.destroy()


LIMIT_QUERIES = [
    "SELECT a, COUNT(*), SUM(m), MIN(d), MAX(m), DISTINCTCOUNTHLL(m) FROM t GROUP BY a LIMIT 1000000",
    "SELECT a, COUNT(*), SUM(m) FROM t WHERE f < 90 GROUP BY a LIMIT 1000000",
    "SELECT a, s, COUNT(*), SUM(d) FROM t WHERE f >= 5 GROUP BY a, s LIMIT 1000000",
    "SELECT a, SUM(m) FROM t GROUP BY a ORDER BY SUM(m) DESC LIMIT 10",           # + device trim (5000)
    "SELECT s, a, MAX(d) FROM t WHERE f < 97 GROUP BY s, a ORDER BY a, s LIMIT 20",  # + key-order trim
]


@pytest.mark.gpu
@pytest.mark.parametrize("nseg", [3, 1])
@pytest.mark.parametrize("mode", ["auto", "hash"])
@pytest.mark.parametrize("sql", LIMIT_QUERIES)
def test_gpu_default_limit_over_100k_groups(sql, mode, nseg, many_groups, monkeypatch):
    """nseg 1 + hash: the normal pass records first-seen docs and the limit pass starts from its table."""
    monkeypatch.setenv("PHIP_GB_HASH", "1" if mode == "hash" else "0")
    raws, segs = many_groups
    raws, segs = raws[:nseg], segs[:nseg]
    qc = parse(sql)
    gblk = _gpu().make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws)
    assert oblk.num_groups_limit_reached and gblk.num_groups_limit_reached
    if getattr(gblk, "num_groups_trimmed", False):
        oblk = trim_groups(qc, oblk)
    _check(qc, gblk, oblk, exact)
    got, want = reduce_blocks(qc, [gblk]).rows, reduce_blocks(qc, [oblk]).rows
    if not qc.order_by:  # no ORDER BY: the broker's LIMIT rows come in table order; compare as sets
        got, want = sorted(got), sorted(want)
    assert fixtures.rows_match(got, want)


@pytest.mark.gpu
def test_gpu_sum_beyond_int64(gpu_lib):
    """A LONG SUM past 2^63, a LONG x LONG product past 2^63 per doc, and both per group: the library
    switches those SUMs to double accumulation (exact-int64 flag off); everything else stays exact."""
    rng = np.random.default_rng(9)
    n = 50_001
    c = SegmentCreator("big", no_dictionary_columns=["r"])
    c.add_column("a", DataType.LONG, rng.integers(2 ** 60, 2 ** 62, n))          # sum ~ 1e23
    c.add_column("b", DataType.LONG, rng.integers(-2 ** 40, 2 ** 40, n))         # a*b ~ 2^101
    c.add_column("r", DataType.LONG, rng.integers(2 ** 61, 2 ** 62, n))          # raw: device min/max bound
    c.add_column("k", DataType.INT, rng.integers(0, 13, n))
    c.add_column("q", DataType.INT, rng.integers(-1000, 1000, n))                # stays exact
    raw = c.build()
    seg = _segs([raw])[0]
    try:
        from tests.test_gpu_parity import _assert_intermediates_equal
        for sql in ("SELECT SUM(a), SUM(a * b), SUM(r), SUM(q), SUM(b), COUNT(*) FROM t",
                    "SELECT SUM(a), SUM(r - a), SUM(q * k) FROM t WHERE k < 7"):
            qc = parse(sql)
            blk = _gpu().make_instance_plan(qc, [seg]).next_block()
            oblk, ex = executor.execute(qc, [raw])
            assert isinstance(blk.results[0], float) and abs(ex[0]) >= 2 ** 63
            _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
        qc = parse("SELECT SUM(q), SUM(b) FROM t")
        blk = _gpu().make_instance_plan(qc, [seg]).next_block()
        assert all(isinstance(x, int) for x in blk.results)  # bound below 2^62: exact int64
        qc = parse("SELECT k, SUM(a * b), SUM(a), SUM(q), COUNT(*) FROM t GROUP BY k")
        gblk = _gpu().make_instance_plan(qc, [seg]).next_block()
        oblk, exact = executor.execute(qc, [raw])
        _check(qc, gblk, oblk, exact)
        assert all(isinstance(v[0], float) and isinstance(v[1], float) and isinstance(v[2], int)
                   for v in gblk.groups.values())
    finally:
        seg.destroy()
