"""GPU parity for filtered aggregations evaluated in ONE pass ("multiple filter programs per
pass"): every FILTER info of AggregationFunctionUtils.buildFilteredAggregationInfos (:312-400) is one filter
program of a single plan (phip_query_desc.num_filter_programs), one filter launch writes a tile mask per program
and one aggregation launch applies each function to its own program's docs.

Checked against the oracle's FilteredAggregationOperator (pinot-core/.../operator/query/
FilteredAggregationOperator.java:67-113): intermediates bit-exact (INT / LONG sums, counts, min / max, HLL
registers), numDocsScanned and numEntriesScannedPostFilter summed over the infos, numSegmentsMatched = segments
where any info matched. Segments are ragged (not multiples of the 2048-doc tile), one column is sorted (doc-range
pruning differs per program), and some programs match nothing, or only some segments."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuFilteredAggregationOperator, GpuInstancePlanMaker
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests.test_gpu_parity import _assert_intermediates_equal

pytestmark = pytest.mark.gpu

SIZES = (20_000, 23_071, 9_999)


def _segments(seed=11):
    rng = np.random.default_rng(seed)
    out = []
    start = 0
    for k, n in enumerate(SIZES):
        c = SegmentCreator(f"fp{k}", inverted_index_columns=["INT_COL"])
        c.add_column("SEG", DataType.INT, np.full(n, k))
        c.add_column("SORTED", DataType.INT, np.arange(start, start + n))
        c.add_column("INT_COL", DataType.INT, rng.integers(0, 1_000_000, n))
        c.add_column("LONG_COL", DataType.LONG, rng.integers(-(1 << 40), 1 << 40, n))
        c.add_column("DBL", DataType.DOUBLE, np.round(rng.normal(0, 1e3, n), 3))
        c.add_column("LOW", DataType.STRING, [f"v{x}" for x in rng.integers(0, 8, n)])
        out.append(c.build())
        start += n
    return out


ONE_PASS = [
    # programs matching only some segments: numSegmentsMatched counts a segment any program matched
    "SELECT COUNT(*) FILTER(WHERE SEG = 1), SUM(INT_COL) FILTER(WHERE SEG = 2), "
    "MIN(DBL) FILTER(WHERE SEG = 2 AND LOW = 'v3') FROM T",
    # sorted-column programs (per-program doc-range pruning) beside a main filter over an inverted index
    "SELECT SUM(LONG_COL) FILTER(WHERE SORTED < 5000), COUNT(*) FILTER(WHERE SORTED BETWEEN 30000 AND 40000), "
    "MAX(DBL) FROM T WHERE INT_COL > 1000",
    # COUNT-only programs (no value column at all)
    "SELECT COUNT(*) FILTER(WHERE INT_COL < 100000), COUNT(*) FILTER(WHERE LOW IN ('v1', 'v5')), COUNT(*) FROM T",
    # programs no doc passes: holder defaults (SUM 0, MIN +inf, MAX -inf, COUNT 0)
    "SELECT SUM(INT_COL) FILTER(WHERE INT_COL < 0), MIN(DBL) FILTER(WHERE INT_COL < 0), "
    "MAX(LONG_COL) FILTER(WHERE SORTED > 99999999), COUNT(*) FROM T",
    # a main filter nothing passes (every program pruned)
    "SELECT SUM(INT_COL) FILTER(WHERE LOW = 'v1'), COUNT(*) FILTER(WHERE LOW = 'v2'), MIN(DBL) FROM T "
    "WHERE SORTED < 0",
    # the same function under different filters must not share a slot
    "SELECT SUM(INT_COL) FILTER(WHERE LOW = 'v0'), SUM(INT_COL) FILTER(WHERE LOW <> 'v0'), SUM(INT_COL) FROM T",
    # OR / NOT programs (general interpreter), HLL, AVG and MINMAXRANGE under filters
    "SELECT DISTINCTCOUNTHLL(LOW) FILTER(WHERE INT_COL BETWEEN 1000 AND 500000), "
    "AVG(DBL) FILTER(WHERE LOW IN ('v1', 'v2') OR INT_COL < 100), "
    "MINMAXRANGE(LONG_COL) FILTER(WHERE NOT (LOW = 'v0')), COUNT(*) FROM T WHERE SORTED >= 1000",
    # an expression under a filter
    "SELECT SUM(INT_COL * SEG) FILTER(WHERE LOW < 'v4'), SUM(INT_COL - SORTED) FILTER(WHERE SEG <> 1), "
    "MAX(INT_COL + SORTED) FROM T",
]

# nine distinct filters: more than kMaxPrograms, so one plan per info (same results)
MANY = ("SELECT " + ", ".join(f"COUNT(*) FILTER(WHERE LOW = 'v{k}')" for k in range(8)) +
        ", SUM(INT_COL) FILTER(WHERE SEG = 0), COUNT(*) FROM T")


@pytest.fixture(scope="module")
def fp(gpu_lib):
    segs = [GpuSegment(s) for s in _segments()]
    yield segs
    for s in segs:
        s.destroy()


def _find(op, cls):
    seen = set()
    while op is not None and id(op) not in seen:
        seen.add(id(op))
        if isinstance(op, cls):
            return op
        op = getattr(op, "inner", None) or getattr(op, "op", None)
    return None


def _check(sql, segs, one_pass):
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
    fop = _find(op, GpuFilteredAggregationOperator)
    assert fop is not None
    assert (fop.one_pass is not None) == one_pass
    blk = op.next_block()
    op.close()
    oblk, exact = executor.execute(qc, [s.segment for s in segs])
    _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, exact)
    s, o = blk.stats, oblk.stats
    assert s.num_docs_scanned == o.num_docs_scanned
    assert s.num_entries_scanned_post_filter == o.num_entries_scanned_post_filter
    assert s.num_segments_matched == o.num_segments_matched
    assert s.num_total_docs == o.num_total_docs == sum(SIZES)
    return blk


@pytest.mark.parametrize("sql", ONE_PASS, ids=[q[:80] for q in ONE_PASS])
def test_gpu_filter_programs_one_pass_vs_oracle(sql, fp):
    _check(sql, fp, one_pass=True)


def test_gpu_filter_programs_many_infos_split(fp):
    _check(MANY, fp, one_pass=False)


def test_gpu_filter_programs_one_launch_each(fp):
    """One filter and one aggregation launch for all programs: the block's kernel times are one plan's, and the
    filter's algorithmic bytes cover every program's tiles."""
    blk = _check(ONE_PASS[0], fp, one_pass=True)
    assert blk.filter_kernel_ms > 0 and blk.agg_kernel_ms > 0
    assert blk.filter_bytes > 0
