"""GPU parity for FILTER + GROUP BY (FilteredGroupByOperator) and CASE-based aggregations.

Mirrors the reference's FilteredAggregationsTest (pinot-core/src/test/java/org/apache/pinot/queries/
FilteredAggregationsTest.java): each FILTER query and its WHERE / CASE twin must give the same rows -- here both
run on the GPU -- and every block is checked against the oracle (FilteredGroupByOperator semantics, CASE evaluated
per doc): group set, intermediates (bit-exact INT sums / counts / min / max), numDocsScanned and post-filter entries."""
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker
from pinot_amd.engine.reduce import broker_response, reduce_blocks
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.query.sql import parse
from tests import fixtures
from tests.test_filtered_aggregations import FT_PAIRS, _ft_segments
from tests.test_gpu_parity import _assert_intermediates_equal

pytestmark = pytest.mark.gpu

EXTRA = [
    # several filters + unfiltered functions + HLL under a filter, mixed widths
    "SELECT COUNT(*), SUM(INT_COL) FILTER(WHERE STRING_COL < 'M'), DISTINCTCOUNTHLL(STRING_COL) FILTER(WHERE INT_COL "
    "BETWEEN 100 AND 20000), MAX(NO_INDEX_COL) FILTER(WHERE BOOLEAN_COL = 1), MIN(INT_COL) FROM MyTable "
    "WHERE NO_INDEX_COL >= 50 GROUP BY BOOLEAN_COL, STATIC_INT_COL",
    # a filter no doc passes: every group keeps the holder defaults for it
    "SELECT SUM(INT_COL) FILTER(WHERE INT_COL < 0), MIN(INT_COL) FILTER(WHERE INT_COL < 0), COUNT(*) "
    "FROM MyTable GROUP BY BOOLEAN_COL",
    # multi-branch CASE with literal and expression branches, under a FILTER, with AVG / MINMAXRANGE
    "SELECT SUM(CASE WHEN INT_COL < 1000 THEN NO_INDEX_COL WHEN INT_COL < 2000 THEN 3 ELSE INT_COL - NO_INDEX_COL END) "
    "FILTER(WHERE BOOLEAN_COL = 0), AVG(CASE WHEN NO_INDEX_COL > 100 THEN INT_COL ELSE 7 END), "
    "MINMAXRANGE(CASE WHEN INT_COL BETWEEN 10 AND 20 THEN INT_COL ELSE 1000 END), "
    "COUNT(CASE WHEN INT_COL > 5 THEN 1 ELSE 0 END) FROM MyTable GROUP BY STATIC_INT_COL",
    "SELECT SUM(CASE WHEN STRING_COL > 'm' THEN INT_COL ELSE 0 END), MAX(CASE WHEN BOOLEAN_COL = 1 THEN 5 "
    "ELSE NO_INDEX_COL END) FROM MyTable WHERE INT_COL > 100",
    # ORDER BY a filtered aggregation with > trimSize groups: server trim after the merge
    "SELECT SUM(INT_COL) FILTER(WHERE BOOLEAN_COL = 1) AS s, COUNT(*) FROM MyTable GROUP BY STRING_COL "
    "ORDER BY s DESC, STRING_COL LIMIT 20",
]


@pytest.fixture(scope="module")
def ft(gpu_lib):
    segs = [GpuSegment(s) for s in _ft_segments()]
    yield segs
    for s in segs:
        s.destroy()


def _check_vs_oracle(sql, segs):
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
    blk = op.next_block()
    op.close()
    oblk, exact = executor.execute(qc, [s.segment for s in segs])
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert blk.stats.num_entries_scanned_post_filter == oblk.stats.num_entries_scanned_post_filter
    if not qc.group_by:
        _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, exact)
    else:
        if getattr(blk, "num_groups_trimmed", False):
            assert set(blk.groups) <= set(oblk.groups)
        else:
            assert set(blk.groups) == set(oblk.groups)
        for k, v in blk.groups.items():
            _assert_intermediates_equal(qc.aggregations, v, oblk.groups[k], exact[k])
    # broker rows of the (possibly trimmed) GPU block == the untrimmed oracle's (no ORDER BY: any row order)
    a, b = reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [oblk]).rows
    if not qc.order_by:
        a, b = sorted(a, key=repr), sorted(b, key=repr)
    assert fixtures.rows_match(a, b)


@pytest.mark.parametrize("pair", FT_PAIRS, ids=[p[0][:70] for p in FT_PAIRS])
def test_gpu_filter_query_equals_twin(pair, ft):
    fq, nq = pair
    pm = GpuInstancePlanMaker()
    a = broker_response(pm, fq, ft).rows
    b = broker_response(pm, nq, ft).rows
    if not parse(fq).order_by:
        a, b = sorted(a, key=repr), sorted(b, key=repr)
    assert fixtures.rows_match(a, b, rel=0.0), (a, b)


@pytest.mark.parametrize("sql", [q for p in FT_PAIRS for q in p] + EXTRA)
def test_gpu_filtered_group_by_vs_oracle(sql, ft):
    _check_vs_oracle(sql, ft)


# ---- one pass: the infos are filter programs of ONE group-by plan --------------------------------------------
LIMIT_QUERIES = [
    # one filtered info + the main info: the reference's info order (filtered first, main last) is defined
    "SELECT STRING_COL, SUM(INT_COL) FILTER(WHERE BOOLEAN_COL = 1), COUNT(*), MAX(NO_INDEX_COL) FROM MyTable "
    "GROUP BY STRING_COL",
    # two filtered infos, COUNTs under different filters, HLL, groups over two columns
    "SELECT STRING_COL, STATIC_INT_COL, COUNT(*) FILTER(WHERE INT_COL > 20000), COUNT(*) FILTER(WHERE NO_INDEX_COL "
    "< 500), DISTINCTCOUNTHLL(INT_COL) FILTER(WHERE INT_COL > 20000), MIN(INT_COL) FROM MyTable "
    "WHERE NO_INDEX_COL > 10 GROUP BY STRING_COL, STATIC_INT_COL",
]


@pytest.mark.parametrize("mode", ["dense", "hash"])
@pytest.mark.parametrize("limit", [100_000, 37, 1])
@pytest.mark.parametrize("sql", LIMIT_QUERIES, ids=["one-filter", "two-filters"])
def test_gpu_filtered_group_by_one_pass_limit(sql, limit, mode, ft, monkeypatch):
    """numGroupsLimit over the shared generator: per segment, groups first-seen over info 0's docs, then info 1's,
    ...; later keys are dropped for every info (FilteredGroupByOperator.java:110-176 with one
    DictionaryBasedGroupKeyGenerator). The GPU's limit pass orders (segment, key) entries by (info, doc)."""
    if mode == "hash":
        monkeypatch.setenv("PHIP_GB_HASH", "1")
    qc = parse(sql)
    op = GpuInstancePlanMaker(num_groups_limit=limit).make_instance_plan(qc, ft)
    assert op.one_pass is not None and op.one_pass.num_programs >= 2
    oblk, exact = executor.execute(qc, [s.segment for s in ft], num_groups_limit=limit)
    if op.num_filtered_infos >= 2 and oblk.num_groups_limit_reached:
        # two filtered infos: the reference's info order is HashMap order, so the kept keys are not defined by
        # the query -- the GPU refuses the execution (the Java plan maker answers on the CPU)
        from pinot_amd.engine.plan import UnsupportedOnGpu
        with pytest.raises(UnsupportedOnGpu):
            op.next_block()
        op.close()
        return
    blk = op.next_block()
    op.close()
    assert blk.num_groups_limit_reached == oblk.num_groups_limit_reached
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert blk.stats.num_entries_scanned_post_filter == oblk.stats.num_entries_scanned_post_filter
    assert set(blk.groups) == set(oblk.groups), (len(blk.groups), len(oblk.groups))
    for k, v in blk.groups.items():
        _assert_intermediates_equal(qc.aggregations, v, oblk.groups[k], exact[k])


def test_gpu_filtered_group_by_skip_empty_groups_one_pass(ft):
    """filteredAggregationsSkipEmptyGroups: no main info, so the groups are the union of the filtered infos'."""
    sql = ("SET filteredAggregationsSkipEmptyGroups = true; SELECT STRING_COL, SUM(INT_COL) FILTER(WHERE INT_COL > "
           "25000), COUNT(*) FILTER(WHERE BOOLEAN_COL = 1 AND INT_COL < 3000) FROM MyTable GROUP BY STRING_COL LIMIT 100000")
    op = GpuInstancePlanMaker().make_instance_plan(parse(sql), ft)
    assert op.one_pass is not None and op.one_pass.num_programs == 2
    op.close()
    _check_vs_oracle(sql, ft)


# ---- CASE statistics: one scan per original filter -------------------------------------------------------------
CASE_STATS_TWINS = [
    # an unfiltered CASE query is a plain AggregationOperator: numEntriesScannedInFilter = its WHERE's scan
    (EXTRA[3], "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 100"),
    # CASE under a FILTER + unfiltered CASE functions, grouped: one info per original filter, as the twin's
    (EXTRA[2], "SELECT SUM(INT_COL) FILTER(WHERE BOOLEAN_COL = 0), SUM(INT_COL) FROM MyTable GROUP BY STATIC_INT_COL"),
    ("SELECT SUM(CASE WHEN NO_INDEX_COL < 5000 THEN INT_COL ELSE 0 END) FROM MyTable WHERE NO_INDEX_COL > 10 "
     "AND INT_COL < 29000", "SELECT SUM(INT_COL) FROM MyTable WHERE NO_INDEX_COL > 10 AND INT_COL < 29000"),
]


@pytest.mark.parametrize("pair", CASE_STATS_TWINS, ids=["where", "filter-group-by", "two-leaf-where"])
def test_gpu_case_entries_scanned_in_filter(pair, ft):
    """The reference evaluates the WHENs in the transform (CaseTransformFunction), so a CASE query scans each
    original filter once; the GPU's branch programs (filter AND WHEN) must not add their scans
    (phip_query_desc.stats_programs). The twin without CASE has the same original filters."""
    pm = GpuInstancePlanMaker()
    counts = []
    for sql in pair:
        op = pm.make_instance_plan(parse(sql), ft)
        blk = op.next_block()
        op.close()
        counts.append(blk.stats.num_entries_scanned_in_filter)
    assert counts[0] == counts[1], counts
