"""GPU star-tree path: queries the plan maker answers from the star-tree documents
(GpuStarTreeOperator: host traversal, then the filter + aggregation kernels over the resident star-tree docs)
equal the same queries over the raw segments -- the reference's BaseStarTreeV2Test criterion -- exactly here
(integer-valued metrics), and numDocsScanned counts the star-tree documents the traversal matched."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.engine.startree import GpuStarTreeOperator
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.segment.startree import StarTreeIndexConfig
from pinot_amd.spi import DataType
from tests.test_startree import QUERIES, _star_answer, make_segment

pytestmark = pytest.mark.gpu

EXTRA = [
    "SELECT d2, d4, SUM(m2), COUNT(*) FROM t GROUP BY d2, d4 ORDER BY SUM(m2) DESC, d4 LIMIT 5",
    "SELECT d1, d3, MAX(m) FROM t WHERE d2 BETWEEN 'v02' AND 'v08' GROUP BY d1, d3 ORDER BY d3 DESC, d1 LIMIT 7",
    "SELECT d2, d4, AVG(m), COUNT(*) FROM t GROUP BY d2, d4 ORDER BY AVG(m) DESC, d2, d4 LIMIT 6",  # host trim
]


@pytest.fixture(scope="module", params=[(50, ()), (1, ("d2",)), (10 ** 9, ())], ids=["leaf50", "leaf1", "root"])
def star_segs(gpu_lib, request):
    max_leaf, skip = request.param
    raws = [make_segment(seed=s, n=30_000 + s, max_leaf=max_leaf, skip=skip, name=f"st{s}") for s in range(3)]
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


def _close(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):  # HLL registers: bit-exact
        return np.array_equal(np.asarray(a), np.asarray(b))
    if isinstance(a, tuple):
        return all(_close(x, y) for x, y in zip(a, b))
    return float(a) == float(b)


@pytest.mark.parametrize("sql", QUERIES + EXTRA)
def test_gpu_star_tree_equals_scan(sql, star_segs):
    raws, segs = star_segs
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
    fits = GpuStarTreeOperator.plan(qc, segs, 100_000) is not None
    assert fits == ("d3 = 1" not in sql)
    blk = op.next_block()
    op.close()
    want, _ = executor.execute(qc, raws)
    if fits:
        assert getattr(blk, "star_tree", False)
        assert blk.stats.num_docs_scanned == sum(_star_answer(qc, r)[1] for r in raws)
        assert blk.stats.num_total_docs == sum(r.num_docs for r in raws)
    if not qc.group_by:
        assert all(_close(a, b) for a, b in zip(blk.results, want.results)), (blk.results, want.results)
    else:
        if getattr(blk, "num_groups_trimmed", False):
            assert set(blk.groups) <= set(want.groups)
        else:
            assert set(blk.groups) == set(want.groups)
        for k, v in blk.groups.items():
            assert all(_close(a, b) for a, b in zip(v, want.groups[k])), (k, v, want.groups[k])
    if not qc.order_by:
        qc.limit = 10 ** 9  # no ORDER BY: LIMIT picks arbitrary groups, so compare them all
    got, exp = reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [want]).rows
    if not qc.order_by:
        got, exp = sorted(got, key=repr), sorted(exp, key=repr)
    assert got == exp
    # useStarTree=false: the scan path, same rows
    qc2 = parse(sql)
    qc2.limit = qc.limit
    qc2.options["useStarTree"] = "false"
    op2 = GpuInstancePlanMaker().make_instance_plan(qc2, segs)
    blk2 = op2.next_block()
    op2.close()
    assert not getattr(blk2, "star_tree", False)
    got2 = reduce_blocks(qc2, [blk2]).rows
    if not qc.order_by:
        got2 = sorted(got2, key=repr)
    assert got2 == exp


def test_gpu_benchmark_queries_star_tree(gpu_lib):
    """BenchmarkQueries' star-tree (pinot-perf/.../BenchmarkQueries.java:92-104: split order SORTED_COL, INT_COL;
    SUM__RAW_INT_COL; maxLeafRecords = Integer.MAX_VALUE) with STARTREE_SUM_QUERY / STARTREE_FILTER_QUERY."""
    rng = np.random.default_rng(11)
    n = 200_000
    cfg = StarTreeIndexConfig(["SORTED_COL", "INT_COL"], ["SUM__RAW_INT_COL"], max_leaf_records=2 ** 31 - 1)
    c = SegmentCreator("bq", no_dictionary_columns=["RAW_INT_COL"], star_tree_configs=[cfg])
    c.add_column("SORTED_COL", DataType.INT, (n - np.arange(n)) // 50)  # groups < numGroupsLimit
    c.add_column("INT_COL", DataType.INT, (-np.log(rng.random(n)) / 0.5).astype(np.int64))
    c.add_column("RAW_INT_COL", DataType.INT, rng.integers(0, 10 ** 6, n))
    raw = c.build()
    seg = GpuSegment(raw)
    try:
        for sql in ("SELECT INT_COL, SORTED_COL, SUM(RAW_INT_COL) from MyTable GROUP BY INT_COL, SORTED_COL "
                    "ORDER BY SORTED_COL, INT_COL ASC",
                    "SELECT INT_COL, SORTED_COL, SUM(RAW_INT_COL) FROM MyTable WHERE INT_COL = 0 and SORTED_COL = 1 "
                    "GROUP BY INT_COL, SORTED_COL ORDER BY SORTED_COL, INT_COL ASC"):
            qc = parse(sql)
            blk = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).next_block()
            assert getattr(blk, "star_tree", False)
            want, _ = executor.execute(qc, [raw])
            assert reduce_blocks(qc, [blk]).rows == reduce_blocks(qc, [want]).rows
    finally:
        seg.destroy()
