"""Filtered aggregations (`agg FILTER(WHERE ...)`) on the host side: parsing, the
oracle's FilteredAggregationOperator semantics, and the property the reference's
FilteredAggregationsTest checks (a filtered aggregation equals the same aggregation under
main AND filter)."""
import numpy as np

from oracle import executor
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.query.context import FilterClause
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType


def _segments():
    rng = np.random.default_rng(9)
    out = []
    for k in range(2):
        n = 20_000 + k
        c = SegmentCreator(f"f{k}", inverted_index_columns=["b"])
        c.add_column("a", DataType.INT, rng.integers(0, 1000, n))
        c.add_column("b", DataType.INT, rng.integers(0, 30, n))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        out.append(c.build())
    return out


def test_parse_filter_clause():
    qc = parse("SELECT SUM(a) FILTER(WHERE b = 3), MAX(a), COUNT(*) FILTER(WHERE b = 3) FROM t WHERE a > 10")
    assert [a.function for a in qc.aggregations] == ["sum", "max", "count"]
    assert qc.aggregations[0].filter is not None and qc.aggregations[1].filter is None
    assert qc.aggregations[0].filter == qc.aggregations[2].filter
    assert isinstance(qc.select[0][0], FilterClause)


def test_filtered_equals_main_and_filter():
    segs = _segments()
    q = ("SELECT SUM(m) FILTER(WHERE b IN (1, 2, 3)), MAX(a) FILTER(WHERE b IN (1, 2, 3)), "
         "MIN(m) FILTER(WHERE a < 100), COUNT(*) FROM t WHERE a BETWEEN 50 AND 900")
    blk, ex = executor.execute(parse(q), segs)
    ref1, ex1 = executor.execute(parse("SELECT SUM(m), MAX(a) FROM t WHERE a BETWEEN 50 AND 900 AND b IN (1, 2, 3)"), segs)
    ref2, _ = executor.execute(parse("SELECT MIN(m) FROM t WHERE a BETWEEN 50 AND 900 AND a < 100"), segs)
    ref3, _ = executor.execute(parse("SELECT COUNT(*) FROM t WHERE a BETWEEN 50 AND 900"), segs)
    assert ex[0] == ex1[0] and blk.results[1] == ref1.results[1]
    assert blk.results[2] == ref2.results[0] and blk.results[3] == ref3.results[0]
    # statistics: one entry per distinct filter, summed (FilteredAggregationOperator.java:97-99)
    assert blk.stats.num_docs_scanned == (ref1.stats.num_docs_scanned + ref2.stats.num_docs_scanned
                                          + ref3.stats.num_docs_scanned)
    rt = reduce_blocks(parse(q), [blk])
    assert rt.rows[0][3] == ref3.results[0]
