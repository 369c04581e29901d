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


# ---------------------------------------------------------------- FILTER + GROUP BY, CASE (f1)
def _ft_segments(n=30_000, seed=5):
    """FilteredAggregationsTest's table (pinot-core/src/test/java/org/apache/pinot/queries/FilteredAggregationsTest.java:116-129):
    INT_COL = NO_INDEX_COL = row number, STATIC_INT_COL = 10, BOOLEAN_COL random, STRING_COL 4 random letters;
    INT_COL with an inverted index; two segments."""
    rng = np.random.default_rng(seed)
    letters = np.array(list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"))
    out = []
    for k in range(2):
        c = SegmentCreator(f"ft{k}", inverted_index_columns=["INT_COL"])
        c.add_column("INT_COL", DataType.INT, np.arange(n))
        c.add_column("NO_INDEX_COL", DataType.INT, np.arange(n))
        c.add_column("STATIC_INT_COL", DataType.INT, np.full(n, 10))
        c.add_column("BOOLEAN_COL", DataType.INT, rng.integers(0, 2, n))
        s = ["".join(x) for x in letters[rng.integers(0, 52, (n, 4))]]
        c.add_column("STRING_COL", DataType.STRING, s)
        out.append(c.build())
    return out


# (filter query, equivalent query) pairs from FilteredAggregationsTest (group-by and CASE cases)
FT_PAIRS = [
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 9999) FROM MyTable WHERE INT_COL < 1000000 GROUP BY BOOLEAN_COL",
     "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 9999 AND INT_COL < 1000000 GROUP BY BOOLEAN_COL"),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 25000) testSum FROM MyTable GROUP BY BOOLEAN_COL ORDER BY BOOLEAN_COL",
     "SELECT SUM(INT_COL) testSum FROM MyTable WHERE INT_COL > 25000 GROUP BY BOOLEAN_COL ORDER BY BOOLEAN_COL"),
    ("SET filteredAggregationsSkipEmptyGroups=true; SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 25000) testSum "
     "FROM MyTable GROUP BY BOOLEAN_COL, STRING_COL ORDER BY BOOLEAN_COL, STRING_COL",
     "SELECT SUM(INT_COL) testSum FROM MyTable WHERE INT_COL > 25000 GROUP BY BOOLEAN_COL, STRING_COL "
     "ORDER BY BOOLEAN_COL, STRING_COL"),
    ("SELECT SUM(INT_COL), SUM(INT_COL) FILTER(WHERE INT_COL > 25000) AS total_sum FROM MyTable "
     "GROUP BY BOOLEAN_COL ORDER BY BOOLEAN_COL",
     "SELECT SUM(INT_COL), SUM(CASE WHEN INT_COL > 25000 THEN INT_COL ELSE 0 END) AS total_sum FROM MyTable "
     "GROUP BY BOOLEAN_COL ORDER BY BOOLEAN_COL"),
    ("SELECT AVG(INT_COL) FILTER(WHERE INT_COL > 25000) testAvg, SUM(INT_COL) FILTER(WHERE INT_COL > 25000) testSum "
     "FROM MyTable GROUP BY BOOLEAN_COL ORDER BY BOOLEAN_COL",
     "SELECT AVG(INT_COL) testAvg, SUM(INT_COL) testSum FROM MyTable WHERE INT_COL > 25000 "
     "GROUP BY BOOLEAN_COL ORDER BY BOOLEAN_COL"),
    ("SELECT MIN(INT_COL) FILTER(WHERE NO_INDEX_COL > 29990) AS total_min, "
     "MAX(INT_COL) FILTER(WHERE INT_COL > 29990) AS total_max, "
     "SUM(INT_COL) FILTER(WHERE NO_INDEX_COL < 5000) AS total_sum, "
     "MAX(NO_INDEX_COL) FILTER(WHERE NO_INDEX_COL < 5000) AS total_max2 "
     "FROM MyTable GROUP BY BOOLEAN_COL ORDER BY BOOLEAN_COL",
     "SELECT MIN(CASE WHEN (NO_INDEX_COL > 29990) THEN INT_COL ELSE 99999 END) AS total_min, "
     "MAX(CASE WHEN (INT_COL > 29990) THEN INT_COL ELSE 0 END) AS total_max, "
     "SUM(CASE WHEN (NO_INDEX_COL < 5000) THEN INT_COL ELSE 0 END) AS total_sum, "
     "MAX(CASE WHEN (NO_INDEX_COL < 5000) THEN NO_INDEX_COL ELSE 0 END) AS total_max2 "
     "FROM MyTable GROUP BY BOOLEAN_COL ORDER BY BOOLEAN_COL"),
    ("SELECT AVG(INT_COL) FILTER(WHERE INT_COL > 25000) testAvg, SUM(INT_COL) FILTER(WHERE INT_COL > 25000) "
     "testSum FROM MyTable GROUP BY BOOLEAN_COL ORDER BY testAvg",
     "SELECT AVG(INT_COL) testAvg, SUM(INT_COL) testSum FROM MyTable WHERE INT_COL > 25000 GROUP BY BOOLEAN_COL "
     "ORDER BY testAvg"),
    ("SELECT SUM(INT_COL), SUM(INT_COL) FILTER(WHERE INT_COL < 5000) AS total_sum, "
     "SUM(INT_COL) FILTER(WHERE INT_COL > 12345) AS total_sum2 FROM MyTable",
     "SELECT SUM(INT_COL), SUM(CASE WHEN INT_COL < 5000 THEN INT_COL ELSE 0 END) AS total_sum, "
     "SUM(CASE WHEN INT_COL > 12345 THEN INT_COL ELSE 0 END) AS total_sum2 FROM MyTable"),
]


def test_parse_set_options_and_case():
    qc = parse("SET filteredAggregationsSkipEmptyGroups=true; SET numGroupsLimit = '7'; "
               "SELECT SUM(CASE WHEN a > 5 THEN b WHEN a < 2 THEN 7 ELSE 0 END) FROM t GROUP BY g")
    assert qc.options == {"filteredAggregationsSkipEmptyGroups": "true", "numGroupsLimit": "7"}
    arg = qc.aggregations[0].argument
    assert arg.name == "case" and len(arg.args) == 5 and arg.args[-1].value == 0
    from pinot_amd.query.context import columns_of
    assert columns_of(arg) == ["a", "b"]


def test_oracle_filter_pairs_like_reference():
    """The reference's own check (FilteredAggregationsTest.testQuery): the FILTER query and its WHERE / CASE
    twin give the same rows -- here on the oracle, which evaluates CASE per doc and FILTER per info."""
    segs = _ft_segments()
    for fq, nq in FT_PAIRS:
        a = reduce_blocks(parse(fq), [executor.execute(parse(fq), segs)[0]] * 2)
        b = reduce_blocks(parse(nq), [executor.execute(parse(nq), segs)[0]] * 2)
        assert a.rows == b.rows, (fq, a.rows, b.rows)


def test_oracle_filtered_group_by_semantics():
    segs = _segments()
    q = parse("SELECT SUM(m) FILTER(WHERE b < 3), COUNT(*), MIN(m) FILTER(WHERE a < 5) FROM t WHERE a < 900 GROUP BY b")
    blk, ex = executor.execute(q, segs)
    main, _ = executor.execute(parse("SELECT COUNT(*) FROM t WHERE a < 900 GROUP BY b"), segs)
    assert set(blk.groups) == set(main.groups)                 # the main info generates every group
    sub, _ = executor.execute(parse("SELECT SUM(m) FROM t WHERE a < 900 AND b < 3 GROUP BY b"), segs)
    for k, v in blk.groups.items():
        assert v[1] == main.groups[k][0]
        if k in sub.groups:
            assert v[0] == sub.groups[k][0]
        else:
            assert v[0] == 0.0                                  # holder default (ensureCapacity)
    # numDocsScanned sums the three infos (FilteredGroupByOperator.java:145-149)
    s2, _ = executor.execute(parse("SELECT MIN(m) FROM t WHERE a < 900 AND a < 5 GROUP BY b"), segs)
    assert blk.stats.num_docs_scanned == (main.stats.num_docs_scanned + sub.stats.num_docs_scanned
                                          + s2.stats.num_docs_scanned)
    # skip-empty-groups: only groups some filter reached
    q.options["filteredAggregationsSkipEmptyGroups"] = "true"
    q2 = parse("SET filteredAggregationsSkipEmptyGroups=true; "
               "SELECT SUM(m) FILTER(WHERE b < 3) FROM t WHERE a < 900 GROUP BY b")
    blk2, _ = executor.execute(q2, segs)
    assert set(blk2.groups) == set(sub.groups)
