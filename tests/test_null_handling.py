"""Null value vectors and enableNullHandling, host side (no GPU): the SQL front end (IS [NOT] NULL, COUNT(col)), the
segment writer / directory round trip of ``<column>.bitmap.nullvalue``, the oracle's three-valued filters and
null-skipping aggregations against hand-derived answers and the reference's NullEnabledQueriesTest known answers, and
the plan's three-valued filter trees (plan._three_valued) evaluated on the host against the oracle.

The GPU parity of the same semantics is tests/test_gpu_null_handling.py."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd import _lib
from pinot_amd.engine import plan
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.query.sql import parse
from pinot_amd.segment import roaring
from pinot_amd.segment.creator import DEFAULT_NULL_VALUES, SegmentCreator
from pinot_amd.segment.dictionary import Dictionary
from pinot_amd.segment.store import read_segment_dir, write_segment_dir
from pinot_amd.spi import DataType


def _seg(name="n0"):
    """x: INT with nulls at docs 1, 3, 6; y: INT, no nulls; s: STRING with a null at doc 2 (inverted index); r: raw
    LONG with nulls; o: sorted INT with a null at doc 0 (its stored Integer.MIN_VALUE keeps it sorted)."""
    c = SegmentCreator(name, no_dictionary_columns=["r"], inverted_index_columns=["s"])
    c.add_column("o", DataType.INT, [0, 1, 1, 2, 3, 3, 4, 9], nulls=[1, 0, 0, 0, 0, 0, 0, 0])
    c.add_column("x", DataType.INT, [5, 0, 7, 0, 5, 9, 0, 1], nulls=[0, 1, 0, 1, 0, 0, 1, 0])
    c.add_column("y", DataType.INT, [1, 1, 2, 2, 3, 3, 1, 2])
    c.add_column("s", DataType.STRING, ["a", "b", "", "a", "c", "b", "a", "c"], nulls=[0, 0, 1, 0, 0, 0, 0, 0])
    c.add_column("r", DataType.LONG, [10, 20, 30, 40, 50, 60, 70, 80], nulls=[1, 0, 0, 0, 0, 0, 0, 1])
    return c.build()


# ----------------------------------------------------------------------------------------------- SQL
def test_sql_is_null_and_count_column():
    q = parse("SELECT COUNT(*) FROM t WHERE x IS NULL OR NOT (y IS NOT NULL)")
    p0 = q.filter.children[0].predicate
    assert (p0.type, p0.column) == ("IS_NULL", "x")
    assert q.filter.children[1].type == "NOT" and q.filter.children[1].children[0].predicate.type == "IS_NOT_NULL"
    # COUNT(col) keeps its argument only under enableNullHandling (CountAggregationFunction.java:44-66)
    assert parse("SELECT COUNT(x) FROM t").aggregations[0].argument is None
    q = parse("SET enableNullHandling = true; SELECT COUNT(x), COUNT(*), COUNT(1) FROM t")
    assert [a.result_column_name for a in q.aggregations] == ["count(x)", "count(*)"]


# ----------------------------------------------------------------------------------------------- segment
def test_creator_stores_default_null_values_and_the_vector():
    seg = _seg()
    os_ = executor.OracleSegment(seg)
    assert os_.nulls("x").tolist() == [False, True, False, True, False, False, True, False]
    assert os_.values("x")[[1, 3, 6]].tolist() == [DEFAULT_NULL_VALUES[DataType.INT]] * 3  # FieldSpec defaults
    assert os_.values("s")[2] == "null" and os_.values("r")[0] == -2 ** 63
    assert seg.columns["y"].null_vector is None  # (NullValueVectorCreator writes no file without a null)
    assert not os_.nulls("y").any()
    assert seg.columns["x"].null_vector == roaring.serialize([1, 3, 6])


@pytest.mark.parametrize("version", [1, 3])
def test_segment_directory_round_trip_keeps_null_vectors(tmp_path, version):
    seg = _seg()
    back = read_segment_dir(write_segment_dir(seg, str(tmp_path / f"v{version}"), version=version))
    for c in ("x", "s", "r", "y"):
        assert back.columns[c].null_vector == seg.columns[c].null_vector


# ----------------------------------------------------------------------------------------------- oracle
def _mask(seg, where, nh=True):
    return executor.eval_filter(executor.OracleSegment(seg), parse(f"SELECT COUNT(*) FROM t WHERE {where}").filter, nh)


def _docs(m):
    return np.nonzero(m)[0].tolist()


def test_oracle_three_valued_filters_hand_derived():
    seg = _seg()  # x = [5, N, 7, N, 5, 9, N, 1], y = [1, 1, 2, 2, 3, 3, 1, 2]
    assert _docs(_mask(seg, "x = 5")) == [0, 4]
    assert _docs(_mask(seg, "x <> 5")) == [2, 5, 7]                 # nulls are not "not 5"
    assert _docs(_mask(seg, "NOT (x = 5)")) == [2, 5, 7]            # falses of the leaf: NOT x=5 AND NOT null
    assert _docs(_mask(seg, "x = 5", nh=False)) == [0, 4]
    assert _docs(_mask(seg, "NOT (x = 5)", nh=False)) == [1, 2, 3, 5, 6, 7]  # two-valued: nulls hold MIN_VALUE
    assert _docs(_mask(seg, "x IS NULL")) == [1, 3, 6]
    assert _docs(_mask(seg, "NOT (x IS NULL)")) == [0, 2, 4, 5, 7]
    # AND falses = NOT(AND of (trues OR nulls)): NOT(x = 5 AND y = 1) -> docs with a definite false
    assert _docs(_mask(seg, "NOT (x = 5 AND y = 1)")) == [2, 3, 4, 5, 7]
    # OR falses = NOT(OR of (trues OR nulls)): NOT(x = 7 OR y = 3) -> docs where both are definitely false
    assert _docs(_mask(seg, "NOT (x = 7 OR y = 3)")) == [0, 7]
    # x >= 0 does not match the stored null value (Integer.MIN_VALUE): a scan leaf, falses = NOT p AND NOT null
    assert _docs(_mask(seg, "x >= 0")) == [0, 2, 4, 5, 7]
    assert _docs(_mask(seg, "NOT (x >= 0)")) == []
    # an always-true predicate over a column with nulls is a bitmap operator: trues = not null, NOT gives the nulls
    assert _docs(_mask(seg, "x <> 12345")) == [0, 2, 4, 5, 7]
    assert _docs(_mask(seg, "NOT (x <> 12345)")) == [1, 3, 6]
    # an always-false one is EmptyFilterOperator: NOT matches every doc, nulls included
    assert _docs(_mask(seg, "NOT (x = 12345)")) == list(range(8))
    # nested NOT: the inner AND has no nulls of its own (AndFilterOperator.getNulls is empty)
    assert _docs(_mask(seg, "NOT (NOT (x = 5 AND y = 1))")) == [0]


@pytest.mark.parametrize("dt,base", [(DataType.INT, 7), (DataType.LONG, -3), (DataType.FLOAT, 5.5),
                                     (DataType.DOUBLE, -1.25)])
def test_oracle_null_enabled_known_answers(dt, base):
    """NullEnabledQueriesTest.testQueries (pinot-core/src/test/.../queries/NullEnabledQueriesTest.java:93-122,
    473-495): 1000 records per segment, record i holds base + i when i is even and null otherwise; over 4 segment
    copies COUNT(col) = 4 x 500, MIN = base, MAX = base + 998, AVG = the mean of the non-null values, SUM = 4 x their
    sum."""
    vals = np.array([base + i for i in range(1000)])
    nulls = np.arange(1000) % 2 == 1
    raws = []
    for k in range(4):
        c = SegmentCreator(f"ne{k}")
        c.add_column("col", dt, vals, nulls=nulls)
        raws.append(c.build())
    q = parse("SET enableNullHandling = true; SELECT COUNT(col) AS count, MIN(col) AS min, MAX(col) AS max, "
              "AVG(col) AS avg, SUM(col) AS sum FROM testTable LIMIT 1000")
    blk, _ = executor.execute(q, raws)
    row = reduce_blocks(q, [blk]).rows[0]
    s = float(sum(base + i for i in range(0, 1000, 2)))
    assert row[0] == 4 * 500
    assert abs(row[1] - base) < 1e-1 and abs(row[2] - (base + 998)) < 1e-1
    assert abs(row[3] - s / 500) < 1e-1 and abs(row[4] - 4 * s) < 1e-1


def test_oracle_null_results_when_nothing_non_null_is_aggregated():
    seg = _seg()
    q = parse("SET enableNullHandling = true; SELECT SUM(x), MIN(x), COUNT(x), COUNT(*), AVG(r), MAX(x) "
              "FILTER (WHERE y = 3) FROM t WHERE x IS NULL")
    blk, _ = executor.execute(q, [seg, seg])
    assert blk.results[0] is None and blk.results[1] is None and blk.results[5] is None
    assert blk.results[2] == 0 and blk.results[3] == 6
    assert blk.results[4] == (260.0, 6)  # r is null at docs 0 and 7 only: 20 + 40 + 70 per segment copy
    assert reduce_blocks(q, [blk]).rows[0] == [None, None, 0, 6, 260.0 / 6, None]
    # SUM(x * y): a doc is skipped when either column is null
    q = parse("SET enableNullHandling = true; SELECT SUM(x * y), SUM(r) FROM t")
    blk, ex = executor.execute(q, [seg])
    assert ex[0] == 5 * 1 + 7 * 2 + 5 * 3 + 9 * 3 + 1 * 2 and ex[1] == 20 + 30 + 40 + 50 + 60 + 70


# ----------------------------------------------------------------------------------------------- plan trees
class _HostSeg:
    """The GpuSegment surface compile_predicate reads, over an ImmutableSegment (no device)."""

    def __init__(self, seg):
        self.segment = seg
        self.name = seg.name
        self.num_docs = seg.num_docs

    def column_metadata(self, c):
        return self.segment.columns[c].metadata

    def dictionary(self, c):
        ci = self.segment.columns[c]
        m = ci.metadata
        return Dictionary(ci.dictionary, m.data_type, m.cardinality, m.string_width)

    def has_null_vector(self, c):
        return bool(self.segment.columns[c].null_vector)

    def inverted_bytes(self, c, dict_ids):
        ci = self.segment.columns[c]
        off = np.frombuffer(ci.inverted[:4 * (ci.metadata.cardinality + 1)], dtype=">u4").astype(np.int64)
        ids = np.asarray(dict_ids, dtype=np.int64)
        return int((off[ids + 1] - off[ids]).sum())

    def sorted_doc_range(self, c, d):
        p = np.frombuffer(self.segment.columns[c].forward, dtype=">i4").reshape(-1, 2)
        return int(p[d, 0]), int(p[d, 1])


def _eval_tree(os_, t):
    """Host evaluation of a compiled leaf/node tree (the library's leaf semantics)."""
    n = os_.num_docs
    if isinstance(t, plan._Node):
        kids = [_eval_tree(os_, c) for c in t.children]
        if t.op == _lib.NODE_NOT:
            return ~kids[0]
        out = kids[0].copy()
        for k in kids[1:]:
            out = (out & k) if t.op == _lib.NODE_AND else (out | k)
        return out
    if t.kind == _lib.LEAF_MATCH_ALL:
        return np.ones(n, dtype=bool)
    if t.kind == _lib.LEAF_MATCH_NONE:
        return np.zeros(n, dtype=bool)
    if t.kind == _lib.LEAF_NULL:
        m = os_.nulls(t.column)
    elif t.kind == _lib.LEAF_DICT_RANGE:
        ids = os_.dict_ids(t.column)
        m = (ids >= t.lo) & (ids < t.hi)
    elif t.kind == _lib.LEAF_DICT_SET:
        m = np.isin(os_.dict_ids(t.column), t.ids)
    elif t.kind == _lib.LEAF_INVERTED:
        m = np.zeros(n, dtype=bool)
        for d in np.asarray(t.ids).tolist():
            m[os_.inverted_docs(t.column, int(d))] = True
    elif t.kind == _lib.LEAF_RAW_RANGE:  # (integral raw column: lo_int <= v <= hi_int)
        rr = _lib.RawRange.from_buffer_copy(np.asarray(t.ids, dtype=np.int32).tobytes())
        v = os_.values(t.column)
        m = (v >= rr.lo_int) & (v <= rr.hi_int)
    elif t.kind == _lib.LEAF_DOC_RANGES:
        m = np.zeros(n, dtype=bool)
        for a, b in np.asarray(t.ids).reshape(-1, 2):
            m[a:b + 1] = True
        return m
    else:
        raise AssertionError(f"leaf kind {t.kind} not expected here")
    return ~m if t.exclusive else m


WHERES = ["x = 5", "x <> 5", "NOT (x = 5)", "x IS NULL", "x IS NOT NULL", "NOT (x IS NOT NULL)", "x >= 0",
          "NOT (x >= 0)", "NOT (x = 12345)", "NOT (x <> 12345)", "x <> 12345 AND y = 1", "NOT (r > 30)", "x IN (5, 9) AND y = 3", "NOT (x = 5 AND y = 1)", "NOT (x = 7 OR y = 3)",
          "NOT (NOT (x = 5 AND y = 1))", "s = 'a' OR x > 6", "NOT (s = 'a' OR x > 6)", "s IS NULL OR x IS NULL",
          "NOT (s IN ('a', 'b') AND NOT (x BETWEEN 1 AND 7))", "y = 2 AND NOT (x = 7)",
          "o BETWEEN 1 AND 3", "NOT (o BETWEEN 1 AND 3)", "NOT (o > 2 OR s = 'c')", "o IS NULL OR s IS NULL",
          "NOT (s = 'b')", "s <> 'zz'", "NOT (s <> 'zz')",
          # raw leaves folded to constants keep the null bitmap as their nulls
          "NOT (r BETWEEN 50 AND 10)", "NOT (r NOT IN (1.5, 2.5))", "NOT (r IN (2.5) AND x = 5)",
          "r BETWEEN 50 AND 10 OR NOT (x = 5)"]


@pytest.mark.parametrize("nh", [True, False])
@pytest.mark.parametrize("where", WHERES)
def test_plan_three_valued_trees_match_the_oracle(where, nh):
    seg = _seg()
    fc = parse(f"SELECT COUNT(*) FROM t WHERE {where}").filter
    tree = plan.compile_filter(_HostSeg(seg), fc, nh)
    os_ = executor.OracleSegment(seg)
    assert _docs(_eval_tree(os_, tree)) == _docs(executor.eval_filter(os_, fc, nh)), where


# ---- GROUP BY under enableNullHandling: null keys and per-group null results --------------------------------------
# NullHandlingEnabledQueriesTest (pinot-core/src/test/java/org/apache/pinot/queries/NullHandlingEnabledQueriesTest
# .java): one segment queried as 2 servers x 2 segments (NUM_OF_SEGMENT_COPIES = 4 in every count), INT dimensions
# whose null docs store Integer.MIN_VALUE -- which a non-null row may hold too (testMultiColumnGroupBy).
NULL_GB_KATS = [
    # testGroupByOrderByNullsLastUsingOrdinal (:153-176): column1 = null x3, 1, 2, 2
    ("SELECT column1, COUNT(*) FROM testTable GROUP BY column1",
     {"column1": ([None, None, None, 1, 2, 2], None)},
     {(2,): [2 * 4], (1,): [4], (None,): [3 * 4]}),
    # testHavingFilterIsNull / IsNotNull (:178-222): (1, 1), (null, 1), (null, 1); COUNT(column2) per column1
    ("SELECT column1, COUNT(column2) FROM testTable GROUP BY column1",
     {"column1": ([1, None, None], None), "column2": ([1, 1, 1], None)},
     {(None,): [2 * 4], (1,): [4]}),
    # testMultiColumnGroupBy (:778-806): a stored Integer.MIN_VALUE is a value, a null doc the null key
    ("SELECT count(*), column1, column2 FROM testTable GROUP BY column1, column2",
     {"column1": ([None, None, None, 1, 1, 1], None),
      "column2": ([None, 1, 1, 1, None, -2 ** 31], None)},
     {(None, None): [4], (None, 1): [2 * 4], (1, 1): [4], (1, None): [4], (1, -2 ** 31): [4]}),
    # testGroupByOrderBy (:834-858): null, 1, 1, 2, 3
    ("SELECT count(*), column1 FROM testTable GROUP BY column1",
     {"column1": ([None, 1, 1, 2, 3], None)},
     {(1,): [2 * 4], (2,): [4], (3,): [4], (None,): [4]}),
]


def _kat_segment(cols):
    c = SegmentCreator("kat")
    for name, (vals, _) in cols.items():
        nulls = [v is None for v in vals]
        c.add_column(name, DataType.INT, [0 if v is None else v for v in vals], nulls=nulls if any(nulls) else None)
    return c.build()


@pytest.mark.parametrize("sql,cols,expect", NULL_GB_KATS, ids=[k[0][:48] for k in NULL_GB_KATS])
def test_oracle_null_group_keys_known_answers(sql, cols, expect):
    """The oracle's null-aware GROUP BY reproduces the reference's rows: the null docs of a group-by column form the
    None key, COUNT(col) skips null inputs (the blocks of 2 x 2 segment copies merged as the broker would)."""
    from pinot_amd.engine.results import merge_intermediate
    seg = _kat_segment(cols)
    qc = parse("SET enableNullHandling = true; " + sql)
    blk, _ = executor.execute(qc, [seg, seg])
    merged = {}
    for _ in range(2):  # two servers, each the same two segments
        for k, v in blk.groups.items():
            merged[k] = [merge_intermediate(a.function, x, y) for a, x, y in zip(qc.aggregations, merged[k], v)] \
                if k in merged else list(v)
    assert merged == expect


def test_oracle_per_group_null_results_hand_derived():
    """SUM / MIN / MAX / AVG over a group whose inputs are all null are None; COUNT(col) is 0; a null key and null
    results together; numGroupsLimit counts the null key in first-seen order."""
    c = SegmentCreator("g")
    c.add_column("k", DataType.INT, [1, 1, 2, 0, 2, 3, 0], nulls=[0, 0, 0, 1, 0, 0, 1])
    c.add_column("v", DataType.LONG, [10, 0, 0, 5, 0, 7, 0], nulls=[0, 1, 1, 0, 1, 0, 1])
    seg = c.build()
    qc = parse("SET enableNullHandling = true; SELECT k, SUM(v), MIN(v), COUNT(v), COUNT(*), AVG(v) FROM t GROUP BY k")
    blk, ex = executor.execute(qc, [seg])
    assert blk.groups[(1,)] == [10.0, 10.0, 1, 2, (10.0, 1)]
    assert blk.groups[(2,)] == [None, None, 0, 2, None]
    assert blk.groups[(None,)] == [5.0, 5.0, 1, 2, (5.0, 1)]
    assert blk.groups[(3,)] == [7.0, 7.0, 1, 1, (7.0, 1)]
    assert ex[(1,)][0] == 10 and ex[(2,)][0] is None
    # numGroupsLimit 2: first seen are 1 (doc 0) and 2 (doc 2); the null key (doc 3) is the third -- dropped
    blk2, _ = executor.execute(qc, [seg], num_groups_limit=2)
    assert set(blk2.groups) == {(1,), (2,)} and blk2.num_groups_limit_reached


def test_oracle_filtered_group_by_null_handling_hand_derived():
    """FILTER + GROUP BY under null handling (FilteredGroupByOperator over the null-aware generator): a FILTER passes
    the docs where it is TRUE (a null comparison is not), the infos share the generator (the main info's docs make
    every group), a nullable function whose info never reached a group -- or reached it with null inputs only -- is
    None (ObjectGroupByResultHolder), COUNT 0; numDocsScanned sums the infos' docs."""
    c = SegmentCreator("fg")
    c.add_column("g", DataType.INT, [1, 1, 2, 0, 3], nulls=[0, 0, 0, 1, 0])
    c.add_column("k", DataType.INT, [5, 0, 7, 9, 0], nulls=[0, 1, 0, 0, 1])
    c.add_column("d", DataType.INT, [10, 1, 0, 8, 6], nulls=[0, 0, 1, 0, 0])
    seg = c.build()
    qc = parse("SET enableNullHandling = true; SELECT g, SUM(k) FILTER (WHERE d > 3), COUNT(k) FILTER (WHERE d > 3), "
               "COUNT(*) FROM t GROUP BY g")
    blk, ex = executor.execute(qc, [seg])
    # info d > 3: docs 0 (g 1, k 5), 3 (g null, k 9), 4 (g 3, k null); the main info: every doc
    assert blk.groups == {(1,): [5.0, 1, 2], (2,): [None, 0, 1], (None,): [9.0, 1, 1], (3,): [None, 0, 1]}
    assert ex[(1,)][0] == 5 and ex[(2,)][0] is None
    assert blk.stats.num_docs_scanned == 3 + 5
    assert blk.stats.num_entries_scanned_post_filter == 3 * 2 + 5 * 1  # (g, k) per filtered doc; g per main doc
