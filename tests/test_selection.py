"""Selection (row-returning) queries on the CPU side: the oracle's SelectionOnlyOperator restatement against the
reference's known answers (InnerSegmentSelectionSingleValueQueriesTest, transcribed into tests/golden/expected.json
by make_fixtures.py), the SQL subset, the broker's selection reduce and the multi-stage leaf composition
(composeSelectTransferableBlock), and metadata-typed group-by keys of the leaf stage."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.leaf_stage import DataSchema, block_schema, compose_select_transferable_block
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.query.context import Function, Identifier
from pinot_amd.query.sql import SqlError, parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures

SEL_CASES = fixtures.expected()["selections"]


def check_selection_case(case, blk):
    """The assertions of the reference test: row count, first row's asserted columns, schema, statistics."""
    assert len(blk.column_names) == case["schema_size"]
    types = dict(zip(blk.column_names, blk.column_types))
    for c, t in case["types"].items():
        if c in types:
            assert types[c] == t, (c, types[c], t)
    assert blk.num_rows == case["num_rows"]
    if case["first"]:
        row = blk.rows[0]
        for c, v in case["first"].items():
            assert row[blk.column_names.index(c)] == v, (c, row)
    assert [blk.stats.num_docs_scanned, blk.stats.num_entries_scanned_post_filter] == case["stats"]
    assert blk.stats.num_total_docs == 30000


@pytest.mark.parametrize("case", SEL_CASES, ids=[c["ref"].split("/")[-1] for c in SEL_CASES])
def test_oracle_selection_known_answers(case):
    blk, _ = executor.execute(parse(case["query"]), [fixtures.test_data_sv_segment()])
    check_selection_case(case, blk)


def test_selection_sql_subset():
    q = parse("SELECT a, b + c, a FROM t WHERE a > 3 LIMIT 7")
    assert q.is_selection and q.limit == 7
    assert q.select_expressions() == [Identifier("a"), Function("plus", (Identifier("b"), Identifier("c")))]
    star = parse("SELECT * FROM t")
    assert [str(e) for e in star.select_expressions(["z", "$docId", "a"])] == ["a", "z"]
    with pytest.raises(SqlError):
        parse("SELECT *, a FROM t")
    assert not parse("SELECT a, COUNT(*) FROM t GROUP BY a").is_selection


def _segments():
    rng = np.random.default_rng(5)
    out = []
    for k in range(3):
        n = 3000 + 501 * k
        c = SegmentCreator(f"sel{k}", no_dictionary_columns=["r"])
        c.add_column("s", DataType.STRING, np.array([f"v{x}" for x in rng.integers(k, 9 + k, n)]))
        c.add_column("i", DataType.INT, rng.integers(-50, 50, n))
        c.add_column("l", DataType.LONG, rng.integers(0, 2 ** 40, n))
        c.add_column("f", DataType.FLOAT, rng.random(n).astype(np.float32))
        c.add_column("r", DataType.LONG, rng.integers(0, 1000, n))
        out.append(c.build())
    return out


def test_oracle_selection_concatenates_segments_up_to_limit():
    segs = _segments()
    q = parse("SELECT s, i, l * r FROM t WHERE i > 40 LIMIT 100")
    blk, _ = executor.execute(q, segs)
    per = [int((executor.OracleSegment(s).values("i") > 40).sum()) for s in segs]
    assert blk.stats.num_docs_scanned == sum(min(100, p) for p in per)
    assert blk.num_rows == min(100, sum(per))
    assert blk.column_types == ["STRING", "INT", "DOUBLE"]
    assert blk.stats.num_entries_scanned_post_filter == blk.stats.num_docs_scanned * 4


def test_selection_broker_reduce_and_leaf_composition():
    segs = _segments()
    q = parse("SELECT i, s, f FROM t WHERE i < -45 LIMIT 1000")
    blk, _ = executor.execute(q, segs)
    table = reduce_blocks(q, [blk, blk])
    assert table.columns == ["i", "s", "f"] and len(table.rows) == min(1000, 2 * blk.num_rows)
    # the stage asks for (s, i) as (STRING, LONG): reordered and converted (TypeUtils.convert)
    desired = DataSchema(["s", "i"], ["STRING", "LONG"])
    tb = compose_select_transferable_block(blk, [Identifier("s"), Identifier("i")], desired)
    assert tb.rows == [[r[1], int(r[0])] for r in blk.rows]
    assert block_schema(blk).column_types == ["INT", "STRING", "FLOAT"]


def test_leaf_group_keys_typed_from_metadata():
    """A LONG group-by key below 2^31 stays LONG in the leaf schema (the column's stored type, not a guess)."""
    c = SegmentCreator("k")
    c.add_column("k", DataType.LONG, np.arange(10) % 3)
    c.add_column("v", DataType.INT, np.arange(10))
    blk, _ = executor.execute(parse("SELECT k, SUM(v) FROM t GROUP BY k"), [c.build()])
    assert block_schema(blk).column_types[0] == "LONG"
