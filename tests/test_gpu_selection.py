"""GPU parity for selection (row-returning) queries -- the leaf of a multi-stage join:
GpuSelectionOperator (one filter launch + select.hip) against the reference's known answers
(InnerSegmentSelectionSingleValueQueriesTest) and against the oracle's SelectionOnlyOperator restatement, row by
row and bit-exactly (INT/LONG values, STRING values, FLOAT/DOUBLE bits, a op b in double), with LIMITs that cut
inside a tile, a segment and the combine; statistics per segment; then the joined-SSB lineorder leaf through
GpuLeafStageOperator."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.leaf_stage import DataSchema, GpuLeafStageOperator
from pinot_amd.engine.plan import GpuInstancePlanMaker, GpuSelectionOperator
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures
from tests.test_selection import SEL_CASES, check_selection_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sv(gpu_lib):
    s = GpuSegment(fixtures.test_data_sv_segment())
    yield s
    s.destroy()


@pytest.mark.parametrize("case", SEL_CASES, ids=[c["ref"].split("/")[-1] for c in SEL_CASES])
def test_gpu_selection_known_answers(case, sv):
    op = GpuInstancePlanMaker().make_instance_plan(case["query"], [sv])
    assert isinstance(op, GpuSelectionOperator)
    blk = op.next_block()
    op.close()
    check_selection_case(case, blk)


def _segments():
    rng = np.random.default_rng(17)
    out = []
    for k in range(3):
        n = 70_000 + 12_345 * k  # ragged last tiles
        c = SegmentCreator(f"gs{k}", no_dictionary_columns=["r", "rd", "rs"], inverted_index_columns=["h"])
        c.add_column("s", DataType.STRING, np.array([f"name{x:04d}" for x in rng.integers(50 * k, 400 + 60 * k, n)]))
        c.add_column("h", DataType.INT, rng.integers(0, 9 + k, n))
        c.add_column("i", DataType.INT, rng.integers(-10 ** 6, 10 ** 6, n))
        c.add_column("l", DataType.LONG, rng.integers(-2 ** 50, 2 ** 50, n))
        c.add_column("f", DataType.FLOAT, (rng.random(n) * 100).astype(np.float32))
        c.add_column("d", DataType.DOUBLE, rng.normal(0, 1e3, n))
        c.add_column("r", DataType.LONG, rng.integers(0, 10 ** 9, n))
        c.add_column("rd", DataType.DOUBLE, rng.random(n))
        c.add_column("srt", DataType.INT, np.sort(rng.integers(0, 5000, n)))
        # raw STRING (rows' bytes gathered by locator on the device): empty, multi-byte and long values
        words = np.array(["", "é", "zz-top", "naïve", "日本", "x" * 40] + [f"w{j}" for j in range(300 + 50 * k)],
                         dtype=object)
        c.add_column("rs", DataType.STRING, words[rng.integers(0, len(words), n)])
        out.append(c.build())
    return out


@pytest.fixture(scope="module")
def segs(gpu_lib):
    raws = _segments()
    g = [GpuSegment(r) for r in raws]
    yield raws, g
    for s in g:
        s.destroy()


def _same(a, b):
    if isinstance(a, float) or isinstance(b, float):
        return np.float64(a).tobytes() == np.float64(b).tobytes() or (a != a and b != b)
    return a == b


QUERIES = [
    "SELECT s, i, l, f, d, r, rd FROM t LIMIT 1000000",                        # every row, every type
    "SELECT * FROM t WHERE h = 3 LIMIT 1000000",                                # inverted leaf, SELECT *
    "SELECT l, s FROM t WHERE i BETWEEN -1000 AND 50000 AND h <> 2 LIMIT 1000000",
    "SELECT i + r, l - i, d * f, s FROM t WHERE srt BETWEEN 100 AND 900 OR rd < 0.01 LIMIT 1000000",
    "SELECT s, d FROM t WHERE r > 999000000 LIMIT 1000000",                     # raw-column filter, sparse
    "SELECT s, i FROM t WHERE h = 100 LIMIT 50",                                # nothing matches
    "SELECT s, i, srt FROM t WHERE h IN (1, 4) LIMIT 10",                       # default-sized LIMIT: first segment
    "SELECT i, s FROM t WHERE i > 0 LIMIT 3000",                                # cuts inside a tile of segment 0
    "SELECT i, s FROM t WHERE i > 900000 LIMIT 7000",                           # ends inside segment 1
    "SELECT i, i, s FROM t WHERE f < 1.5 LIMIT 1000000",                        # a repeated expression
    "SELECT rs, i, s, rs FROM t WHERE h = 2 LIMIT 1000000",                     # raw STRING values
    "SELECT rs FROM t WHERE rs >= 'w2' AND rs < 'x' LIMIT 5000",                # raw STRING leaf and values
    "SELECT rs, i FROM t WHERE h = 100 LIMIT 50",                               # raw STRING, nothing matches
]


@pytest.mark.parametrize("sql", QUERIES)
def test_gpu_selection_vs_oracle(sql, segs):
    raws, g = segs
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, g)
    blk = op.next_block()
    op.close()
    oblk, _ = executor.execute(qc, raws)
    assert blk.column_names == oblk.column_names and blk.column_types == oblk.column_types
    assert blk.num_rows == oblk.num_rows
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert blk.stats.num_entries_scanned_post_filter == oblk.stats.num_entries_scanned_post_filter
    assert blk.stats.num_segments_matched == oblk.stats.num_segments_matched
    for ra, rb in zip(blk.rows, oblk.rows):
        assert all(_same(x, y) for x, y in zip(ra, rb)), (ra, rb)


def test_gpu_selection_repeatable_and_concurrent_plans(segs):
    """A prepared selection plan re-executes to the same rows (its tile ranks and bases are per execution)."""
    raws, g = segs
    qc = parse("SELECT l, s FROM t WHERE h = 5 LIMIT 1000000")
    op = GpuInstancePlanMaker().make_instance_plan(qc, g)
    a = op.next_block().rows
    b = op.next_block().rows
    op.close()
    assert a == b and len(a) > 0


def test_gpu_ssb_lineorder_join_leaf(gpu_lib):
    """Joined SSB as written (Q2.1's lineorder side): the leaf stage projects the join keys and the metric of the
    lineorder rows that pass the leaf filter -- here every row, and a filtered variant -- and ships them as a row
    block of the stage's schema (INT keys widened to LONG by TypeUtils.convert)."""
    from tools import ssb
    raws = ssb.make_segments(1, ["LO_ORDERDATE", "LO_PARTKEY", "LO_SUPPKEY", "LO_REVENUE", "LO_QUANTITY"],
                             segments=[0, 1], segment_rows=500_000)
    g = [GpuSegment(r) for r in raws]
    try:
        for where in ("", " WHERE LO_QUANTITY < 10"):
            sql = f"SELECT LO_ORDERDATE, LO_PARTKEY, LO_SUPPKEY, LO_REVENUE FROM lineorder{where} LIMIT 100000000"
            desired = DataSchema(["LO_ORDERDATE", "LO_PARTKEY", "LO_SUPPKEY", "LO_REVENUE"],
                                 ["LONG", "LONG", "LONG", "LONG"])
            leaf = GpuLeafStageOperator(sql, g, desired)
            tb = leaf.next_block()
            eos = leaf.next_block()
            oblk, _ = executor.execute(parse(sql), raws)
            assert eos.is_end_of_stream and eos.stats["numDocsScanned"] == oblk.stats.num_docs_scanned
            assert tb.schema == desired and len(tb.rows) == oblk.num_rows
            assert tb.rows == [[int(v) for v in r] for r in oblk.rows]
    finally:
        for s in g:
            s.destroy()
