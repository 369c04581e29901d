"""Doc-order values of value-only dictionary columns (runtime.cpp ensure_vals / load.hip materialize_kernel): a
SUM / MIN / MAX operand with a large dictionary is read as one value per doc instead of id bits + a dictionary
gather. Every path that projects values (fused filter+aggregation, the aggregation kernel's dense and sparse walks,
LDS / HBM / hash group-by tables, filtered aggregations) must give the oracle's answers with the values on
(PHIP_MATERIALIZE_MIN_DICT=0: every numeric dictionary), at the default threshold, and off (PHIP_MATERIALIZE=0);
columns a filter or group-by also reads keep their ids. DISTINCTCOUNTHLL over a large dictionary reads doc-order
registers entries (ensure_hll_doc) the same way: registers bit-exact. INT / LONG values whose range fits fewer bits
than the type are bit-packed at that width relative to the dictionary's minimum (DevCol.vpack; "typed" mode turns
that off): negative values, ranges of 1 value, LONG columns around 2^40 and a 32-bit range are all exact."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures

pytestmark = pytest.mark.gpu

MODES = {"all": {"PHIP_MATERIALIZE_MIN_DICT": "0"}, "default": {}, "off": {"PHIP_MATERIALIZE": "0"},
         "typed": {"PHIP_MATERIALIZE_MIN_DICT": "0", "PHIP_VPACK": "0"}}


@pytest.fixture(scope="module")
def mat_segments(gpu_lib):
    from pinot_amd.engine.segment import GpuSegment
    rng = np.random.default_rng(77)
    raws = []
    for k, n in enumerate((300_001, 2048 * 5 + 3, 70_000)):
        c = SegmentCreator(f"mz{k}")
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        c.add_column("g", DataType.INT, rng.integers(0, 9, n))
        c.add_column("p", DataType.INT, rng.integers(0, 10 ** 9, n))       # large dictionary (> 1 MiB at 300K docs)
        c.add_column("q", DataType.INT, rng.integers(1, 50, n))            # small dictionary
        c.add_column("l", DataType.LONG, rng.integers(-10 ** 15, 10 ** 15, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.normal(0, 1e4, n), 2))
        c.add_column("fl", DataType.FLOAT, np.round(rng.normal(0, 50, n), 1).astype(np.float32))
        c.add_column("ni", DataType.INT, rng.integers(-70_000, 60_000, n))                  # negative, 17 bits
        c.add_column("nl", DataType.LONG, (1 << 40) + rng.integers(-5_000_000, 5_000_000, n))  # LONG in 24 bits
        c.add_column("w", DataType.INT, rng.integers(-2 ** 31, 2 ** 31 - 1, n))            # 32-bit range: typed
        c.add_column("lw", DataType.LONG, rng.integers(0, 2 ** 32, n) - 2 ** 31)            # LONG in 32 bits
        c.add_column("one", DataType.INT, np.full(n, -17 + k))                              # one value: 1 bit
        raws.append(c.build())
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


AGG = [
    "SELECT SUM(p * q), COUNT(*) FROM t WHERE f < 30 AND g BETWEEN 1 AND 4",   # fused
    "SELECT SUM(p), MIN(l), MAX(d), SUM(fl) FROM t WHERE f >= 2",              # dense walk
    "SELECT SUM(l - p), MIN(p), MAX(p) FROM t WHERE f = 7",                     # sparse
    "SELECT SUM(p), MAX(d) FROM t",                                             # no filter
    "SELECT SUM(p), COUNT(*) FROM t WHERE p < 500000000 AND g = 2",             # p also filtered: ids
    "SELECT SUM(p) FILTER (WHERE f < 10), MAX(l) FILTER (WHERE g = 3), COUNT(*) FROM t WHERE q > 5",
    "SELECT DISTINCTCOUNTHLL(p), COUNT(*) FROM t WHERE f < 30",                # doc-order HLL entries
    "SELECT DISTINCTCOUNTHLL(l, 10), DISTINCTCOUNTHLL(q, 10), SUM(p) FROM t WHERE g <> 4",
    "SELECT SUM(ni), MIN(ni), MAX(nl), SUM(nl), SUM(one), MIN(lw) FROM t WHERE f < 30 AND g BETWEEN 1 AND 4",
    "SELECT SUM(ni * q), MAX(w), MIN(w), SUM(lw), SUM(w) FROM t WHERE f >= 2",
    "SELECT SUM(nl - ni), MIN(one), MAX(lw), SUM(one * ni) FROM t WHERE f = 7",
    "SELECT SUM(ni), SUM(nl), SUM(lw), MAX(one) FROM t",
]
GROUP_BY = [
    "SELECT g, SUM(p), MAX(d), COUNT(*) FROM t WHERE f < 50 GROUP BY g LIMIT 1000",
    "SELECT g, q, SUM(l), MIN(p) FROM t GROUP BY g, q LIMIT 100000",
    "SELECT f, SUM(p * q) FROM t WHERE g < 5 GROUP BY f ORDER BY SUM(p * q) DESC LIMIT 10",
    "SELECT p, COUNT(*) FROM t WHERE f < 3 GROUP BY p LIMIT 100000",               # p a key: ids
    "SELECT g, DISTINCTCOUNTHLL(p), SUM(l) FROM t WHERE f < 60 GROUP BY g LIMIT 100",  # HLL in an LDS table
    "SELECT g, q, DISTINCTCOUNTHLL(l) FROM t GROUP BY g, q LIMIT 100000",
    "SELECT g, SUM(ni), MIN(nl), MAX(lw), SUM(one * ni) FROM t WHERE f < 50 GROUP BY g LIMIT 1000",
    "SELECT g, q, SUM(nl), MAX(ni), SUM(w) FROM t GROUP BY g, q LIMIT 100000",
]


def _run(sql, mode, mat_segments, monkeypatch):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    for k in ("PHIP_MATERIALIZE", "PHIP_MATERIALIZE_MIN_DICT"):
        monkeypatch.delenv(k, raising=False)
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    raws, segs = mat_segments
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
    blk = op.next_block()
    op.close()
    oblk, ex = executor.execute(qc, raws)
    return qc, blk, oblk, ex


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("sql", AGG)
def test_gpu_materialized_values_aggregation(sql, mode, mat_segments, monkeypatch):
    from tests.test_gpu_parity import _assert_intermediates_equal
    qc, blk, oblk, ex = _run(sql, mode, mat_segments, monkeypatch)
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("sql", GROUP_BY)
def test_gpu_materialized_values_group_by(sql, mode, mat_segments, monkeypatch):
    from tests.test_gpu_limits import _check
    qc, blk, oblk, ex = _run(sql, mode, mat_segments, monkeypatch)
    got, want = reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [oblk]).rows
    if not qc.order_by:
        _check(qc, blk, oblk, ex)
        got, want = sorted(got), sorted(want)
    assert fixtures.rows_match(got, want)


def test_gpu_materialized_values_memory(mat_segments, monkeypatch):
    """The values are made once per (segment, column) and stay with the segment: num_docs x width bytes."""
    raws, segs = mat_segments
    before = [s.device_bytes() for s in segs]
    _run("SELECT SUM(d) FROM t WHERE f < 40", "all", mat_segments, monkeypatch)
    after = [s.device_bytes() for s in segs]
    _run("SELECT MAX(d) FROM t WHERE g = 1", "all", mat_segments, monkeypatch)
    again = [s.device_bytes() for s in segs]
    assert again == after
    for r, b, a in zip(raws, before, after):
        assert a - b in (0, 8 * r.num_docs)  # (0: an earlier test of this module made them)


def test_gpu_packed_values_memory(mat_segments, monkeypatch):
    """Packed values take whole 2048-doc tiles x bits / 32 + 4 guard words: ni's range needs 17 bits, nl's 24."""
    raws, segs = mat_segments
    for col, bits in (("ni", 17), ("nl", 24)):
        before = [s.device_bytes() for s in segs]
        _run(f"SELECT SUM({col}) FROM t WHERE f < 40", "all", mat_segments, monkeypatch)
        after = [s.device_bytes() for s in segs]
        for r, b, a in zip(raws, before, after):
            assert a - b in (0, 4 * (-(-r.num_docs // 2048) * 2048 * bits // 32 + 4))
