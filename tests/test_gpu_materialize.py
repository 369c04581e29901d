"""Doc-order values of value-only dictionary columns (runtime.cpp ensure_vals / load.hip materialize_kernel): a
SUM / MIN / MAX operand with a large dictionary is read as one value per doc instead of id bits + a dictionary
gather. Every path that projects values (fused filter+aggregation, the aggregation kernel's dense and sparse walks,
LDS / HBM / hash group-by tables, filtered aggregations) must give the oracle's answers with the values on
(PHIP_MATERIALIZE_MIN_DICT=0: every numeric dictionary), at the default threshold, and off (PHIP_MATERIALIZE=0);
columns a filter or group-by also reads keep their ids. DISTINCTCOUNTHLL over a large dictionary reads doc-order
registers entries (ensure_hll_doc) the same way: registers bit-exact."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures

pytestmark = pytest.mark.gpu

MODES = {"all": {"PHIP_MATERIALIZE_MIN_DICT": "0"}, "default": {}, "off": {"PHIP_MATERIALIZE": "0"}}


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
]
GROUP_BY = [
    "SELECT g, SUM(p), MAX(d), COUNT(*) FROM t WHERE f < 50 GROUP BY g LIMIT 1000",
    "SELECT g, q, SUM(l), MIN(p) FROM t GROUP BY g, q LIMIT 100000",
    "SELECT f, SUM(p * q) FROM t WHERE g < 5 GROUP BY f ORDER BY SUM(p * q) DESC LIMIT 10",
    "SELECT p, COUNT(*) FROM t WHERE f < 3 GROUP BY p LIMIT 100000",               # p a key: ids
    "SELECT g, DISTINCTCOUNTHLL(p), SUM(l) FROM t WHERE f < 60 GROUP BY g LIMIT 100",  # HLL in an LDS table
    "SELECT g, q, DISTINCTCOUNTHLL(l) FROM t GROUP BY g, q LIMIT 100000",
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
