"""The fused filter + aggregation path (filter.hip fused_tile): conjunctive programs without group-by / HLL
aggregate inside the filter kernel, value columns streamed with the tile or gathered per matched doc. Every
variant (PHIP_FUSE=0 keeps the separate aggregation kernel; PHIP_STREAM_VALUES forces streaming on / off)
must give the oracle's answers: ragged tiles, sorted-column doc ranges cutting tiles, raw columns, INT /
LONG / DOUBLE dictionaries, several aggregations, empty results."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType

pytestmark = pytest.mark.gpu

VARIANTS = [("0", None), ("1", "0"), ("1", "1"), ("1", None)]


@pytest.fixture(scope="module")
def fused_segments(gpu_lib):
    from pinot_amd.engine.segment import GpuSegment
    rng = np.random.default_rng(51)
    raws = []
    for k, n in enumerate((2048 * 29 + 777, 100_003, 2048 * 3)):
        c = SegmentCreator(f"fz{k}", no_dictionary_columns=["r"])
        c.add_column("t", DataType.INT, np.sort(rng.integers(0, 40, n)))          # sorted -> doc ranges
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        c.add_column("g", DataType.INT, rng.integers(0, 7, n))
        c.add_column("p", DataType.INT, rng.integers(0, 2_000_000, n))             # ~21-bit dictionary
        c.add_column("l", DataType.LONG, rng.integers(-10 ** 12, 10 ** 12, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.normal(0, 1e3, n), 3))
        c.add_column("r", DataType.INT, rng.integers(-2 ** 31, 2 ** 31 - 1, n))
        raws.append(c.build())
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


QUERIES = [
    "SELECT SUM(p * g) FROM t WHERE f < 30 AND g BETWEEN 1 AND 4",
    "SELECT SUM(p), COUNT(*), MIN(d), MAX(l) FROM t WHERE t BETWEEN 7 AND 21 AND f >= 50",
    "SELECT SUM(l - p), SUM(d), COUNT(*) FROM t WHERE t = 13 AND g = 3",
    "SELECT SUM(r), MAX(r) FROM t WHERE f < 90",
    "SELECT SUM(d * g), MIN(p) FROM t WHERE t > 38 AND f < 2",
    "SELECT COUNT(*), SUM(p) FROM t WHERE f > 1000",
    "SELECT SUM(p + l) FROM t WHERE t < 5",
]


@pytest.mark.parametrize("fuse,stream", VARIANTS, ids=["unfused", "gather", "stream", "auto"])
@pytest.mark.parametrize("sql", QUERIES)
def test_gpu_fused_aggregation_vs_oracle(sql, fuse, stream, fused_segments, monkeypatch):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from tests.test_gpu_parity import _assert_intermediates_equal
    monkeypatch.setenv("PHIP_FUSE", fuse)
    if stream is None:
        monkeypatch.delenv("PHIP_STREAM_VALUES", raising=False)
    else:
        monkeypatch.setenv("PHIP_STREAM_VALUES", stream)
    raws, segs = fused_segments
    qc = parse(sql)
    blk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
    oblk, ex = executor.execute(qc, raws)
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
    if fuse == "1" and "SUM(p * g)" in sql:
        assert blk.agg_kernel_ms == 0.0 and blk.filter_kernel_ms > 0  # one kernel did both


@pytest.mark.parametrize("fuse", ["0", "1"])
@pytest.mark.parametrize("layout", ["unsorted", "sorted"])
def test_gpu_fused_ssb_q1(layout, fuse, gpu_lib, monkeypatch):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from tests.test_gpu_parity import _assert_intermediates_equal
    from tools import ssb
    monkeypatch.setenv("PHIP_FUSE", fuse)
    qs = ["Q1.1", "Q1.2", "Q1.3"]
    raws = ssb.make_segments(1, ssb.columns_for(qs), seed=3, segment_rows=1_000_000, layout=layout)
    segs = [GpuSegment(r) for r in raws]
    try:
        for q in qs:
            qc = parse(ssb.SSB_QUERIES[q])
            blk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
            oblk, ex = executor.execute(qc, raws)
            assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
            _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
    finally:
        for s in segs:
            s.destroy()


@pytest.mark.parametrize("fold", ["0", "1"])
@pytest.mark.parametrize("fuse", ["0", "1"])
@pytest.mark.parametrize("sql", QUERIES)
def test_gpu_folded_finalize(sql, fuse, fold, fused_segments, monkeypatch):
    """PHIP_FOLD_FINAL=1: the last workgroup of the plan's last kernel finalizes (agg_common.h finalize_tail, a
    two-level sharded ticket) instead of a finalize launch; 0 (default) keeps the launch -- same answers."""
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from tests.test_gpu_parity import _assert_intermediates_equal
    monkeypatch.setenv("PHIP_FUSE", fuse)
    monkeypatch.setenv("PHIP_FOLD_FINAL", fold)
    raws, segs = fused_segments
    qc = parse(sql)
    op = GpuInstancePlanMaker().make_instance_plan(qc, segs)
    oblk, ex = executor.execute(qc, raws)
    for _ in range(3):  # (the ticket counter resets between executions)
        blk = op.next_block()
        assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
        _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
    op.close()


@pytest.mark.parametrize("fuse", ["0", "1"])
def test_gpu_ext_launch_events(fuse, fused_segments, monkeypatch):
    """PHIP_EXT_EVENTS=1: a one-kernel plan's timing events ride on its dispatch packet (hipExtLaunchKernel) -- same
    answers, a positive kernel time."""
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from tests.test_gpu_parity import _assert_intermediates_equal
    monkeypatch.setenv("PHIP_FUSE", fuse)
    monkeypatch.setenv("PHIP_EXT_EVENTS", "1")
    raws, segs = fused_segments
    for sql in (QUERIES[0], QUERIES[3], "SELECT COUNT(*) FROM t WHERE f < 20"):
        qc = parse(sql)
        blk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
        oblk, ex = executor.execute(qc, raws)
        _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
        assert (blk.filter_kernel_ms or 0) + (blk.agg_kernel_ms or 0) > 0
