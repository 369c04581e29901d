"""GPU parity of the result-changing group-by query options (InstancePlanMakerImplV2.applyQueryOptions,
pinot-core/.../plan/maker/InstancePlanMakerImplV2.java:230-300): each option set in the query and the oracle run
under the same option give the same groups and intermediates.

  numGroupsLimit           per segment the first N keys in doc order (InterSegmentAggregationSingleValueQueriesTest
                           .testNumGroupsLimit :763-775 known answer)
  minSegmentGroupTrimSize  each segment's top getTableCapacity(limit, n) groups by the ORDER BY before the merge
                           (GroupByOperator.java:118-133)
  groupTrimThreshold       a combine that can resize mid-merge over several segments is refused (UnsupportedOnGpu,
                           the CPU plan maker answers); one segment, or fewer records than the threshold, stay exact
"""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.reduce import reduce_blocks, trim_groups
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures
from tests.test_gpu_limits import _check, _gpu, _segs


@pytest.fixture(scope="module")
def trim_segments(gpu_lib):
    """3 segments x ~40K docs over 15K keys (distinct SUMs: no ties at any trim boundary)."""
    rng = np.random.default_rng(7)
    raws = []
    for s in range(3):
        n = 40_000 + 777 * s
        c = SegmentCreator(f"qo{s}")
        c.add_column("a", DataType.INT, rng.integers(0, 15_000, n))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 12, 10 ** 12, n))
        c.add_column("f", DataType.INT, rng.integers(0, 1000, n))
        raws.append(c.build())
    segs = _segs(raws)
    yield raws, segs
    for g in segs:
        g.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("limit", [1000, 6582, 6583])
def test_gpu_num_groups_limit_option(gpu_lib, limit):
    """SET numGroupsLimit = n gives the oracle's first-seen groups under that limit (6582 distinct column1 values:
    6582 reaches it, 6583 does not); the server's own limit stays the default."""
    seg = _segs([fixtures.segment_for("test_data_sv")])[0]
    try:
        qc = parse(f"SET numGroupsLimit = {limit}; SELECT column1, COUNT(*), SUM(column3) FROM testTable "
                   "GROUP BY column1 LIMIT 100000")
        gblk = _gpu().make_instance_plan(qc, [seg, seg]).next_block()
        oblk, exact = executor.execute(qc, [seg.segment, seg.segment], num_groups_limit=limit)
        assert oblk.num_groups_limit_reached == (limit <= 6582)
        _check(qc, gblk, oblk, exact)
    finally:
        seg.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["SUM(m) DESC", "SUM(m)", "COUNT(*) DESC, a"])
@pytest.mark.parametrize("min_seg", [200, 1000])
def test_gpu_min_segment_group_trim_size(trim_segments, min_seg, order):
    """Every segment holds ~10K groups > trimSize: each keeps its own top trimSize, the merge sums the survivors
    (a key kept by one segment and trimmed by another carries only the first's share), the server trim runs
    after the merge."""
    raws, segs = trim_segments
    qc = parse(f"SET minSegmentGroupTrimSize = {min_seg}; SELECT a, SUM(m), COUNT(*) FROM t GROUP BY a "
               f"ORDER BY {order} LIMIT 10")
    op = _gpu().make_instance_plan(qc, segs)
    try:
        gblk = op.next_block()
    finally:
        op.close()
    assert getattr(gblk, "segment_trimmed", False)
    oblk, exact = executor.execute(qc, raws, min_segment_group_trim_size=min_seg)
    full, _ = executor.execute(qc, raws)
    assert len(oblk.groups) < len(full.groups)
    oblk = trim_groups(qc, oblk)
    _check(qc, gblk, oblk, exact)
    assert fixtures.rows_match(reduce_blocks(qc, [gblk]).rows, reduce_blocks(qc, [oblk]).rows)


@pytest.mark.gpu
def test_gpu_min_segment_group_trim_size_not_reached(trim_segments):
    """A filter that leaves each segment fewer docs than trimSize: no segment can trim, the one-launch plan
    answers (no per-segment pass) and equals the untrimmed oracle."""
    raws, segs = trim_segments
    qc = parse("SET minSegmentGroupTrimSize = 1000; SELECT a, SUM(m) FROM t WHERE f < 20 GROUP BY a "
               "ORDER BY SUM(m) DESC LIMIT 10")
    gblk = _gpu().make_instance_plan(qc, segs).next_block()
    assert not getattr(gblk, "segment_trimmed", False)
    oblk, exact = executor.execute(qc, raws, min_segment_group_trim_size=1000)
    _check(qc, gblk, oblk, exact)


class _Cpu:
    def __init__(self):
        self.calls = 0

    def make_instance_plan(self, query, segments):
        self.calls += 1
        return type("P", (), {"next_block": lambda s: "cpu", "close": lambda s: None})()


@pytest.mark.gpu
def test_gpu_group_trim_threshold(trim_segments):
    """groupTrimThreshold 10 -> trim threshold max(10, 2 x 5000) = 10000 records: three segments of ~10K groups
    can resize mid-merge (refused, the CPU plan answers); one segment, or a filter leaving fewer records, are
    answered on the GPU exactly."""
    from pinot_amd.engine.plan import UnsupportedOnGpu
    raws, segs = trim_segments
    sql = "SET groupTrimThreshold = 10; SELECT a, SUM(m) FROM t {w} GROUP BY a ORDER BY SUM(m) DESC LIMIT 10"
    qc = parse(sql.format(w=""))
    with pytest.raises(UnsupportedOnGpu):
        _gpu().make_instance_plan(qc, segs).next_block()
    cpu = _Cpu()
    assert _gpu(cpu_plan_maker=cpu).make_instance_plan(qc, segs).next_block() == "cpu" and cpu.calls == 1
    gblk = _gpu().make_instance_plan(qc, segs[:1]).next_block()
    oblk, exact = executor.execute(qc, raws[:1])
    _check(qc, gblk, trim_groups(qc, oblk), exact)
    qc = parse(sql.format(w="WHERE f < 50"))  # ~2K docs per segment: < 10000 records in all
    gblk = _gpu().make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws)
    _check(qc, gblk, trim_groups(qc, oblk), exact)


@pytest.mark.gpu
def test_gpu_default_threshold_overlapping_segments(gpu_lib):
    """The default groupTrimThreshold (10^6) over 12 segments whose per-segment bounds (100K docs, numGroupsLimit
    100K) sum to 1.2M records, but whose keys overlap (150K distinct values in all): the reference's combine never
    holds 10^6 keys, so the GPU answers, equal to the oracle."""
    rng = np.random.default_rng(11)
    raws = []
    for s in range(12):
        c = SegmentCreator(f"ov{s}")
        c.add_column("k", DataType.INT, rng.integers(0, 150_000, 100_000))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, 100_000))
        raws.append(c.build())
    segs = _segs(raws)
    try:
        qc = parse("SELECT k, SUM(m) FROM t GROUP BY k ORDER BY SUM(m) DESC LIMIT 10")
        gblk = _gpu().make_instance_plan(qc, segs).next_block()
        oblk, exact = executor.execute(qc, raws)
        _check(qc, gblk, trim_groups(qc, oblk), exact)
    finally:
        for g in segs:
            g.destroy()
