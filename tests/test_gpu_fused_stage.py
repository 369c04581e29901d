"""GPU parity: a fused conjunctive filter + aggregation whose staged sources exceed the segment's stage array
(six scan leaves and four dense value columns: DevSeg.stage holds kMaxStage = 8 sources). The value columns
that do not fit are gathered instead of streamed; results must equal the oracle's bit-exactly."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests.test_gpu_parity import _assert_intermediates_equal

pytestmark = pytest.mark.gpu


def test_gpu_fused_more_sources_than_stage_slots(gpu_lib):
    rng = np.random.default_rng(17)
    n = 150_001
    c = SegmentCreator("fs")
    for k in range(6):
        c.add_column(f"f{k}", DataType.INT, rng.integers(0, 8, n))
    for k in range(4):
        c.add_column(f"v{k}", DataType.INT, rng.integers(0, 50, n) * (k + 1))
    raw = c.build()
    g = GpuSegment(raw)
    try:
        q = ("SELECT SUM(v0), SUM(v1), MIN(v2), MAX(v3) FROM t WHERE f0 < 7 AND f1 > 0 AND f2 <= 6 AND f3 >= 1 "
             "AND f4 < 7 AND f5 > 0")
        qc = parse(q)
        blk = GpuInstancePlanMaker().make_instance_plan(qc, [g]).next_block()
        oblk, exact = executor.execute(qc, [raw])
        _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, exact)
        assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    finally:
        g.destroy()
