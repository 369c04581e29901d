"""numEntriesScannedInFilter of ORs on one scanned column: the broker's MergeEqInFilterOptimizer
(pinot-core/.../query/optimizer/filter/MergeEqInFilterOptimizer.java:40-120) merges EQ / IN predicates of one column
under an OR into one IN -- one scan operator, numDocs entries -- and leaves range predicates apart: an OR of two
ranges is two scan operators, 2 x numDocs entries (ScanBasedFilterOperator counts one entry per doc scanned,
SVScanDocIdIterator.java:88,106). Doc sets and aggregations equal the oracle's either way."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("where, scans", [("c > 5 OR c < 2", 2), ("c = 5 OR c = 7", 1), ("c IN (1, 2) OR c = 8", 1),
                                          ("c BETWEEN 2 AND 3 OR c = 8", 2)])
def test_gpu_or_entries_scanned_in_filter(gpu_lib, where, scans):
    from pinot_amd.engine.segment import GpuSegment
    rng = np.random.default_rng(5)
    n = 50_000
    c = SegmentCreator("orstats")
    c.add_column("c", DataType.INT, rng.integers(0, 10, n))
    c.add_column("m", DataType.LONG, rng.integers(0, 1000, n))
    raw = c.build()
    seg = GpuSegment(raw)
    try:
        qc = parse(f"SELECT COUNT(*), SUM(m) FROM t WHERE {where}")
        op = GpuInstancePlanMaker().make_instance_plan(qc, [seg])
        blk = op.next_block()
        op.close()
        ob, ex = executor.execute(qc, [raw])
        assert blk.stats.num_docs_scanned == ob.stats.num_docs_scanned
        assert blk.results[0] == ob.results[0] and blk.results[1] == ex[1]
        assert blk.stats.num_entries_scanned_in_filter == scans * n
    finally:
        seg.destroy()
