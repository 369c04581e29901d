"""GPU leaf stage: GpuLeafStageOperator runs the leaf query on the GPU and returns the
row block + end-of-stream statistics; rows equal the oracle's block converted the same way."""
import pytest

from oracle import executor
from pinot_amd.engine import leaf_stage as ls
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.query.sql import parse
from tests.test_filtered_aggregations import _segments

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sql", [
    "SELECT SUM(m), COUNT(*), MAX(a) FROM t WHERE a BETWEEN 10 AND 800",
    "SELECT b, SUM(m), MIN(m), COUNT(*) FROM t WHERE a > 100 GROUP BY b",
    "SELECT b, SUM(m) FILTER(WHERE a < 300), COUNT(*) FROM t GROUP BY b",
])
def test_gpu_leaf_stage_rows(gpu_lib, sql):
    raws = _segments()
    segs = [GpuSegment(r) for r in raws]
    try:
        q = parse(sql)
        op = ls.GpuLeafStageOperator(q, segs)
        data = op.next_block()
        eos = op.next_block()
        assert not data.is_end_of_stream and eos.is_end_of_stream
        oblk, _ = executor.execute(q, raws)
        want = ls.compose_transferable_block(oblk, ls.block_schema(oblk))
        assert data.schema.column_types == want.schema.column_types
        assert sorted(map(repr, data.rows)) == sorted(map(repr, want.rows))
        assert eos.stats["numDocsScanned"] == oblk.stats.num_docs_scanned
        assert eos.stats["totalDocs"] == sum(r.num_docs for r in raws)
    finally:
        for s in segs:
            s.destroy()
