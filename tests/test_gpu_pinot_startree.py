"""GPU star-tree path over Pinot's OWN star-tree bytes (tests/golden/pinot_startree; test_pinot_startree.py pins
them against the raw rows): the parsed OffHeapStarTree and its documents are loaded beside the 313-row segment,
GpuStarTreeOperator answers from them, and every answer equals the oracle over the raw rows and the GPU scan path
(useStarTree=false); numDocsScanned is the number of star-tree documents the traversal matched."""
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.engine.startree import GpuStarTreeOperator
from pinot_amd.query.sql import parse
from tests.test_pinot_startree import QUERIES, star_segment
from tests.test_startree import _star_answer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pinot_star(gpu_lib):
    raw = star_segment()
    seg = GpuSegment(raw)
    yield raw, seg
    seg.destroy()


@pytest.mark.parametrize("sql", QUERIES)
def test_gpu_pinot_star_tree_equals_scan(sql, pinot_star):
    raw, seg = pinot_star
    qc = parse(sql)
    assert GpuStarTreeOperator.plan(qc, [seg], 100_000) is not None
    op = GpuInstancePlanMaker().make_instance_plan(qc, [seg])
    blk = op.next_block()
    op.close()
    assert getattr(blk, "star_tree", False)
    assert blk.stats.num_docs_scanned == _star_answer(qc, raw)[1]
    assert blk.stats.num_total_docs == 313
    want, _ = executor.execute(qc, [raw])
    if not qc.group_by:
        assert [float(x) for x in blk.results] == [float(x) for x in want.results]
    else:
        assert set(blk.groups) == set(want.groups)
        for k, v in want.groups.items():
            assert [float(x) for x in blk.groups[k]] == [float(x) for x in v], k
    exp = reduce_blocks(qc, [want]).rows
    assert reduce_blocks(qc, [blk]).rows == exp
    qc2 = parse(sql)
    qc2.options["useStarTree"] = "false"
    op2 = GpuInstancePlanMaker().make_instance_plan(qc2, [seg])
    blk2 = op2.next_block()
    op2.close()
    assert not getattr(blk2, "star_tree", False)
    assert reduce_blocks(qc2, [blk2]).rows == exp
