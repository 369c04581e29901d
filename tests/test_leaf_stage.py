"""Multi-stage engine leaf stage on the host: results blocks -> row blocks in the stage's
schema (LeafStageTransferableBlockOperator.composeTransferableBlock / convertRow, TypeUtils.convert)."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine import leaf_stage as ls
from pinot_amd.query.sql import parse
from tests.test_filtered_aggregations import _segments


def test_type_utils_convert():
    assert ls.convert(3.9, ls.INT) == 3 and ls.convert(-3.9, ls.LONG) == -3
    assert ls.convert(2 ** 31, ls.INT) == -2 ** 31             # Long.intValue wraps
    assert ls.convert(1e12, ls.INT) == 2 ** 31 - 1             # Double.intValue saturates
    assert ls.convert(float("nan"), ls.LONG) == 0
    assert ls.convert(7, ls.DOUBLE) == 7.0 and isinstance(ls.convert(7, ls.DOUBLE), float)
    assert ls.convert(0.1, ls.FLOAT) == float(np.float32(0.1))
    assert ls.convert(12, ls.STRING) == "12"


def test_aggregation_leaf_rows():
    segs = _segments()
    q = parse("SELECT SUM(m), COUNT(*), MIN(a), AVG(b) FROM t WHERE a < 500")
    blk, _ = executor.execute(q, segs)
    sch = ls.block_schema(blk)
    assert sch.column_types == [ls.DOUBLE, ls.LONG, ls.DOUBLE, ls.OBJECT]
    tb = ls.compose_transferable_block(blk, sch)
    assert len(tb.rows) == 1 and tb.rows[0][1] == blk.results[1] and isinstance(tb.rows[0][0], float)
    # a stage that wants the count as INT and the sum as LONG gets converted values
    want = ls.DataSchema(sch.column_names, [ls.LONG, ls.INT, ls.DOUBLE, ls.OBJECT])
    tb2 = ls.compose_transferable_block(blk, want)
    assert tb2.rows[0][0] == int(blk.results[0]) and tb2.rows[0][1] == blk.results[1]


def test_group_by_leaf_rows():
    segs = _segments()
    q = parse("SELECT b, SUM(m), COUNT(*) FROM t GROUP BY b")
    blk, _ = executor.execute(q, segs)
    tb = ls.compose_transferable_block(blk, ls.block_schema(blk))
    assert len(tb.rows) == len(blk.groups)
    got = {r[0]: r[1:] for r in tb.rows}
    for k, v in blk.groups.items():
        assert got[k[0]] == [float(v[0]), int(v[1])]
    with pytest.raises(ValueError):
        ls.compose_transferable_block(blk, ls.DataSchema(["x"], [ls.INT]))
