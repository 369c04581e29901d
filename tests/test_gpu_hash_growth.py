"""A full group-by hash table grows and the execution reruns on the device (runtime.cpp execute_growing; the reference's
holders grow with their maps, DictionaryBasedGroupKeyGenerator.java:150-185), where round 5 refused the query with
PHIP_ERR_UNSUPPORTED. The table is sized at plan creation to twice the groups possible, so the tests shrink it with
PHIP_GB_HASH_CAP (64 slots for thousands of groups): every execution doubles it until the groups fit, and the blocks
equal the oracle's -- plain, with a trim, and past numGroupsLimit (the first-seen limit pass over the grown table)."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.reduce import trim_groups
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests.test_gpu_limits import _check, _gpu, _segs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def segments(gpu_lib):
    rng = np.random.default_rng(57)
    raws = []
    for k in range(3):
        n = 40_000 + 313 * k
        c = SegmentCreator(f"hg{k}")
        c.add_column("a", DataType.INT, rng.integers(0, 90, n))
        c.add_column("b", DataType.INT, rng.integers(0, 70 + 5 * k, n))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 6, 10 ** 6, n))
        c.add_column("h", DataType.INT, rng.integers(0, 5000, n))
        raws.append(c.build())
    segs = _segs(raws)
    yield raws, segs
    for s in segs:
        s.destroy()


QUERIES = ["SELECT a, b, COUNT(*), SUM(m), MAX(m), DISTINCTCOUNTHLL(h) FROM t GROUP BY a, b LIMIT 100000",
           "SELECT a, b, SUM(m) FROM t WHERE h < 2500 GROUP BY a, b ORDER BY SUM(m) DESC LIMIT 10"]


@pytest.mark.parametrize("sql", QUERIES)
def test_gpu_hash_table_grows(sql, segments, monkeypatch):
    monkeypatch.setenv("PHIP_GB_HASH", "1")
    monkeypatch.setenv("PHIP_GB_HASH_CAP", "64")
    raws, segs = segments
    qc = parse(sql)
    qc.options["minServerGroupTrimSize"] = "5"
    op = _gpu().make_instance_plan(qc, segs)
    for _ in range(2):  # (the second execution starts from the grown table)
        gblk = op.next_block()
        oblk, exact = executor.execute(qc, raws)
        if getattr(gblk, "num_groups_trimmed", False):
            oblk = trim_groups(qc, oblk)
        _check(qc, gblk, oblk, exact)
    op.close()


def test_gpu_hash_table_grows_past_limit(segments, monkeypatch):
    monkeypatch.setenv("PHIP_GB_HASH", "1")
    monkeypatch.setenv("PHIP_GB_HASH_CAP", "64")
    raws, segs = segments
    qc = parse("SELECT a, b, COUNT(*), SUM(m) FROM t GROUP BY a, b LIMIT 100000")
    gblk = _gpu(num_groups_limit=1000).make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws, num_groups_limit=1000)
    assert oblk.num_groups_limit_reached
    _check(qc, gblk, oblk, exact)
