"""The id-histogram aggregation (agg_kernel kHist, runtime.cpp Plan::hist_mask): SUM / MIN / MAX of one INT / LONG
column with a small dictionary count the matched docs per dictionary id in per-wave LDS bins and fold count x value
into the accumulators when a segment ends, from the execution after one in which at least 30 % of the docs matched.
Every execution -- the first (value gathers) and the later ones (histogram) -- equals the CPU oracle: exact integer
sums, MIN / MAX, COUNT beside them, per-segment dictionaries that differ."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests.test_gpu_limits import _gpu, _segs
from tests.test_gpu_parity import _assert_intermediates_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def segments(gpu_lib):
    rng = np.random.default_rng(91)
    raws = []
    for k in range(5):
        n = 300_000 + 7_919 * k
        c = SegmentCreator(f"ah{k}")
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        c.add_column("m", DataType.LONG, rng.integers(-50_000, 50_000, 900 + 150 * k)[rng.integers(0, 900 + 150 * k, n)]
                     * (10 ** 9 if k % 2 else 1))
        c.add_column("i", DataType.INT, rng.integers(-1000, 1000, n))
        raws.append(c.build())
    segs = _segs(raws)
    yield raws, segs
    for s in segs:
        s.destroy()


QUERIES = ["SELECT SUM(m) FROM t WHERE f < 70",
           "SELECT SUM(m), COUNT(*) FROM t WHERE f >= 20",
           "SELECT MIN(m), MAX(m) FROM t WHERE f < 90",
           "SELECT SUM(i) FROM t",
           "SELECT MAX(i), COUNT(*) FROM t WHERE f < 5"]  # (sparse: stays on the value gathers)


@pytest.mark.parametrize("hist", ["default", "off"])
@pytest.mark.parametrize("sql", QUERIES, ids=[f"q{i}" for i in range(len(QUERIES))])
def test_gpu_agg_hist_vs_oracle(sql, hist, segments, monkeypatch):
    if hist == "off":
        monkeypatch.setenv("PHIP_AGG_HIST", "0")
    monkeypatch.setenv("PHIP_FUSE", "0")  # (the separate aggregation kernel, where the histogram lives)
    raws, segs = segments
    qc = parse(sql)
    oblk, exact = executor.execute(qc, raws)
    op = _gpu().make_instance_plan(qc, segs)
    for _ in range(3):
        gblk = op.next_block()
        assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
        _assert_intermediates_equal(qc.aggregations, gblk.results, oblk.results, exact)
    if hasattr(op, "close"):
        op.close()
