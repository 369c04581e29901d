"""Group-by records (runtime.cpp build_records, agg_kernel.h rec_load / group_chunk_rec / group_ring_batch_rec): the
fields a matched doc's group-by update reads -- key dictionary ids, packed values or value ids, 16-bit HLL entries --
packed into one record per doc, so the aggregation kernel reads one 16-byte record instead of one line per column.
The records only change where the bytes come from: every block equals the CPU oracle's (keys, exact sums, MIN / MAX,
HLL registers, docs), under both group-by walks, with the value columns materialized (packed values, doc-order HLL
entries) or kept as dictionary ids, and with a null-key segment beside record segments (that segment keeps its
columns' layouts: the kernel decides per segment). PHIP_GB_RECORD=1 builds a record for any number of fields."""
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
    rng = np.random.default_rng(71)
    raws = []
    for k in range(4):
        n = 50_000 + 977 * k
        c = SegmentCreator(f"gr{k}")
        c.add_column("y", DataType.INT, rng.integers(1992, 1999, n))
        c.add_column("g", DataType.STRING, np.array([f"n{x}" for x in rng.integers(0, 25, n)]))
        c.add_column("p", DataType.INT, rng.integers(0, 300 + 40 * k, n))
        c.add_column("rev", DataType.LONG, rng.integers(0, 6_000_000, n))  # wide: packed values when materialized
        c.add_column("cost", DataType.INT, rng.integers(0, 120_000, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.random(n) * 1000, 2))
        c.add_column("cust", DataType.INT, rng.integers(0, 200_000, n))
        # a nullable key column with nulls in segment 2 only: that segment has no record
        c.add_column("z", DataType.INT, rng.integers(0, 9, n), nulls=(rng.random(n) < 0.2) if k == 2 else None)
        raws.append(c.build())
    segs = _segs(raws)
    yield raws, segs
    for s in segs:
        s.destroy()


QUERIES = [
    "SELECT y, g, DISTINCTCOUNTHLL(cust), SUM(rev - cost) FROM t WHERE p < 150 GROUP BY y, g LIMIT 100000",
    "SELECT y, g, p, SUM(rev) FROM t WHERE cost > 30000 GROUP BY y, g, p LIMIT 100000",
    "SELECT g, COUNT(*), SUM(rev), MIN(d), MAX(cost), AVG(d) FROM t GROUP BY g LIMIT 100000",
    "SELECT y, SUM(rev * cost), MAX(d + cost), DISTINCTCOUNTHLL(cust, 10) FROM t WHERE d < 400 GROUP BY y LIMIT 100000",
    "SELECT y, g, SUM(rev) FROM t GROUP BY y, g ORDER BY SUM(rev) DESC LIMIT 5",
    "SET enableNullHandling = true; SELECT z, y, COUNT(*), SUM(rev) FROM t GROUP BY z, y LIMIT 100000",
]

SETTINGS = {
    "ids": {"PHIP_GB_RECORD": "1"},
    "materialized": {"PHIP_GB_RECORD": "1", "PHIP_MATERIALIZE_MIN_DICT": "0"},
    "materialized-batched": {"PHIP_GB_RECORD": "1", "PHIP_MATERIALIZE_MIN_DICT": "0", "PHIP_GB_BATCH": "1"},
    "materialized-one-chunk": {"PHIP_GB_RECORD": "1", "PHIP_MATERIALIZE_MIN_DICT": "0", "PHIP_GB_BATCH": "0"},
    "default": {},
}


@pytest.mark.parametrize("setting", list(SETTINGS))
@pytest.mark.parametrize("sql", QUERIES, ids=[f"q{i}" for i in range(len(QUERIES))])
def test_gpu_group_records_vs_oracle(sql, setting, segments, monkeypatch):
    for k, v in SETTINGS[setting].items():
        monkeypatch.setenv(k, v)
    raws, segs = segments
    qc = parse(sql)
    op = _gpu().make_instance_plan(qc, segs)
    for _ in range(2):  # (the second execution may take the other walk: Plan::walk_adaptive)
        gblk = op.next_block()
        oblk, exact = executor.execute(qc, raws)
        if getattr(gblk, "num_groups_trimmed", False):
            oblk = trim_groups(qc, oblk)
        _check(qc, gblk, oblk, exact)
    if hasattr(op, "close"):
        op.close()


def test_gpu_group_records_budget_zero(segments, monkeypatch):
    """A zero record budget (PHIP_GB_RECORD_GIB=0) builds no record: the columns' layouts, the same answers."""
    monkeypatch.setenv("PHIP_GB_RECORD", "1")
    monkeypatch.setenv("PHIP_GB_RECORD_GIB", "0")
    raws, segs = segments
    qc = parse("SELECT y, g, p, COUNT(*), SUM(cost) FROM t GROUP BY y, g, p LIMIT 100000")
    gblk = _gpu().make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws)
    _check(qc, gblk, oblk, exact)
