"""GROUP BY whose mixed-radix key space exceeds 2^62 on the GPU: tuple keys.

The reference switches DictionaryBasedGroupKeyGenerator from the int / long raw-key holders to a map over the key
tuple once the product of the columns' cardinalities leaves a long (LongMapBasedHolder / ArrayMapBasedHolder,
DictionaryBasedGroupKeyGenerator.java:150-185; the no-dictionary generators key by value tuples). Here each doc's
tuple of query-global key ids is packed into <= 4 u64 words, ranked per segment and across segments on the device
(keys.hip tuple_words_kernel / launch_tuple_rank), and the group-by runs over that one virtual key column; the result's
keys expand back to the query's columns. Three raw columns whose value ranges span ~3M each make a ~2^64 key space,
which the mixed radix refused before. PHIP_TUPLE_KEYS=1 forces the same path on small key spaces (null keys included).
Every block equals the oracle's."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.reduce import reduce_blocks, trim_groups
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures
from tests.test_gpu_limits import _check, _gpu, _segs

pytestmark = pytest.mark.gpu

SPAN = 3_000_000


@pytest.fixture(scope="module")
def tuple_segments(gpu_lib):
    rng = np.random.default_rng(57)
    raws = []
    pool_a = np.concatenate([[0, SPAN - 1], rng.integers(0, SPAN, 40)])
    pool_b = np.concatenate([[-SPAN, 0], rng.integers(-SPAN, 0, 30)])
    pool_c = np.concatenate([[7, SPAN + 6], rng.integers(7, SPAN + 7, 25)])
    for s, n in enumerate((20_000, 33_333, 4097)):
        c = SegmentCreator(f"tk{s}", no_dictionary_columns=["ra", "rb", "rc", "rd"])
        c.add_column("ra", DataType.LONG, rng.choice(pool_a, n))
        c.add_column("rb", DataType.LONG, rng.choice(pool_b, n))
        c.add_column("rc", DataType.INT, rng.choice(pool_c, n).astype(np.int32))
        c.add_column("rd", DataType.DOUBLE, np.round(rng.normal(0, 20, n), 2) + 0.0)
        c.add_column("s", DataType.STRING, np.array([f"v{x}" for x in rng.integers(0, 6 + s, n)]))
        c.add_column("g", DataType.INT, rng.integers(0, 5, n))
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        raws.append(c.build())
    segs = _segs(raws)
    yield raws, segs
    for g in segs:
        g.destroy()


TUPLE_QUERIES = [
    "SELECT ra, rb, rc, COUNT(*), SUM(f) FROM t GROUP BY ra, rb, rc LIMIT 1000000",
    "SELECT s, ra, rb, g, rc, SUM(rd), MAX(f), MIN(rd), DISTINCTCOUNTHLL(f) FROM t WHERE f < 50 "
    "GROUP BY s, ra, rb, g, rc LIMIT 1000000",
    "SELECT ra, rb, rc, SUM(f) FROM t GROUP BY ra, rb, rc ORDER BY SUM(f) DESC, ra, rb, rc LIMIT 10",  # agg trim
    "SELECT ra, rb, rc, COUNT(*) FROM t WHERE g <> 2 GROUP BY ra, rb, rc ORDER BY rc, ra DESC, rb LIMIT 12",
    "SELECT rb, s, rc, ra, AVG(f), COUNT(*) FROM t WHERE f BETWEEN 10 AND 30 GROUP BY rb, s, rc, ra LIMIT 1000000",
    "SELECT ra, rb, rc, COUNT(*) FROM t WHERE f = -1 GROUP BY ra, rb, rc LIMIT 10",  # nothing matches
]


def _run(qc, raws, segs, **kw):
    op = _gpu(**kw).make_instance_plan(qc, segs)
    gblk = op.next_block()
    op.close()
    oblk, exact = executor.execute(qc, raws, **{k: v for k, v in kw.items() if k == "num_groups_limit"})
    if getattr(gblk, "num_groups_trimmed", False):
        oblk = trim_groups(qc, oblk)
    return gblk, oblk, exact


@pytest.mark.parametrize("mode", ["auto", "hash"])
@pytest.mark.parametrize("sql", TUPLE_QUERIES)
def test_gpu_tuple_keys(sql, mode, tuple_segments, monkeypatch):
    monkeypatch.setenv("PHIP_GB_HASH", "1" if mode == "hash" else "0")
    raws, segs = tuple_segments
    qc = parse(sql)
    qc.options["minServerGroupTrimSize"] = "3"  # (the ORDER BY SUM query trims on the device)
    gblk, oblk, exact = _run(qc, raws, segs)
    _check(qc, gblk, oblk, exact)
    assert gblk.key_types == oblk.key_types
    got, want = reduce_blocks(qc, [gblk]).rows, reduce_blocks(qc, [oblk]).rows
    if not qc.order_by:
        got, want = sorted(got), sorted(want)
    assert fixtures.rows_match(got, want)


@pytest.mark.parametrize("limit", [1, 60])
def test_gpu_tuple_keys_num_groups_limit(limit, tuple_segments):
    """numGroupsLimit over tuple keys: per segment the first `limit` tuples in doc order."""
    raws, segs = tuple_segments
    qc = parse("SELECT ra, rb, rc, COUNT(*), SUM(f) FROM t GROUP BY ra, rb, rc LIMIT 1000000")
    gblk, oblk, exact = _run(qc, raws, segs, num_groups_limit=limit)
    assert oblk.num_groups_limit_reached
    _check(qc, gblk, oblk, exact)


FORCED = [
    "SELECT s, g, COUNT(*), SUM(rd) FROM t GROUP BY s, g LIMIT 100000",
    "SELECT g, rc, s, MAX(rd) FROM t WHERE f < 40 GROUP BY g, rc, s ORDER BY s DESC, g, rc LIMIT 9",
    "SELECT rd, s, COUNT(*) FROM t WHERE f < 10 GROUP BY rd, s LIMIT 100000",  # a raw DOUBLE key's ids in the tuple
]


@pytest.mark.parametrize("sql", FORCED)
def test_gpu_tuple_keys_forced(sql, tuple_segments, monkeypatch):
    """PHIP_TUPLE_KEYS=1: the tuple path on key spaces the mixed radix would take."""
    monkeypatch.setenv("PHIP_TUPLE_KEYS", "1")
    raws, segs = tuple_segments
    qc = parse(sql)
    gblk, oblk, exact = _run(qc, raws, segs)
    _check(qc, gblk, oblk, exact)
    got, want = reduce_blocks(qc, [gblk]).rows, reduce_blocks(qc, [oblk]).rows
    if not qc.order_by:
        got, want = sorted(got), sorted(want)
    assert fixtures.rows_match(got, want)

