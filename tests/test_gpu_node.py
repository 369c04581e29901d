"""Node plans on the GPU (include/pinot_hip.h "node plans", pinot_amd/csrc/node.cpp): one prepared query over segments
on several devices of one process -- the sub-plans run concurrently, their dense partial tables meet on the root device
(an RCCL reduce over the node's communicator, or the peer merge kernel), and the record-shaped queries merge on the
host by key value (BaseCombineOperator.java:98-143 / GroupByCombineOperator.java:138-147 inside one server process).

The one-GPU box rehearses it with PHIP_NODE_SPLIT: k parts of the query's segments on the one device (two parts cannot
join one RCCL communicator, so the exchange is the peer merge: the non-root tables folded into the root's by
node_merge.hip), and k = 1, one part over a one-rank RCCL communicator (ncclCommInitAll + the grouped ncclReduce
calls, exactly as with eight devices). Every block equals the CPU oracle's over all segments and the single-device
plan's: groups, exact sums, MIN / MAX, HLL registers, numDocsScanned, per-segment matched docs."""
import numpy as np
import pytest

from oracle import executor
from pinot_amd import _lib
from pinot_amd.engine.plan import GpuCombineOperator, GpuInstancePlanMaker
from pinot_amd.engine.reduce import reduce_blocks, trim_groups
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures
from tests.test_gpu_parity import _assert_intermediates_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ssb_sf1(gpu_lib):
    """SSB SF1 in 3 segments (per-segment dictionaries): C5 and the C3 group-bys split over parts."""
    from tools import ssb
    names = ["Q2.1", "Q3.1", "Q4.3", "C5", "Q1.1"]
    raws = ssb.make_segments(1, ssb.columns_for(names), seed=11, segment_rows=2_000_000)
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


@pytest.fixture(scope="module")
def mixed(gpu_lib):
    """Five ragged segments: dictionary INT / LONG / STRING keys, a raw LONG key, nullable columns, doubles."""
    rng = np.random.default_rng(29)
    raws = []
    for k in range(5):
        n = 30_000 + 977 * k
        c = SegmentCreator(f"nd{k}", no_dictionary_columns=["r"])
        c.add_column("g", DataType.STRING, np.array([f"k{x}" for x in rng.integers(2 * k, 15 + 3 * k, n)]))
        c.add_column("h", DataType.INT, rng.integers(0, 40 + 10 * k, n))
        c.add_column("l", DataType.LONG, rng.integers(-30, 30, n) * 10 ** 10)
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.random(n) * 100, 3))
        c.add_column("r", DataType.LONG, rng.integers(0, 300, n))
        c.add_column("n", DataType.INT, rng.integers(0, 25, n), nulls=rng.random(n) < 0.2)
        c.add_column("x", DataType.LONG, rng.integers(0, 1000, n), nulls=rng.random(n) < 0.3)
        raws.append(c.build())
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


def _check(qc, gblk, raws, **kw):
    oblk, exact = executor.execute(qc, raws, **kw)
    assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert gblk.stats.num_segments_processed == oblk.stats.num_segments_processed
    assert gblk.stats.num_total_docs == oblk.stats.num_total_docs
    if not qc.group_by:
        _assert_intermediates_equal(qc.aggregations, gblk.results, oblk.results, exact)
        return
    if getattr(gblk, "num_groups_trimmed", False):
        oblk = trim_groups(qc, oblk)
    assert gblk.num_groups_limit_reached == oblk.num_groups_limit_reached
    assert set(gblk.groups) == set(oblk.groups)
    for k, v in oblk.groups.items():
        _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])


def _exchange(op, depth=0):
    """(parts, kind) of the first prepared GpuCombineOperator inside a plan-maker operator (the FILTER / null-handling
    / combine wrappers hold theirs as attributes)."""
    if isinstance(op, GpuCombineOperator) and getattr(op, "_plan", None):
        return op.exchange()
    if depth > 3:
        return None
    kids = []
    for v in getattr(op, "__dict__", {}).values():
        kids += list(v) if isinstance(v, (list, tuple)) else [v]
    for v in kids:
        if isinstance(v, (GpuCombineOperator,)) or hasattr(v, "__dict__") and type(v).__module__.startswith("pinot_amd"):
            r = _exchange(v, depth + 1)
            if r is not None:
                return r
    return None


def _run(sql, segs, monkeypatch, split, exchange=None, num_groups_limit=None):
    monkeypatch.setenv("PHIP_NODE_SPLIT", str(split))
    if exchange:
        monkeypatch.setenv("PHIP_NODE_EXCHANGE", exchange)
    qc = parse(sql)
    pm = GpuInstancePlanMaker() if num_groups_limit is None else GpuInstancePlanMaker(num_groups_limit=num_groups_limit)
    op = pm.make_instance_plan(qc, segs)
    blk = op.next_block()
    parts, kind = _exchange(op) or (None, None)
    if hasattr(op, "close"):
        op.close()
    return qc, blk, parts, kind


@pytest.mark.parametrize("split", [1, 3])
@pytest.mark.parametrize("name", ["C5", "Q2.1", "Q3.1", "Q4.3"])
def test_gpu_node_ssb_group_by(name, split, ssb_sf1, monkeypatch):
    """The SSB group-bys over a node plan: split 1 = one part over a one-rank RCCL communicator, split 3 = three parts
    on the one GPU merged by the peer kernel; groups, exact sums and HLL registers equal the oracle's and the
    single-device plan's, and every segment's matched docs are reported in query order."""
    from tools import ssb
    raws, segs = ssb_sf1
    qc, blk, parts, kind = _run(ssb.SSB_QUERIES[name], segs, monkeypatch, split)
    assert parts == split
    assert kind == (_lib.EXCHANGE_RCCL if split == 1 else _lib.EXCHANGE_PEER), kind
    _check(qc, blk, raws)
    monkeypatch.delenv("PHIP_NODE_SPLIT")
    single = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
    assert blk.segment_docs_matched == single.segment_docs_matched
    assert set(blk.groups) == set(single.groups)
    for k, v in single.groups.items():
        for a, b in zip(blk.groups[k], v):
            assert np.array_equal(np.asarray(a), np.asarray(b)), (k, a, b)


def test_gpu_node_ssb_aggregation(ssb_sf1, monkeypatch):
    """An aggregation-only query (one group): the parts' slots merged on the host, exact."""
    from tools import ssb
    raws, segs = ssb_sf1
    qc, blk, parts, kind = _run(ssb.SSB_QUERIES["Q1.1"], segs, monkeypatch, 3)
    assert parts == 3 and kind == _lib.EXCHANGE_RECORDS
    _check(qc, blk, raws)


MIXED = [
    # dense tables: the device exchange
    ("SELECT h, g, COUNT(*), SUM(m), MIN(d), MAX(m), DISTINCTCOUNTHLL(l) FROM t WHERE m > -500000000 GROUP BY h, g "
     "LIMIT 100000", "dense"),
    ("SELECT g, COUNT(*), DISTINCTCOUNTHLL(h, 8), DISTINCTCOUNTHLL(l, 10), AVG(d) FROM t GROUP BY g LIMIT 100000", "dense"),
    ("SELECT g, SUM(m) FROM t GROUP BY g ORDER BY SUM(m) DESC LIMIT 3", "dense"),  # trim after the merge, on the root
    ("SELECT h, COUNT(*) FILTER(WHERE d < 30), SUM(m) FILTER(WHERE g = 'k3'), COUNT(*) FROM t GROUP BY h "
     "LIMIT 100000", "dense"),
    # record-shaped: the host merge by key value
    ("SELECT r, COUNT(*), SUM(m), MAX(d) FROM t GROUP BY r LIMIT 100000", "records"),  # raw key
    ("SELECT COUNT(*), SUM(m), MIN(m), MAX(d), DISTINCTCOUNTHLL(g), MINMAXRANGE(l) FROM t WHERE h < 30", "records"),
    ("SET enableNullHandling = true; SELECT n, h, COUNT(*), SUM(x), MIN(x), COUNT(x) FROM t GROUP BY n, h "
     "LIMIT 100000", "any"),
]


@pytest.mark.parametrize("split", [2, 4])
@pytest.mark.parametrize("sql,path", MIXED, ids=[f"q{i}" for i in range(len(MIXED))])
def test_gpu_node_mixed(sql, path, split, mixed, monkeypatch):
    raws, segs = mixed
    qc, blk, parts, kind = _run(sql, segs, monkeypatch, split)
    assert parts == split, (parts, kind)
    if path == "dense":
        assert kind == _lib.EXCHANGE_PEER, kind
    elif path == "records":
        assert kind == _lib.EXCHANGE_RECORDS, kind
    _check(qc, blk, raws)
    if qc.group_by:
        got, want = reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [executor.execute(qc, raws)[0]]).rows
        if not qc.order_by:
            got, want = sorted(got, key=str), sorted(want, key=str)
        assert fixtures.rows_match(got, want)


@pytest.mark.parametrize("limit", [7, 50])
def test_gpu_node_num_groups_limit(limit, mixed, monkeypatch):
    """A device whose groups reach numGroupsLimit hands no partial table: the parts run to their records (each
    segment's first-seen groups) and merge on the host, as the reference's combine merges its segments' blocks."""
    raws, segs = mixed
    qc, blk, parts, kind = _run("SELECT h, COUNT(*), SUM(m) FROM t GROUP BY h LIMIT 100000", segs, monkeypatch, 3,
                                num_groups_limit=limit)
    assert blk.num_groups_limit_reached
    assert kind == _lib.EXCHANGE_RECORDS
    _check(qc, blk, raws, num_groups_limit=limit)


def test_gpu_node_rccl_refused_on_shared_device(mixed, monkeypatch):
    """PHIP_NODE_EXCHANGE=rccl with two parts on one device: RCCL cannot hold both, and the plan says so."""
    raws, segs = mixed
    with pytest.raises(_lib.PhipError):
        _run("SELECT h, COUNT(*) FROM t GROUP BY h LIMIT 100000", segs, monkeypatch, 2, exchange="rccl")


def test_gpu_node_repeated_executions(ssb_sf1, monkeypatch):
    """A prepared node plan executed again gives the same block (the parts' tables are reset between executions)."""
    from tools import ssb
    raws, segs = ssb_sf1
    monkeypatch.setenv("PHIP_NODE_SPLIT", "3")
    qc = parse(ssb.SSB_QUERIES["C5"])
    op = GpuCombineOperator(qc, segs, 100_000)
    first = op.next_block()
    for _ in range(3):
        again = op.next_block()
        assert set(again.groups) == set(first.groups)
        for k, v in first.groups.items():
            for a, b in zip(again.groups[k], v):
                assert np.array_equal(np.asarray(a), np.asarray(b))
    op.close()


HASHED = [MIXED[0][0], MIXED[1][0], MIXED[2][0], MIXED[3][0],
          "SELECT h, l, COUNT(*), SUM(d), MIN(m) FROM t WHERE d > 20 GROUP BY h, l LIMIT 100000"]


@pytest.mark.parametrize("split", [2, 4])
@pytest.mark.parametrize("sql", HASHED, ids=[f"h{i}" for i in range(len(HASHED))])
def test_gpu_node_hash_tables(sql, split, mixed, monkeypatch):
    """Hash-table group-bys (PHIP_GB_HASH=1 forces the open-addressing table, as a key space above 2^26 does): each part's
    table holds the same node-global keys in its own slots, so the exchange inserts the non-root parts' groups into the
    root's table by key (node_merge.hip hash_merge_*) and the root finishes it -- groups, sums, MIN / MAX, HLL registers
    and the trimmed ORDER BY equal the oracle's."""
    raws, segs = mixed
    monkeypatch.setenv("PHIP_GB_HASH", "1")
    qc, blk, parts, kind = _run(sql, segs, monkeypatch, split)
    assert parts == split and kind == _lib.EXCHANGE_HASH, (parts, kind)
    _check(qc, blk, raws)
    got, want = reduce_blocks(qc, [blk]).rows, reduce_blocks(qc, [executor.execute(qc, raws)[0]]).rows
    if not qc.order_by:
        got, want = sorted(got, key=str), sorted(want, key=str)
    assert fixtures.rows_match(got, want)


@pytest.mark.parametrize("name", ["C5", "Q3.1"])
def test_gpu_node_hash_ssb(name, ssb_sf1, monkeypatch):
    """SSB group-bys over three hash-table parts, executed three times (the tables are reset in between): the oracle's
    groups each time, and the single-device plan's blocks bit for bit."""
    from tools import ssb
    raws, segs = ssb_sf1
    monkeypatch.setenv("PHIP_GB_HASH", "1")
    monkeypatch.setenv("PHIP_NODE_SPLIT", "3")
    qc = parse(ssb.SSB_QUERIES[name])
    op = GpuCombineOperator(qc, segs, 100_000)
    blocks = [op.next_block() for _ in range(3)]
    assert op.exchange() == (3, _lib.EXCHANGE_HASH)
    op.close()
    _check(qc, blocks[0], raws)
    for b in blocks[1:]:
        assert set(b.groups) == set(blocks[0].groups)
        for k, v in blocks[0].groups.items():
            for a, c in zip(b.groups[k], v):
                assert np.array_equal(np.asarray(a), np.asarray(c)), (k, a, c)


def test_gpu_node_hash_full_falls_back(mixed, monkeypatch):
    """A part whose hash table is too small for its groups (PHIP_GB_HASH_CAP) hands no partial: the parts run to their
    records (each growing its table) and merge on the host."""
    raws, segs = mixed
    monkeypatch.setenv("PHIP_GB_HASH", "1")
    monkeypatch.setenv("PHIP_GB_HASH_CAP", "64")
    qc, blk, parts, kind = _run("SELECT h, g, COUNT(*), SUM(m) FROM t GROUP BY h, g LIMIT 100000", segs, monkeypatch, 2)
    assert kind == _lib.EXCHANGE_RECORDS
    _check(qc, blk, raws)


@pytest.mark.parametrize("split", [2, 3])
@pytest.mark.parametrize("sql", [MIXED[0][0], MIXED[1][0], MIXED[3][0]], ids=["r0", "r1", "r3"])
def test_gpu_node_with_group_records(sql, split, mixed, monkeypatch):
    """Node parts whose aggregation walks read group-by records (PHIP_GB_RECORD=1, values materialized): the dense
    partial tables still merge on the devices and equal the oracle."""
    raws, segs = mixed
    monkeypatch.setenv("PHIP_GB_RECORD", "1")
    monkeypatch.setenv("PHIP_MATERIALIZE_MIN_DICT", "0")
    qc, blk, parts, kind = _run(sql, segs, monkeypatch, split)
    assert parts == split and kind == _lib.EXCHANGE_PEER, (parts, kind)
    _check(qc, blk, raws)
