"""Group-by keys and DISTINCTCOUNTHLL over raw (no-dictionary) columns on the GPU.

  group-by   NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator
             (DefaultGroupByExecutor.java:106-116): a raw INT / LONG column keys by its values; on the GPU the key
             dimension is value - min over the query's segments (value order = key order), mixed with dictionary
             columns' global ids, and a result's dictionary holds only the values its groups use. A raw FLOAT / DOUBLE
             column keys through the sorted distinct values over the segments (keys.hip, a doc-order id column); a raw
             STRING column through its distinct strings sorted bytewise (64-bit hashes sorted and verified on the device,
             the representatives' bytes merged on the host).
  HLL        DistinctCountHLLAggregationFunction over raw INT / LONG / FLOAT / DOUBLE values (:106-145): every matched
             doc's value hashed on the device (clearspring MurmurHash.hashLong, the dictionary path's mapping); raw
             STRING values by MurmurHash.hash of their UTF-8 bytes (seed -1, HyperLogLog.offer of a String).

Every block equals the oracle's (values read from the raw chunks: an independent route)."""
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


@pytest.fixture(scope="module")
def raw_segments(gpu_lib):
    """Three ragged segments; r* columns raw (no dictionary), d* dictionary-encoded; value ranges differ per segment
    (negative LONGs, a segment whose INT range sits inside another's)."""
    rng = np.random.default_rng(31)
    raws = []
    for s, n in enumerate((20_000, 33_333, 4097)):
        c = SegmentCreator(f"raw{s}", no_dictionary_columns=["ri", "rl", "rf", "rd", "rm", "rs", "rz"])
        c.add_column("ri", DataType.INT, rng.integers(-50 + 7 * s, 60 + 3 * s, n).astype(np.int32))
        c.add_column("rl", DataType.LONG, rng.integers(-3_000_000_000, -2_999_990_000, n) + 1_000_000 * s)
        # (+ 0.0: no -0.0 -- the reference keys it apart from 0.0 by its bits, Double2IntOpenHashMap, and so does the
        # GPU, but value-keyed Python dicts and the oracle's np.unique fold the two)
        c.add_column("rf", DataType.FLOAT, (np.round(rng.normal(0, 5, n), 1) + 0.0).astype(np.float32))
        c.add_column("rd", DataType.DOUBLE, np.round(rng.normal(0, 50, n), 2) + 0.0)
        c.add_column("rm", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        # -0.0 and 0.0 (and values around them): two keys by their bits on the device, in the oracle and in the
        # block's {key: intermediates} view (results.JavaDoubleKey)
        c.add_column("rz", DataType.DOUBLE, np.array([-0.0, 0.0, 0.5, -0.25, 3.0])[rng.integers(0, 5 - (s == 2), n)])
        c.add_column("dk", DataType.STRING, np.array([f"k{x}" for x in rng.integers(0, 9 + s, n)]))
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        # raw STRING: lengths 0-14 (every murmur tail), multi-byte UTF-8, values shared across segments or not
        words = ["", "a", "ab", "abc", "abcd", "zé", "ÿÿÿ", "日本語", "naïve-x", "k" * 13, "Z", "mid", "abcde"] + \
            [f"s{s}-{j}" for j in range(5 + 40 * s)]
        c.add_column("rs", DataType.STRING, np.array(words, dtype=object)[rng.integers(0, len(words), n)])
        raws.append(c.build())
    segs = _segs(raws)
    yield raws, segs
    for g in segs:
        g.destroy()


RAW_GROUP_BY = [
    "SELECT ri, COUNT(*), SUM(rm), MAX(rd) FROM t GROUP BY ri LIMIT 100000",
    "SELECT rl, COUNT(*), MIN(ri) FROM t WHERE f < 30 GROUP BY rl LIMIT 100000",
    "SELECT dk, ri, SUM(rm), DISTINCTCOUNTHLL(rl) FROM t WHERE f >= 10 GROUP BY dk, ri LIMIT 100000",
    "SELECT ri, dk, COUNT(*) FROM t GROUP BY ri, dk ORDER BY COUNT(*) DESC, ri, dk LIMIT 7",  # device trim
    "SELECT ri, SUM(rm) FROM t GROUP BY ri ORDER BY ri DESC LIMIT 5",  # key-order trim over raw values
    # raw FLOAT / DOUBLE keys (keys.hip: the sorted distinct values over the segments, a doc-order id column each)
    "SELECT rf, COUNT(*), SUM(rm) FROM t GROUP BY rf LIMIT 100000",
    "SELECT rd, dk, COUNT(*), MIN(ri), DISTINCTCOUNTHLL(rf) FROM t WHERE f < 50 GROUP BY rd, dk LIMIT 100000",
    "SELECT rf, rd, COUNT(*) FROM t WHERE f < 20 GROUP BY rf, rd ORDER BY rf DESC, rd LIMIT 9",  # key-order trim
    "SELECT rf, SUM(rd), MAX(rf) FROM t WHERE rf > 1.5 GROUP BY rf LIMIT 100000",  # key column also filtered / aggregated
    "SELECT rz, COUNT(*), SUM(rm) FROM t GROUP BY rz LIMIT 100000",  # -0.0 and 0.0: two groups
    "SELECT dk, rz, COUNT(*), MIN(rd) FROM t WHERE f < 70 GROUP BY dk, rz LIMIT 100000",
    # raw STRING keys (distinct strings over the segments sorted bytewise, a doc-order id column each)
    "SELECT rs, COUNT(*), SUM(rm) FROM t GROUP BY rs LIMIT 100000",
    "SELECT rs, dk, ri, COUNT(*), DISTINCTCOUNTHLL(rs) FROM t WHERE f < 50 GROUP BY rs, dk, ri LIMIT 100000",
    "SELECT rs, SUM(ri) FROM t WHERE f < 70 GROUP BY rs ORDER BY rs DESC LIMIT 6",  # key-order trim
    "SELECT rs, COUNT(*) FROM t WHERE rs >= 'abc' AND rs < 'zz' GROUP BY rs LIMIT 100000",  # raw STRING leaf too
]


@pytest.mark.parametrize("mode", ["auto", "hash"])
@pytest.mark.parametrize("sql", RAW_GROUP_BY)
def test_gpu_group_by_raw_columns(sql, mode, raw_segments, monkeypatch):
    monkeypatch.setenv("PHIP_GB_HASH", "1" if mode == "hash" else "0")
    raws, segs = raw_segments
    qc = parse(sql)
    qc.options["minServerGroupTrimSize"] = "3"  # (so the ORDER BY queries trim on the device)
    op = _gpu().make_instance_plan(qc, segs)
    gblk = op.next_block()
    op.close()
    oblk, exact = executor.execute(qc, raws)
    if getattr(gblk, "num_groups_trimmed", False):
        oblk = trim_groups(qc, oblk)
    _check(qc, gblk, oblk, exact)
    assert gblk.key_types == oblk.key_types
    if " rz," in sql:
        z = [e.name for e in qc.group_by].index("rz")
        zeros = {bool(np.signbit(k[z])) for k in gblk.groups if float(k[z]) == 0.0}
        assert zeros == {True, False}, "-0.0 and 0.0 must be two groups"
    got, want = reduce_blocks(qc, [gblk]).rows, reduce_blocks(qc, [oblk]).rows
    if not qc.order_by:  # (-0.0 before 0.0, as Double.compare orders them: Python's sort would tie the two)
        def order(r):
            return [(float(x), not np.signbit(x)) if isinstance(x, float) else x for x in r]
        got, want = sorted(got, key=order), sorted(want, key=order)
    assert fixtures.rows_match(got, want)


@pytest.mark.parametrize("limit", [1, 25])
def test_gpu_group_by_raw_num_groups_limit(limit, raw_segments):
    """numGroupsLimit over a raw key: per segment the first `limit` values in doc order (the no-dictionary
    generators' first-seen map, like the dictionary ones)."""
    raws, segs = raw_segments
    qc = parse("SELECT ri, COUNT(*), SUM(rm) FROM t GROUP BY ri LIMIT 100000")
    gblk = _gpu(num_groups_limit=limit).make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws, num_groups_limit=limit)
    assert oblk.num_groups_limit_reached
    _check(qc, gblk, oblk, exact)


RAW_HLL = [
    "SELECT DISTINCTCOUNTHLL(ri), DISTINCTCOUNTHLL(rl), DISTINCTCOUNTHLL(rf), DISTINCTCOUNTHLL(rd) FROM t",
    "SELECT DISTINCTCOUNTHLL(rm), COUNT(*) FROM t WHERE f < 40",
    "SELECT dk, DISTINCTCOUNTHLL(rd), DISTINCTCOUNTHLL(ri) FROM t GROUP BY dk LIMIT 100000",
    "SELECT DISTINCTCOUNTHLL(rl, 12), SUM(ri) FROM t WHERE f BETWEEN 20 AND 80",
    # over expressions: the transform's DOUBLE values offered as java.lang.Double (hashLong of the bits)
    "SELECT DISTINCTCOUNTHLL(ri * f), DISTINCTCOUNTHLL(rd - rf), COUNT(*) FROM t WHERE f < 60",
    "SELECT dk, DISTINCTCOUNTHLL(ri + f), SUM(rm) FROM t GROUP BY dk LIMIT 100000",
    # raw STRING values: MurmurHash.hash(bytes) on the device
    "SELECT DISTINCTCOUNTHLL(rs), DISTINCTCOUNTHLL(rs, 10), COUNT(*) FROM t WHERE f < 70",
    "SELECT dk, DISTINCTCOUNTHLL(rs, 6), SUM(ri) FROM t GROUP BY dk LIMIT 100000",
]


@pytest.mark.parametrize("sql", RAW_HLL)
def test_gpu_distinctcounthll_raw_columns(sql, raw_segments):
    """Registers bit-exact against the oracle's offers of the raw values (aggregation and group-by walks)."""
    raws, segs = raw_segments
    qc = parse(sql)
    gblk = _gpu().make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws)
    if qc.group_by:
        _check(qc, gblk, oblk, exact)
    else:
        from tests.test_gpu_parity import _assert_intermediates_equal
        _assert_intermediates_equal(qc.aggregations, gblk.results, oblk.results, exact)
    got, want = reduce_blocks(qc, [gblk]).rows, reduce_blocks(qc, [oblk]).rows
    if not qc.order_by:  # (no ORDER BY: the broker's rows come in table order; compare as sets)
        got, want = sorted(got), sorted(want)
    assert got == want


@pytest.mark.parametrize("how", ["collide", "exact"])
def test_gpu_raw_string_keys_hash_collisions(how, gpu_lib, monkeypatch):
    """Raw STRING group keys whose 64-bit device hashes collide take the exact host path (every doc's bytes keyed by
    themselves) instead of refusing the plan (round 5: PHIP_ERR_UNSUPPORTED). PHIP_STR_HASH_BITS=6 narrows the hash to
    64 values for ~300 distinct strings, so collisions occur inside and across segments; PHIP_STR_KEYS_EXACT=1 takes
    the exact path outright. Both equal the oracle."""
    if how == "collide":
        monkeypatch.setenv("PHIP_STR_HASH_BITS", "6")
    else:
        monkeypatch.setenv("PHIP_STR_KEYS_EXACT", "1")
    rng = np.random.default_rng(71 if how == "collide" else 72)
    raws = []
    for s in range(3):
        n = 9000 + 101 * s
        c = SegmentCreator(f"sc{how}{s}", no_dictionary_columns=["rs"])
        words = np.array([f"w{j}-{'x' * (j % 7)}" for j in range(80 * s, 80 * s + 150)] + ["", "zé", "日本"], dtype=object)
        c.add_column("rs", DataType.STRING, words[rng.integers(0, len(words), n)])
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 6, 10 ** 6, n))
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        raws.append(c.build())
    segs = _segs(raws)
    try:
        for sql in ("SELECT rs, COUNT(*), SUM(m) FROM t GROUP BY rs LIMIT 100000",
                    "SELECT rs, f, MAX(m) FROM t WHERE f < 20 GROUP BY rs, f LIMIT 100000"):
            qc = parse(sql)
            gblk = _gpu().make_instance_plan(qc, segs).next_block()
            oblk, exact = executor.execute(qc, raws)
            _check(qc, gblk, oblk, exact)
    finally:
        for g in segs:
            g.destroy()
