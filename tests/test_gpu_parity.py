"""GPU parity: libpinot_hip.so vs the reference's known answers and vs the CPU oracle.

Bar (north_star): bit-exact doc-id sets, counts, INT/LONG sums, group keys and HLL registers;
<= 1e-9 relative for DOUBLE sums.
"""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker
from pinot_amd.engine.reduce import broker_response, reduce_blocks
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType
from tests import fixtures

pytestmark = pytest.mark.gpu
CASES = fixtures.expected()["queries"]
REL = 1e-9  # DOUBLE-sum tolerance stated by north_star


@pytest.fixture(scope="module")
def gsegs(gpu_lib):
    out = {name: GpuSegment(fixtures.segment_for(name)) for name in ("test_data_sv", "fast_filtered_count")}
    yield out
    for s in out.values():
        s.destroy()


def _words_from_mask(mask):
    n = len(mask)
    pad = np.zeros(((n + 63) // 64) * 64, dtype=np.uint8)
    pad[:n] = mask
    return np.packbits(pad.reshape(-1, 64)[:, ::-1], axis=1).view(">u8").reshape(-1).astype(np.uint64)


def _assert_intermediates_equal(aggs, gpu_vals, ora_vals, ora_exact):
    for ag, g, o, ex in zip(aggs, gpu_vals, ora_vals, ora_exact):
        f = ag.function
        if f in ("distinctcounthll", "distinctcountrawhll"):
            assert np.array_equal(np.asarray(g), np.asarray(o)), "HLL registers differ"
        elif f == "count":
            assert g == o
        elif f == "sum":
            if ex is not None and isinstance(g, int):
                assert g == ex, (g, ex)  # exact int64
                if abs(ex) < 2 ** 53:
                    assert float(g) == o
            elif ex is not None:
                # integer inputs whose |sum| bound passed 2^58: the library summed in double, as
                # SumAggregationFunction does -- within REL of both the exact sum and the reference's fold
                assert isinstance(g, float), g
                assert abs(g - ex) <= REL * max(abs(ex), 1.0), (g, ex)
                assert g == o or abs(g - o) <= REL * max(abs(g), abs(o)), (g, o)
            else:
                assert g == o or abs(g - o) <= REL * max(abs(g), abs(o))
        elif f in ("min", "max"):
            assert g == o
        elif f == "avg":
            assert g[1] == o[1]
            assert float(g[0]) == o[0] or abs(g[0] - o[0]) <= REL * abs(o[0])
        elif f == "minmaxrange":
            assert tuple(map(float, g)) == tuple(o)


@pytest.mark.parametrize("case", CASES, ids=[f"{c['ref'].split('/')[-1]}|{c['query'][:60]}" for c in CASES])
def test_gpu_known_answers(case, gsegs):
    seg = gsegs[case["data"]]
    pm = GpuInstancePlanMaker()
    if case["data"] == "test_data_sv":
        rt = broker_response(pm, case["query"], [seg, seg])
        docs, post, total = case["stats"]
        assert rt.stats.num_docs_scanned == docs
        assert rt.stats.num_entries_scanned_post_filter == post
        assert rt.stats.num_total_docs == total
    else:
        qc = parse(case["query"])
        rt = reduce_blocks(qc, [pm.make_instance_plan(qc, [seg]).next_block()])
    assert fixtures.rows_match(rt.rows, case["rows"]), (rt.rows, case["rows"])


@pytest.mark.parametrize("case", CASES, ids=[f"{c['ref'].split('/')[-1]}|{c['query'][:60]}" for c in CASES])
def test_gpu_intermediates_vs_oracle(case, gsegs):
    seg = gsegs[case["data"]]
    qc = parse(case["query"])
    op = GpuInstancePlanMaker().make_instance_plan(qc, [seg, seg])
    gblk = op.next_block()
    oblk, exact = executor.execute(qc, [seg.segment, seg.segment])
    assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    if not qc.group_by:
        _assert_intermediates_equal(qc.aggregations, gblk.results, oblk.results, exact)
    else:
        assert set(gblk.groups) == set(oblk.groups)
        for k, v in oblk.groups.items():
            _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])


FILTERS = [
    "column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000 AND column5 = 'gFuH'"
    " AND (column6 < 500000000 OR column11 NOT IN ('t', 'P')) AND daysSinceEpoch = 126164076",
    "column11 IN ('t', 'P')",
    "NOT column11 IN ('t', 'P')",
    "column6 <> 296467636 OR column9 < 50000",
    "column7 IN (675695, 2147483647) AND NOT (column17 = 83386499 OR column18 >= 1000)",
    "column12 BETWEEN 'H' AND 'p' AND daysSinceEpoch <> 126164076",
    "column1 < 0",
    "column9 IN (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20) OR column3 > 2000000000",
]


@pytest.mark.parametrize("flt", FILTERS)
def test_gpu_filter_bitmap_bit_exact(flt, gsegs):
    seg = gsegs["test_data_sv"]
    qc = parse("SELECT COUNT(*) FROM testTable WHERE " + flt)
    words = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).filter_bitmap()
    expect = _words_from_mask(executor.filter_mask(qc, seg.segment))
    assert np.array_equal(words, expect)


@pytest.mark.parametrize("case", fixtures.expected()["docsets"], ids=lambda c: c["ref"].split("/")[-1])
@pytest.mark.parametrize("prefix", ["s", "t"])
def test_gpu_docset_kats(case, prefix, gpu_lib):
    seg = GpuSegment(fixtures.docset_segment(case["sets"], case["num_docs"]))
    try:
        qc = parse("SELECT COUNT(*) FROM t WHERE " + fixtures.docset_filter(case["op"], len(case["sets"]), prefix))
        words = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).filter_bitmap()
        docs = [i for i in range(case["num_docs"]) if (int(words[i // 64]) >> (i % 64)) & 1]
        assert docs == case["expected"]
    finally:
        seg.destroy()


# ---- property tests mirroring FixedBitIntReaderTest / FixedBitSVForwardIndexReaderV2Test ----------
@pytest.mark.parametrize("bits", list(range(1, 32)))
def test_gpu_scan_all_widths(bits, gpu_lib):
    rng = np.random.default_rng(bits)
    for n in (1, 95, 4097, 99_999):
        card = min(2 ** bits, n + 1)
        # dictionary values 0..card-1 with the width's max id present so getNumBitsPerValue == bits
        vals = rng.integers(0, card, n).astype(np.int64)
        vals[rng.integers(0, n)] = 2 ** bits - 1 if card == 2 ** bits else card - 1
        c = SegmentCreator("w").add_column("x", DataType.LONG, vals * 3 + 7)
        raw = c.build()
        if raw.columns["x"].metadata.bits_per_element != bits:
            continue
        seg = GpuSegment(raw)
        try:
            d = np.unique(vals * 3 + 7)
            lo, hi = d[len(d) // 4], d[(3 * len(d)) // 4]
            for flt in (f"x BETWEEN {lo} AND {hi}", f"x <> {d[0]}", f"x IN ({d[0]}, {d[-1]}, {hi})"):
                qc = parse(f"SELECT COUNT(*), SUM(x), MIN(x), MAX(x) FROM t WHERE {flt}")
                op = GpuInstancePlanMaker().make_instance_plan(qc, [seg])
                words = op.filter_bitmap()
                mask = executor.filter_mask(qc, raw)
                assert np.array_equal(words, _words_from_mask(mask)), (bits, n, flt)
                blk = op.next_block()
                oblk, ex = executor.execute(qc, [raw])
                _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
        finally:
            seg.destroy()


def _roaring_segment(n, rng):
    # values chosen so the inverted index holds array, bitmap and run containers
    v = np.zeros(n, dtype=np.int32)
    v[rng.random(n) < 0.5] = 1                    # dense -> bitmap containers
    v[rng.random(n) < 0.001] = 2                  # sparse -> array containers
    for s in range(0, n, 70_000):                 # long runs -> run containers
        v[s:s + 5000] = 3
    v[-1] = 4
    c = SegmentCreator("roar", inverted_index_columns=["v"])
    c.add_column("v", DataType.INT, v)
    c.add_column("w", DataType.INT, rng.integers(0, 1000, n))
    return c.build()


def test_gpu_roaring_all_container_kinds(gpu_lib):
    rng = np.random.default_rng(7)
    raw = _roaring_segment(300_001, rng)
    seg = GpuSegment(raw)
    try:
        for flt in ("v = 1", "v = 2", "v = 3", "v IN (2, 3)", "v NOT IN (1, 4)", "v <> 3 AND w < 500",
                    "v = 4 OR (v = 2 AND w > 10)"):
            qc = parse(f"SELECT COUNT(*), SUM(w) FROM t WHERE {flt}")
            op = GpuInstancePlanMaker().make_instance_plan(qc, [seg])
            assert np.array_equal(op.filter_bitmap(), _words_from_mask(executor.filter_mask(qc, raw))), flt
    finally:
        seg.destroy()


def test_gpu_group_by_across_segment_dictionaries(gpu_lib):
    """Per-segment dictionaries differ: keys merge by value through the query-global dictionary."""
    rng = np.random.default_rng(3)
    raws = []
    for k in range(3):
        n = 20_000 + 1000 * k
        c = SegmentCreator(f"s{k}")
        c.add_column("g", DataType.STRING, np.array([f"k{x}" for x in rng.integers(k, 40 + 5 * k, n)]))
        c.add_column("h", DataType.INT, rng.integers(0, 7 + k, n))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 12, 10 ** 12, n))
        c.add_column("d", DataType.DOUBLE, rng.random(n) * 1000)
        raws.append(c.build())
    segs = [GpuSegment(r) for r in raws]
    try:
        qc = parse("SELECT g, h, COUNT(*), SUM(m), SUM(d), MIN(d), MAX(m), DISTINCTCOUNTHLL(m) FROM t "
                   "WHERE h <> 3 GROUP BY g, h ORDER BY g, h LIMIT 100000")
        gblk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
        oblk, exact = executor.execute(qc, raws)
        assert set(gblk.groups) == set(oblk.groups)
        for k, v in oblk.groups.items():
            _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])
    finally:
        for s in segs:
            s.destroy()


def test_gpu_raw_long_metric(gpu_lib):
    """BenchmarkQueries-style raw (no-dictionary) LONG metric, PASS_THROUGH chunks (v2 and v3)."""
    rng = np.random.default_rng(5)
    n = 123_457
    c = SegmentCreator("raw", no_dictionary_columns=["RAW_LONG"])
    c.add_column("INT_COL", DataType.INT, rng.integers(0, 5000, n))
    c.add_column("RAW_LONG", DataType.LONG, rng.integers(-2 ** 40, 2 ** 40, n))
    raw = c.build()
    seg = GpuSegment(raw)
    try:
        for q in ("SELECT SUM(RAW_LONG) FROM t",
                  "SELECT SUM(RAW_LONG), COUNT(*), MAX(RAW_LONG) FROM t WHERE INT_COL > 5 AND INT_COL < 1499"):
            qc = parse(q)
            blk = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).next_block()
            oblk, ex = executor.execute(qc, [raw])
            _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
    finally:
        seg.destroy()


def test_gpu_empty_result_and_tiny_segment(gpu_lib):
    c = SegmentCreator("one").add_column("a", DataType.INT, [42])
    raw = c.build()
    seg = GpuSegment(raw)
    try:
        for q in ("SELECT COUNT(*), SUM(a), MIN(a), MAX(a) FROM t WHERE a = 42",
                  "SELECT COUNT(*), SUM(a), MIN(a), MAX(a) FROM t WHERE a <> 42",
                  "SELECT a, COUNT(*) FROM t WHERE a = 42 GROUP BY a"):
            qc = parse(q)
            blk = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).next_block()
            oblk, ex = executor.execute(qc, [raw])
            if qc.group_by:
                assert set(blk.groups) == set(oblk.groups)
            else:
                _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
    finally:
        seg.destroy()


# ---- conjunctive fast path: mixed widths (P-layout windows of 1/2/4/8 docs), wide dictionaries -------
@pytest.fixture(scope="module")
def wide_segment(gpu_lib):
    """600,003 docs; column wN has exactly N bits per value (card in (2^(N-1), 2^N])."""
    rng = np.random.default_rng(20)
    n = 600_003
    c = SegmentCreator("wide")
    for b in list(range(1, 10)) + [12, 16, 19, 20]:
        card = min(n, (1 << (b - 1)) + 1 + int(rng.integers(0, 1 << (b - 1))))
        v = rng.integers(0, card, n)
        v[:card] = np.arange(card)  # every dictionary value present
        rng.shuffle(v)
        c.add_column(f"w{b}", DataType.INT, v * 7 - 3)
    raw = c.build()
    for b in list(range(1, 10)) + [12, 16, 19, 20]:
        assert raw.columns[f"w{b}"].metadata.bits_per_element == b
    seg = GpuSegment(raw)
    yield raw, seg
    seg.destroy()


CONJ_CASES = [(1, 2, 3), (3, 4, 6), (4, 5, 7), (2, 9, 12), (3, 19, 5), (8, 8), (16, 2), (20, 1), (6, 7, 8, 9),
              (1, 2, 3, 4, 5, 6)]


@pytest.mark.parametrize("widths", CONJ_CASES, ids=lambda w: "w" + "_".join(map(str, w)))
def test_gpu_conjunction_mixed_widths(widths, wide_segment):
    raw, seg = wide_segment
    rng = np.random.default_rng(sum(widths))
    preds = []
    for i, b in enumerate(widths):
        card = raw.columns[f"w{b}"].metadata.cardinality
        if b <= 6 and i % 2 == 1:  # a small-set (card <= 64) leaf
            ids = sorted(set(rng.integers(0, card, 1 + card // 2).tolist()))
            preds.append(f"w{b} IN ({', '.join(str(x * 7 - 3) for x in ids)})")
        else:
            lo = int(rng.integers(0, card))
            hi = int(rng.integers(lo, card))
            span = max(1, card // (2 if i == 0 else 1))
            hi = min(card - 1, max(hi, lo + span // 2))
            preds.append(f"w{b} BETWEEN {lo * 7 - 3} AND {hi * 7 - 3}")
    qc = parse(f"SELECT COUNT(*), SUM(w{widths[0]}) FROM t WHERE " + " AND ".join(preds))
    op = GpuInstancePlanMaker().make_instance_plan(qc, [seg])
    expect = executor.filter_mask(qc, raw)
    assert np.array_equal(op.filter_bitmap(), _words_from_mask(expect)), preds
    blk = op.next_block()
    oblk, ex = executor.execute(qc, [raw])
    _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)


# ---- SSB queries (flattened lineorder, tools/ssbgen.c) vs the oracle: 3 segments, per-segment dicts ---
SSB_NAMES = ["Q1.1", "Q1.2", "Q1.3", "Q2.1", "Q2.2", "Q2.3", "Q3.1", "Q3.2", "Q3.3", "Q3.4", "Q4.1", "Q4.2", "Q4.3", "C5"]


@pytest.fixture(scope="module", params=["unsorted", "sorted"])
def ssb_segments(gpu_lib, request):
    """SF1 in 3 segments; 'sorted' = rows ordered by LO_ORDERDATE, so the date columns
    carry sorted forward indexes and their predicates become SortedIndexBasedFilterOperator doc ranges."""
    from tools import ssb
    cols = ssb.columns_for(SSB_NAMES)
    raws = ssb.make_segments(1, cols, seed=7, segment_rows=2_000_000, layout=request.param)
    if request.param == "sorted":
        assert all(r.columns["D_YEAR"].metadata.is_sorted for r in raws)
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


@pytest.mark.parametrize("name", SSB_NAMES)
def test_gpu_ssb_vs_oracle(name, ssb_segments):
    from tools import ssb
    raws, segs = ssb_segments
    qc = parse(ssb.SSB_QUERIES[name])
    gblk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws)
    assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    if not qc.group_by:
        _assert_intermediates_equal(qc.aggregations, gblk.results, oblk.results, exact)
    else:
        assert set(gblk.groups) == set(oblk.groups)
        for k, v in oblk.groups.items():
            _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])


# ---- fused group-by (filter_kernel.h fused_defer_gb): the filter kernel runs the dense HBM-table walk ------
GB_SSB = [n for n in SSB_NAMES if not n.startswith("Q1")]


@pytest.mark.parametrize("mode", ["2", "3", "4"], ids=["hbm_table", "xcd_copies", "lds_table"])
@pytest.mark.parametrize("name", GB_SSB)
def test_gpu_ssb_fused_group_by(name, mode, ssb_segments, monkeypatch):
    """PHIP_FUSED_GB=2 fuses every dense group-by into one HBM table (the LDS-sized tables too), =3 into XCD-private
    copies merged after the launch (tables up to PHIP_FUSED_GB_XCD_MAX), =4 the LDS-sized tables into each workgroup's
    LDS table (slabs reduced after the launch; other tables keep the two launches): the same groups, sums and HLL
    registers as the oracle, and the one launch reports itself fused. (Over the sorted layout a segment whose date
    predicate is an OR of two doc ranges takes the general filter program, which does not fuse.)"""
    from tools import ssb
    monkeypatch.setenv("PHIP_FUSED_GB", mode)
    raws, segs = ssb_segments
    qc = parse(ssb.SSB_QUERIES[name])
    gblk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
    if not raws[0].columns["D_YEAR"].metadata.is_sorted and mode != "4":
        assert gblk.fused
    if gblk.fused:
        assert gblk.agg_kernel_ms == 0.0
    oblk, exact = executor.execute(qc, raws)
    assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    assert set(gblk.groups) == set(oblk.groups)
    for k, v in oblk.groups.items():
        _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])


@pytest.mark.parametrize("limit", [10 ** 9, 5000], ids=["no_limit", "limit_reached"])
def test_gpu_fused_group_by_limit_pass(limit, gpu_lib):
    """A 240K-key dense space (HBM table: fused by default) over 3 segments with different dictionaries. With
    numGroupsLimit 5000 the limit pass runs, which first has the plain filter write the tile masks the fused launch
    never produced; both ways every group equals the oracle's."""
    rng = np.random.default_rng(43)
    raws = []
    for k in range(3):
        n = 120_000 + 511 * k
        c = SegmentCreator(f"fl{k}")
        c.add_column("a", DataType.INT, rng.integers(0, 600, n))
        c.add_column("b", DataType.LONG, rng.integers(0, 400, n) * 5 + 1)
        c.add_column("f", DataType.INT, rng.integers(0, 100, n))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
        raws.append(c.build())
    segs = [GpuSegment(r) for r in raws]
    try:
        qc = parse("SELECT a, b, COUNT(*), SUM(m), MAX(m) FROM t WHERE f < 70 AND a >= 3 GROUP BY a, b LIMIT 10000000")
        gblk = GpuInstancePlanMaker(num_groups_limit=limit).make_instance_plan(qc, segs).next_block()
        oblk, exact = executor.execute(qc, raws, num_groups_limit=limit)
        assert gblk.fused
        assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
        assert gblk.num_groups_limit_reached == oblk.num_groups_limit_reached == (limit == 5000)
        assert set(gblk.groups) == set(oblk.groups)
        for k, v in oblk.groups.items():
            _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])
    finally:
        for s in segs:
            s.destroy()


# ---- dense tiles: batched lane-major aggregation walk vs per-64-doc chunks vs the oracle ------------
DENSE_QUERIES = [
    "SELECT COUNT(*), SUM(a), SUM(r), SUM(d), MIN(d), MAX(a), MIN(r), DISTINCTCOUNTHLL(a) FROM t",
    "SELECT COUNT(*), SUM(a), SUM(r), SUM(d), MIN(d), MAX(a), DISTINCTCOUNTHLL(a) FROM t WHERE f < 90",
    "SELECT SUM(a * d), SUM(a - r), SUM(a + a), MAX(d), COUNT(*) FROM t WHERE f >= 40",
    "SELECT SUM(a), COUNT(*), MIN(a) FROM t WHERE f < 33",
    "SELECT SUM(r), MAX(r) FROM t WHERE f BETWEEN 10 AND 99",
    "SELECT SUM(s), SUM(sl), SUM(sd), MIN(sd), MAX(sl), SUM(s * sd), SUM(sl - s), COUNT(*) FROM t WHERE f < 80",
    "SELECT SUM(s), SUM(sl * s), MAX(s), DISTINCTCOUNTHLL(s), SUM(a) FROM t",
]


@pytest.mark.parametrize("walk", ["chunks", "batch", "staged", "staged_lds_dict"])
@pytest.mark.parametrize("q", DENSE_QUERIES)
def test_gpu_dense_tile_batches(q, walk, monkeypatch, gpu_lib):
    """Tiles with >= kDenseMin matched docs take agg_batch (aggregate.hip) when PHIP_DENSE_BATCH allows,
    with the dict-id words LDS-staged unless PHIP_AGG_STAGE=0; every walk must give the oracle's answers
    (ragged last tile, raw INT, dict INT / DOUBLE, HLL)."""
    monkeypatch.setenv("PHIP_DENSE_BATCH", "0" if walk == "chunks" else "1")
    monkeypatch.setenv("PHIP_AGG_STAGE", "1" if walk.startswith("staged") else "0")
    monkeypatch.setenv("PHIP_AGG_LDS_DICT", "1" if walk == "staged_lds_dict" else "0")
    rng = np.random.default_rng(31)
    n = 2048 * 37 + 1234
    c = SegmentCreator("dense", no_dictionary_columns=["r"])
    c.add_column("a", DataType.INT, rng.integers(-3000, 5000, n))
    c.add_column("d", DataType.DOUBLE, np.round(rng.normal(0, 1e4, n), 2))
    c.add_column("r", DataType.INT, rng.integers(-2 ** 31, 2 ** 31 - 1, n))
    c.add_column("f", DataType.INT, rng.integers(0, 100, n))
    c.add_column("s", DataType.INT, rng.integers(-50, 50, n))                  # 400-B dictionary
    c.add_column("sl", DataType.LONG, rng.integers(0, 60, n) * 10 ** 12)       # 480-B dictionary
    c.add_column("sd", DataType.DOUBLE, rng.integers(0, 50, n) * 0.37 - 3.5)  # 400-B dictionary
    raw = c.build()
    seg = GpuSegment(raw)
    try:
        qc = parse(q)
        blk = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).next_block()
        oblk, ex = executor.execute(qc, [raw])
        assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
        _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
    finally:
        seg.destroy()


# ---- high-cardinality group-by: open-addressing hash table in HBM (GB_HASH) -------------------------
GB_CASES = [c for c in CASES if "group by" in c["query"].lower()]


@pytest.mark.parametrize("case", GB_CASES, ids=[f"{c['ref'].split('/')[-1]}|{c['query'][:60]}" for c in GB_CASES])
def test_gpu_group_by_hash_table_known_answers(case, gsegs, monkeypatch):
    """PHIP_GB_HASH=1 forces the hash table for small key spaces too: same known answers."""
    monkeypatch.setenv("PHIP_GB_HASH", "1")
    test_gpu_known_answers(case, gsegs)
    test_gpu_intermediates_vs_oracle(case, gsegs)


@pytest.mark.parametrize("limit", [None, 10 ** 9], ids=["default_limit", "no_limit"])
def test_gpu_group_by_high_cardinality(gpu_lib, limit):
    """Key space 30011 x 20011 x 7 (> 2^26) over 3 segments with different dictionaries -> GB_HASH
    without any override; every group and intermediate equals the oracle's. With the default
    numGroupsLimit (100,000) every segment holds more distinct keys than the limit: the first-seen
    100,000 per segment are kept (limit.hip), as the oracle's IntGroupIdMap restatement does."""
    rng = np.random.default_rng(41)
    raws = []
    for k in range(3):
        n = 150_000 + 777 * k
        c = SegmentCreator(f"hc{k}")
        c.add_column("a", DataType.INT, rng.integers(0, 30011, n))
        c.add_column("b", DataType.LONG, rng.integers(0, 20011, n) * 3 - 7)
        c.add_column("s", DataType.STRING, np.array([f"v{x}" for x in rng.integers(0, 7, n)]))
        c.add_column("m", DataType.LONG, rng.integers(-10 ** 12, 10 ** 12, n))
        c.add_column("d", DataType.DOUBLE, np.round(rng.random(n) * 1000, 3))
        raws.append(c.build())
    segs = [GpuSegment(r) for r in raws]
    try:
        qc = parse("SELECT a, b, s, COUNT(*), SUM(m), SUM(d), MIN(d), MAX(m), DISTINCTCOUNTHLL(m) FROM t "
                   "WHERE a < 25000 GROUP BY a, b, s LIMIT 10000000")
        kw = {} if limit is None else {"num_groups_limit": limit}
        gblk = GpuInstancePlanMaker(**kw).make_instance_plan(qc, segs).next_block()
        oblk, exact = executor.execute(qc, raws, **kw)
        assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
        assert gblk.num_groups_limit_reached == oblk.num_groups_limit_reached == (limit is None)
        assert set(gblk.groups) == set(oblk.groups)
        for k, v in oblk.groups.items():
            _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])
    finally:
        for s in segs:
            s.destroy()


# ---- config C1: BenchmarkQueries-style segments (tools/bq.py), every query of the GPU subset ----------
@pytest.fixture(scope="module")
def bq_segments(gpu_lib):
    from tools import bq
    raws = bq.make_segments(250_000, num_segments=2, scenario="EXP(0.001)")
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


def _check_vs_oracle(qc, raws, segs):
    """Default numGroupsLimit on both sides (first-seen keys per segment past 100,000)."""
    gblk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
    oblk, exact = executor.execute(qc, raws)
    assert gblk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    if not qc.group_by:
        _assert_intermediates_equal(qc.aggregations, gblk.results, oblk.results, exact)
    else:
        if getattr(gblk, "num_groups_trimmed", False):
            # server-level trim (IndexedTable.finish): the oracle's full group set, trimmed the same way
            from pinot_amd.engine.reduce import trim_groups
            oblk = trim_groups(qc, oblk)
        assert gblk.num_groups_limit_reached == oblk.num_groups_limit_reached
        assert set(gblk.groups) == set(oblk.groups)
        for k, v in oblk.groups.items():
            _assert_intermediates_equal(qc.aggregations, gblk.groups[k], v, exact[k])


@pytest.mark.parametrize("name", sorted(__import__("tools.bq", fromlist=["QUERIES"]).QUERIES))
def test_gpu_c1_benchmark_queries_vs_oracle(name, bq_segments):
    from tools import bq
    raws, segs = bq_segments
    _check_vs_oracle(parse(bq.QUERIES[name]), raws, segs)


# ---- config C4: 5-predicate AND/OR/NOT over inverted indexes, selectivity sweep (tools/c4.py) ---------
@pytest.fixture(scope="module")
def c4_segments(gpu_lib):
    from tools import c4
    raws = [c4.make_segment(i, num_rows=1_000_003) for i in range(2)]
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


@pytest.mark.parametrize("policy", ["cost", "always"])
@pytest.mark.parametrize("agg", ["COUNT(*)", "SUM(M), COUNT(*), MAX(C5)"])
@pytest.mark.parametrize("sel", __import__("tools.c4", fromlist=["SELECTIVITIES"]).SELECTIVITIES)
def test_gpu_c4_inverted_sweep_vs_oracle(sel, agg, policy, c4_segments, monkeypatch):
    """policy 'always' = the reference's leaf choice (every EQ/IN/NOT leaf on the inverted index);
    'cost' = the GPU planner's (inverted only while its bitmaps are cheaper than the forward scan)."""
    from tools import c4
    monkeypatch.setenv("PINOT_AMD_INVERTED", "always" if policy == "always" else "")
    raws, segs = c4_segments
    qc = parse(c4.query(sel, agg))
    _check_vs_oracle(qc, raws, segs)
    # bit-exact doc-id set of the first segment through the filter-only entry point
    op = GpuInstancePlanMaker().make_instance_plan(qc, [segs[0]])
    assert np.array_equal(op.filter_bitmap(), _words_from_mask(executor.filter_mask(qc, raws[0])))


# ---- raw (no-dictionary) columns in filters: value-based scan leaves (RAW_RANGE / RAW_SET) ----------
RAW_FILTERS = [
    "ri BETWEEN -1000 AND 250000", "ri > 5.5 AND ri <= 100000", "ri IN (3, 7, 11, -5, 2.5)", "ri NOT IN (3, 7)",
    "rl >= 1099511627776 OR rl < -5", "rl = 42", "rf > 0.1 AND rf < 0.7", "rf = 0.25", "rf IN (0.1, 0.5)",
    "rd >= 0.5", "rd < 0.25 OR NOT (ri BETWEEN 0 AND 1000000 AND rd > 0.9)", "d IN (1, 2) AND rd <> 0.5",
    # long raw IN lists (unsorted, with duplicates): binary search over the library's sorted copy
    "ri IN (" + ", ".join(str(x) for x in np.random.default_rng(3).integers(-2000, 2_000_000, 3000)) + ")",
    "rd NOT IN (" + ", ".join(f"{x:.3f}" for x in np.random.default_rng(4).random(2500)) + ")",
    "rl IN (42, " + ", ".join(str(x) for x in np.random.default_rng(5).integers(-2 ** 41, 2 ** 41, 1500)) + ", 42)",
    "rf IN (0.0, -0.0, 0.5, 0.25, 0.5)",
]


@pytest.mark.parametrize("flt", RAW_FILTERS)
def test_gpu_raw_column_filters(flt, gpu_lib):
    rng = np.random.default_rng(77)
    n = 2048 * 13 + 77
    c = SegmentCreator("rawf", no_dictionary_columns=["ri", "rl", "rf", "rd"])
    c.add_column("ri", DataType.INT, rng.integers(-2000, 2_000_000, n))
    c.add_column("rl", DataType.LONG, np.where(rng.random(n) < 0.01, 42, rng.integers(-2 ** 41, 2 ** 41, n)))
    c.add_column("rf", DataType.FLOAT, np.round(rng.random(n), 2).astype(np.float32))
    c.add_column("rd", DataType.DOUBLE, np.round(rng.random(n), 3))
    c.add_column("d", DataType.INT, rng.integers(0, 5, n))
    raw = c.build()
    seg = GpuSegment(raw)
    try:
        qc = parse("SELECT COUNT(*), SUM(ri), MAX(rd) FROM t WHERE " + flt)
        blk = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).next_block()
        oblk, ex = executor.execute(qc, [raw])
        assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
        _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
        words = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).filter_bitmap()
        assert np.array_equal(words, _words_from_mask(executor.filter_mask(qc, raw)))
    finally:
        seg.destroy()
