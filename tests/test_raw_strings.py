"""Raw (no-dictionary) STRING columns: the var-byte chunk forward index and value-based string predicates
(SURVEY.md §8 a9 / a16 for STRING; RangePredicateEvaluatorFactory's StringRawValueBasedRangePredicateEvaluator and the
raw EQ / IN evaluators, String.compareTo order).

Pinned by Pinot-written bytes: varByteStrings{Raw,Compressed}.v2 and varByteStrings.v1 (the reference's test data,
copied by tests/golden/make_pinot_written.py), which VarByteChunkSVForwardIndexTest.testBackwardCompatibility
(:146-161) reads as data[i % 4]; our writer reproduces the PASS_THROUGH file byte for byte. GPU tests compare the
HIP filter (doc bitmaps through the C ABI) and aggregations with the oracle over Pinot's files and over segments of
every chunk codec, version and chunk size."""
import os

import numpy as np
import pytest

from oracle import executor
from oracle.executor import OracleSegment, java_string_key
from pinot_amd import _lib
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import (ColumnIndexes, ColumnMetadata, ImmutableSegment, SegmentCreator,
                                       _var_byte_forward)
from pinot_amd.spi import DataType

PW = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pinot_written")
DATA_V2 = ["abcdefghijk", "12456887", "pqrstuv", "500"]
DATA_V1 = ["abcde", "fgh", "ijklmn", "12345"]
VAR_FILES = [("varByteStringsRaw.v2", 1000, DATA_V2), ("varByteStringsCompressed.v2", 1000, DATA_V2),
             ("varByteStrings.v1", 5003, DATA_V1)]
CODECS = ["PASS_THROUGH", "SNAPPY", "ZSTANDARD", "LZ4", "LZ4_LENGTH_PREFIXED", "GZIP"]
# BMP below the surrogates, U+E000.. (after surrogate pairs in String order), supplementary, empty, long
ALPHABET = ["", "a", "ab", "abc", "b", "B", "z", "zz", "0", "10", "9", "é", "ñu", "中文", "x",
            "￿", "\U0001F600", "\U0001F600a", "a" * 40, "mid", "mi", "mé"]


def _raw_segment(fname, n):
    with open(os.path.join(PW, fname), "rb") as f:
        fwd = f.read()
    meta = ColumnMetadata("v", DataType.STRING, n, 0, 0, False, False, False)
    return ImmutableSegment(fname, n, {"v": ColumnIndexes(meta, fwd)})


def _synthetic(n, seed, codec, version=3, docs_per_chunk=1000):
    rng = np.random.default_rng(seed)
    s = [ALPHABET[i] for i in rng.integers(0, len(ALPHABET), n)]
    # some unique values too (a large IN list hits them)
    for i in rng.integers(0, n, n // 10):
        s[i] = f"k{i:05d}"
    x = rng.integers(-1000, 1000, n).astype(np.int32)
    g = rng.integers(0, 7, n).astype(np.int32)
    c = SegmentCreator(f"rs_{codec}_{version}_{docs_per_chunk}", no_dictionary_columns=["s"],
                       raw_compression={"s": codec}, docs_per_chunk=docs_per_chunk, raw_version=version)
    return c.add_column("s", DataType.STRING, s).add_column("x", DataType.INT, x).add_column("g", DataType.INT, g).build()


# ---------------------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("fname,n,data", VAR_FILES)
def test_oracle_reads_pinot_var_byte_files(fname, n, data):
    vals = OracleSegment(_raw_segment(fname, n)).values("v")
    assert vals.tolist() == [data[i % 4] for i in range(n)]


def test_var_byte_writer_matches_pinot_pass_through():
    """numDocsPerChunk = 1 MiB / (lengthOfLongestEntry + 4) = 69905 (SingleValueVarByteRawIndexCreator
    .getNumDocsPerChunk :95-98), writer version 2, PASS_THROUGH: Pinot's bytes exactly."""
    vals = np.array([DATA_V2[i % 4] for i in range(1000)])
    with open(os.path.join(PW, "varByteStringsRaw.v2"), "rb") as f:
        assert _var_byte_forward(vals, docs_per_chunk=69905, version=2) == f.read()


@pytest.mark.parametrize("version", [2, 3])
@pytest.mark.parametrize("codec", CODECS)
@pytest.mark.parametrize("docs_per_chunk", [7, 1000])
def test_var_byte_round_trip(version, codec, docs_per_chunk):
    raw = _synthetic(2051, 3, codec, version, docs_per_chunk)
    col = raw.columns["s"]
    assert not col.metadata.has_dictionary
    got = OracleSegment(raw).values("s").tolist()
    rng = np.random.default_rng(3)
    want = [ALPHABET[i] for i in rng.integers(0, len(ALPHABET), 2051)]
    for i in rng.integers(0, 2051, 2051 // 10):
        want[i] = f"k{i:05d}"
    assert got == want


def test_java_string_order():
    """String.compareTo compares UTF-16 code units: a supplementary character (a surrogate pair, 0xD83D..) sorts
    below U+E000..U+FFFF although its code point is larger."""
    assert java_string_key("\U0001F600") < java_string_key("")
    assert java_string_key("퟿") < java_string_key("\U0001F600")
    assert java_string_key("ab") < java_string_key("abc") < java_string_key("abd")
    assert java_string_key("") < java_string_key("\0")


def test_raw_string_leaf_payloads():
    from pinot_amd.engine.plan import _raw_string_predicate
    from pinot_amd.query.predicate import Predicate
    from pinot_amd.query.context import Identifier
    leaf = _raw_string_predicate("s", Predicate("IN", Identifier("s"), ("bb", "a", "bb", 5)))
    assert leaf.kind == _lib.LEAF_RAW_STRING_SET and not leaf.exclusive
    w = leaf.ids
    assert w[0] == 3 and list(w[1:5]) == [0, 1, 2, 4]  # "5", "a", "bb" (bytes order; the library re-sorts)
    assert w[5:].tobytes()[:4] == b"5abb"
    rng = _raw_string_predicate("s", Predicate("RANGE", Identifier("s"), (), "b", "*", True, False))
    assert rng.kind == _lib.LEAF_RAW_STRING_RANGE
    assert list(rng.ids[:4]) == [1, -1, 1, 0] and rng.ids[4:].tobytes()[:1] == b"b"
    none = _raw_string_predicate("s", Predicate("NOT_IN", Identifier("s"), ()))
    assert none.kind == _lib.LEAF_MATCH_ALL


# ---------------------------------------------------------------------------------------------- GPU
def _gpu_check(raw, sqls):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from tests.test_gpu_parity import _assert_intermediates_equal, _words_from_mask
    seg = GpuSegment(raw)
    os_ = OracleSegment(raw)
    try:
        for sql in sqls:
            qc = parse(sql)
            op = GpuInstancePlanMaker().make_instance_plan(qc, [seg])
            blk = op.next_block()
            oblk, ex = executor.execute(qc, [raw])
            if qc.group_by:
                assert set(blk.groups) == set(oblk.groups), sql
                for k, v in blk.groups.items():
                    _assert_intermediates_equal(qc.aggregations, v, oblk.groups[k], ex[k])
            else:
                _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
            assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned, sql
            if qc.filter is not None and not qc.group_by:
                words = op.filter_bitmap()
                want = _words_from_mask(executor.eval_filter(os_, qc.filter))
                assert np.array_equal(words, want), sql
            op.close()
    finally:
        seg.destroy()


PINOT_FILE_FILTERS = ["v = '{0}'", "v <> '{1}'", "v IN ('{2}', '{3}', 'nope')", "v NOT IN ('{0}', '{2}')",
                      "v > '2'", "v >= '{1}'", "v < 'abc'", "v BETWEEN '1' AND '5'", "v < '{0}' OR v = '{3}'"]


@pytest.mark.gpu
@pytest.mark.parametrize("fname,n,data", VAR_FILES)
def test_gpu_pinot_var_byte_files(gpu_lib, fname, n, data):
    """Pinot-written var-byte chunks (PASS_THROUGH v2, SNAPPY v2, SNAPPY v1) pinned and decoded on the GPU, then
    filtered by value; COUNT per predicate = the known pattern's."""
    raw = _raw_segment(fname, n)
    sqls = [f"SELECT COUNT(*) FROM t WHERE " + f.format(*data) for f in PINOT_FILE_FILTERS]
    _gpu_check(raw, sqls)
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    seg = GpuSegment(raw)
    try:
        blk = GpuInstancePlanMaker().make_instance_plan(parse(f"SELECT COUNT(*) FROM t WHERE v = '{data[1]}'"),
                                                       [seg]).next_block()
        assert blk.results[0] == len(range(1, n, 4))
    finally:
        seg.destroy()


SYNTH_QUERIES = [
    "SELECT COUNT(*), SUM(x) FROM t WHERE s = 'abc'",
    "SELECT COUNT(*), SUM(x), MIN(x) FROM t WHERE s <> ''",
    "SELECT COUNT(*), MAX(x) FROM t WHERE s IN ('a', 'zz', '\U0001F600', 'x', 'k00017', '')",
    "SELECT COUNT(*), SUM(x) FROM t WHERE s NOT IN ('a', 'b', 'B')",
    "SELECT COUNT(*), SUM(x) FROM t WHERE s > 'm'",
    "SELECT COUNT(*), SUM(x) FROM t WHERE s >= 'mi' AND s < 'mid'",
    "SELECT COUNT(*), SUM(x) FROM t WHERE s BETWEEN 'a' AND 'b'",
    # String order: the supplementary character sorts below U+E000 (UTF-16 code units)
    "SELECT COUNT(*), SUM(x) FROM t WHERE s > '\U0001F600' AND s < '￿'",
    "SELECT COUNT(*), SUM(x) FROM t WHERE s < ''",
    "SELECT COUNT(*), SUM(x) FROM t WHERE (s < '1' OR s > 'z') AND x > 0",
    "SELECT COUNT(*), SUM(x) FROM t WHERE NOT (s = 'a') AND g IN (1, 2, 3)",
    "SELECT g, COUNT(*), SUM(x) FROM t WHERE s BETWEEN 'k00100' AND 'k01500' GROUP BY g",
]


@pytest.mark.gpu
@pytest.mark.parametrize("codec,version,docs_per_chunk", [("PASS_THROUGH", 3, 1000), ("PASS_THROUGH", 2, 7),
                                                         ("SNAPPY", 3, 1000), ("ZSTANDARD", 3, 333),
                                                         ("LZ4", 2, 1000), ("LZ4_LENGTH_PREFIXED", 3, 64),
                                                         ("GZIP", 3, 1000)])
def test_gpu_raw_string_predicates(gpu_lib, codec, version, docs_per_chunk):
    _gpu_check(_synthetic(9001, 11, codec, version, docs_per_chunk), SYNTH_QUERIES)


@pytest.mark.gpu
def test_gpu_raw_string_long_in_list(gpu_lib):
    """A long IN list (binary search over the library's sorted, deduplicated copy) and its NOT IN."""
    raw = _synthetic(20000, 5, "PASS_THROUGH")
    vals = ", ".join(f"'k{i:05d}'" for i in range(0, 20000, 3))
    _gpu_check(raw, [f"SELECT COUNT(*), SUM(x) FROM t WHERE s IN ({vals}, 'a')",
                     f"SELECT COUNT(*), SUM(x) FROM t WHERE s NOT IN ({vals})"])


@pytest.mark.gpu
def test_gpu_raw_string_multi_segment(gpu_lib):
    """Segments of different codecs in one query (one combine over all of them)."""
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from tests.test_gpu_parity import _assert_intermediates_equal
    raws = [_synthetic(5000 + 37 * i, 20 + i, c) for i, c in enumerate(CODECS)]
    segs = [GpuSegment(r) for r in raws]
    try:
        for sql in SYNTH_QUERIES[:8]:
            qc = parse(sql)
            blk = GpuInstancePlanMaker().make_instance_plan(qc, segs).next_block()
            oblk, ex = executor.execute(qc, raws)
            _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
            assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
            assert blk.stats.num_entries_scanned_in_filter > 0
    finally:
        for s in segs:
            s.destroy()
