"""Index bytes WRITTEN BY PINOT (the reference's own test data, tests/golden/pinot_written/, copied by
tests/golden/make_pinot_written.py) through the loader, the oracle and the GPU.

* paddingNull/ : a v1 segment directory (5 docs; INT / STRING / FLOAT / LONG dictionary columns with
  fixed-bit forward indexes) written by Pinot's segment creator. Values below are decoded by hand from the
  file bytes (MSB-first b-bit ids, BE dictionaries) and agree with the metadata (segment.start.time 246 /
  end.time 902 = min / max of outgoingName1).
* paddingOld/, paddingPercent/ : the same data with '%' padding; the reference refuses to load them
  (ColumnMetadataImpl.java:250-253, "Only support zero padding"), and so does read_segment_dir.
* fixedByte{Raw,Compressed}.v2, fixedByteSVRDoubles.v1 : DOUBLE fixed-byte chunk forward indexes
  (PASS_THROUGH v2, SNAPPY v2, SNAPPY v1) that FixedByteChunkSVForwardIndexTest.testBackwardCompatibility
  (:331-345) reads as value(i) = i + 100.2356 (2000 docs) and i + 0 (10009 docs).
"""
import os
import struct

import numpy as np
import pytest

from oracle import executor
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import ColumnIndexes, ColumnMetadata, ImmutableSegment, SegmentCreator, _chunk_forward
from pinot_amd.segment.store import read_segment_dir, write_segment_dir
from pinot_amd.spi import DataType

PW = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pinot_written")
PERCENT_DICT = [struct.unpack(">f", bytes.fromhex(h))[0] for h in ("43aaefd7", "43cddc91", "44466a89", "445829c1", "44675045")]
DOCS = {
    "age": [1228, 837, 1209, 617, 824],                       # ids 4,2,3,0,1 of (617, 824, 837, 1209, 1228)
    "name": ["lynda", "lynda 2.0", "lynda 2.0", "lynda 2.0", "lynda"],  # ids 0,1,1,1,0
    "percent": [PERCENT_DICT[i] for i in (0, 2, 4, 3, 1)],
    "outgoingName1": [902, 467, 310, 246, 336],               # ids 4,3,1,0,2 of (246, 310, 336, 467, 902)
}
TYPES = {"age": DataType.INT, "name": DataType.STRING, "percent": DataType.FLOAT, "outgoingName1": DataType.LONG}
CHUNK_FILES = [("fixedByteRaw.v2", 2000, 100.2356), ("fixedByteCompressed.v2", 2000, 100.2356),
               ("fixedByteSVRDoubles.v1", 10009, 0.0)]


def _padding_null():
    return read_segment_dir(os.path.join(PW, "paddingNull"))


def test_read_pinot_v1_segment_values():
    seg = _padding_null()
    assert seg.num_docs == 5 and set(seg.columns) == set(DOCS)
    from oracle.executor import OracleSegment
    os_ = OracleSegment(seg)
    for col, want in DOCS.items():
        got = os_.values(col).tolist()
        assert got == (want if col != "percent" else [float(np.float32(x)) for x in want]), col


@pytest.mark.parametrize("col", sorted(DOCS))
def test_segment_creator_writes_pinot_bytes(col):
    """Our writer, given the decoded values, emits Pinot's forward-index and dictionary bytes exactly
    (FixedBitSVForwardIndexWriter.java:33-50, SegmentDictionaryCreator)."""
    pinot = _padding_null().columns[col]
    ours = SegmentCreator("x").add_column(col, TYPES[col], DOCS[col]).build().columns[col]
    assert ours.forward == pinot.forward
    assert ours.dictionary == pinot.dictionary
    assert ours.metadata.bits_per_element == pinot.metadata.bits_per_element
    assert ours.metadata.cardinality == pinot.metadata.cardinality


@pytest.mark.parametrize("name", ["paddingOld", "paddingPercent"])
def test_non_zero_padding_rejected(name):
    with pytest.raises(ValueError, match="non-zero string padding"):
        read_segment_dir(os.path.join(PW, name))


@pytest.mark.parametrize("version", [1, 3])
def test_segment_dir_round_trip(tmp_path, version):
    rng = np.random.default_rng(4)
    n = 3001
    c = SegmentCreator("rt", inverted_index_columns=["a"], no_dictionary_columns=["r"])
    c.add_column("a", DataType.INT, rng.integers(0, 50, n))
    c.add_column("s", DataType.STRING, np.array([f"v{x}" for x in rng.integers(0, 9, n)]))
    c.add_column("t", DataType.LONG, np.arange(n) // 7)  # sorted
    c.add_column("r", DataType.DOUBLE, rng.random(n))
    seg = c.build()
    back = read_segment_dir(write_segment_dir(seg, str(tmp_path / "seg"), version=version))
    assert back.num_docs == n and list(back.columns) == list(seg.columns)
    for col, ci in seg.columns.items():
        bi = back.columns[col]
        assert bi.metadata == ci.metadata, col
        assert (bi.forward, bi.dictionary, bi.inverted) == (ci.forward, ci.dictionary, ci.inverted), col


def _chunk_segment(fname, n):
    with open(os.path.join(PW, fname), "rb") as f:
        fwd = f.read()
    meta = ColumnMetadata("v", DataType.DOUBLE, n, 0, 0, False, False, False)
    return ImmutableSegment(fname, n, {"v": ColumnIndexes(meta, fwd)})


@pytest.mark.parametrize("fname,n,start", CHUNK_FILES)
def test_oracle_reads_pinot_chunk_files(fname, n, start):
    from oracle.executor import OracleSegment
    vals = OracleSegment(_chunk_segment(fname, n)).values("v")
    assert vals.tolist() == [i + start for i in range(n)]


def test_chunk_writer_matches_pinot_pass_through():
    vals = np.array([i + 100.2356 for i in range(2000)])
    with open(os.path.join(PW, "fixedByteRaw.v2"), "rb") as f:
        assert _chunk_forward(vals, DataType.DOUBLE, docs_per_chunk=1000, version=2) == f.read()


# ---------------------------------------------------------------------------------------------- GPU
PADDING_QUERIES = [
    "SELECT name, COUNT(*), SUM(age), MIN(percent), MAX(outgoingName1), DISTINCTCOUNTHLL(age) FROM t GROUP BY name",
    "SELECT COUNT(*), SUM(outgoingName1), MAX(percent) FROM t WHERE age > 800 AND name = 'lynda 2.0'",
    "SELECT COUNT(*), DISTINCTCOUNTHLL(name), MIN(age) FROM t WHERE percent < 800 OR outgoingName1 = 902",
    "SELECT outgoingName1, age, SUM(percent) FROM t WHERE name <> 'lynda' GROUP BY outgoingName1, age",
]


@pytest.mark.gpu
@pytest.mark.parametrize("sql", PADDING_QUERIES)
def test_gpu_pinot_written_segment(gpu_lib, sql):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from tests.test_gpu_limits import _check
    from tests.test_gpu_parity import _assert_intermediates_equal
    raw = _padding_null()
    seg = GpuSegment(raw)
    try:
        qc = parse(sql)
        blk = GpuInstancePlanMaker().make_instance_plan(qc, [seg]).next_block()
        oblk, ex = executor.execute(qc, [raw])
        if qc.group_by:
            _check(qc, blk, oblk, ex)
        else:
            assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
            _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
        if sql.startswith("SELECT name"):
            assert blk.groups[("lynda",)][:2] == [2, 1228 + 824]
            assert blk.groups[("lynda 2.0",)][:2] == [3, 837 + 1209 + 617]
            assert blk.groups[("lynda",)][3] == 902.0
        if "age > 800" in sql:
            assert blk.results[0] == 2 and blk.results[1] == 467 + 310
    finally:
        seg.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("fname,n,start", CHUNK_FILES)
def test_gpu_pinot_chunk_files(gpu_lib, fname, n, start):
    """PASS_THROUGH v2 / SNAPPY v2 / SNAPPY v1 chunks written by Pinot, decoded at pin time on the GPU."""
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from tests.test_gpu_parity import _assert_intermediates_equal, _words_from_mask
    raw = _chunk_segment(fname, n)
    seg = GpuSegment(raw)
    try:
        half = n // 2 + start
        for sql in ("SELECT COUNT(*), SUM(v), MIN(v), MAX(v) FROM t",
                    f"SELECT COUNT(*), SUM(v), MIN(v) FROM t WHERE v >= {half!r}"):
            qc = parse(sql)
            op = GpuInstancePlanMaker().make_instance_plan(qc, [seg])
            blk = op.next_block()
            oblk, ex = executor.execute(qc, [raw])
            _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
            if "WHERE" in sql:
                assert blk.results[0] == n - n // 2 and blk.results[2] == half
                words = op.filter_bitmap()
                assert np.array_equal(words, _words_from_mask(np.arange(n) >= n // 2))
            else:
                assert blk.results[0] == n and blk.results[2] == start and blk.results[3] == n - 1 + start
    finally:
        seg.destroy()
