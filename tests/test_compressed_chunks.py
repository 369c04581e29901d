"""Compressed raw forward indexes: SNAPPY / LZ4 / LZ4_LENGTH_PREFIXED chunks.

Reference: BaseChunkForwardIndexWriter.writeChunk (BaseChunkForwardIndexWriter.java:175-200) compresses each
fixed-byte chunk with the column's ChunkCompressionType; BaseChunkForwardIndexReader.decompressChunk
(BaseChunkForwardIndexReader.java:204-232) sizes chunk k as offset_{k+1} - offset_k (the last one runs to the
end of the buffer) and hands it to lz4-java 1.8.0 / snappy-java 1.1.10.7 (LZ4Decompressor.java,
LZ4WithLengthDecompressor.java, SnappyDecompressor.java).

Parity pinning: the reference holds no compressed-chunk fixtures, and its codecs are third-party JVM
libraries absent here. The oracle's decoders (oracle/pinot_oracle.c) are therefore pinned against an
independent implementation of the same published block formats -- Arrow's bundled liblz4 ("lz4_raw") and
libsnappy -- in both directions (Arrow encodes, the oracle decodes; the oracle's output equals Arrow's
decode). The GPU path (chunk_decode_kernel, decoded once at pin time) must be bit-exact with the oracle.
"""
import numpy as np
import pyarrow as pa
import pytest

from oracle import executor, lib as oracle_lib
from pinot_amd.segment.creator import CHUNK_COMPRESSION, SegmentCreator, _compress_chunk
from pinot_amd.spi import DataType

CODECS = ("SNAPPY", "LZ4", "LZ4_LENGTH_PREFIXED")
ENTROPY = ("ZSTANDARD", "GZIP")  # decoded by pinot_amd/csrc/codec.h (tests/test_codec.py pins it on the host)


def _payloads():
    rng = np.random.default_rng(11)
    return {
        "empty": b"",
        "one": b"\x07",
        "zeros8000": bytes(8000),
        "ramp_i64": np.arange(1000, dtype=">i8").tobytes(),
        "lowcard_i64": rng.integers(0, 5, 1000).astype(">i8").tobytes(),
        "random_i64": rng.integers(-2 ** 62, 2 ** 62, 1000).astype(">i8").tobytes(),
        "period3": b"abc" * 3000,             # match offset 3 < length: overlapping copies
        "period1": b"z" * 5000,                # offset 1
        "long_literal": rng.integers(0, 256, 300, dtype=np.uint8).tobytes() + bytes(700),  # literal len > 270
        "mixed": (rng.integers(0, 256, 17, dtype=np.uint8).tobytes() + b"q" * 300) * 20,
    }


def _decode(codec, blob, cap):
    src = np.frombuffer(blob, dtype=np.uint8).copy() if blob else np.zeros(1, np.uint8)
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    got = oracle_lib().oracle_chunk_decode(codec, src.ctypes.data, len(blob), dst.ctypes.data, cap)
    return got, dst[:max(got, 0)].tobytes()


@pytest.mark.parametrize("codec", CODECS)
def test_oracle_decoders_match_arrow(codec):
    cid = CHUNK_COMPRESSION[codec]
    for name, data in _payloads().items():
        blob = _compress_chunk(data, cid)
        got, out = _decode(cid, blob, len(data))
        assert got == len(data) and out == data, (codec, name, got)
        # the independent decoder agrees on the same bytes
        body = blob[4:] if cid == 4 else blob
        ref = pa.decompress(body, decompressed_size=len(data), codec="snappy" if cid == 1 else "lz4_raw",
                            asbytes=True) if data else b""
        assert ref == out, (codec, name)


def test_oracle_handcrafted_lz4_sequences():
    # token 0x1f: 1 literal 'x', match length 15+ext; ext byte 1 -> 15+1+4 = 20; offset 1 -> 'x' * 21
    blob = bytes([0x1F, ord("x"), 1, 0, 1, 0x10, ord("!")])
    got, out = _decode(3, blob, 22)
    assert got == 22 and out == b"x" * 21 + b"!"
    # length-prefixed wrapper: LE length then the block
    got, out = _decode(4, (22).to_bytes(4, "little") + blob, 22)
    assert got == 22 and out == b"x" * 21 + b"!"


@pytest.mark.parametrize("blob,codec", [
    (bytes([0x10, ord("a"), 0, 0]), 3),          # offset 0
    (bytes([0x10, ord("a"), 5, 0]), 3),          # offset beyond the decoded prefix
    (bytes([0xF0]), 3),                           # truncated literal-length extension
    (bytes([0x50, 1, 2]), 3),                     # literals run past the input
    ((9).to_bytes(4, "little") + bytes([0x10, ord("a")]), 4),  # prefixed length disagrees
    (bytes([0x05, 0x04, ord("a")]), 1),           # snappy: literal shorter than declared length
    (bytes([0x04, 0x01, 0x05]), 1),               # snappy: copy before any output
])
def test_oracle_rejects_malformed(blob, codec):
    got, _ = _decode(codec, blob, 64)
    assert got == -1


def _segment(n, codec, seed=3, docs_per_chunk=1000, version=3):
    rng = np.random.default_rng(seed)
    c = SegmentCreator(f"cmp_{codec}", no_dictionary_columns=["L", "I", "F", "D", "LC"],
                       raw_compression={k: codec for k in ("L", "I", "F", "D", "LC")},
                       docs_per_chunk=docs_per_chunk, raw_version=version)
    c.add_column("INT_COL", DataType.INT, rng.integers(0, 5000, n))
    c.add_column("L", DataType.LONG, rng.integers(-2 ** 40, 2 ** 40, n))
    c.add_column("I", DataType.INT, rng.integers(-2 ** 31, 2 ** 31, n))
    c.add_column("F", DataType.FLOAT, rng.standard_normal(n).astype(np.float32))
    c.add_column("D", DataType.DOUBLE, rng.standard_normal(n) * 1e6)
    c.add_column("LC", DataType.LONG, rng.integers(0, 7, n) * 1000)  # compressible
    return c.build(), c._cols


@pytest.mark.parametrize("codec", CODECS + ENTROPY + ("PASS_THROUGH",))
@pytest.mark.parametrize("docs_per_chunk,version", [(1000, 3), (7, 2), (4096, 3), (1000, 4), (100, 5)])
def test_oracle_reads_compressed_segment(codec, docs_per_chunk, version):
    n = 10_007
    seg, cols = _segment(n, codec, docs_per_chunk=docs_per_chunk, version=version)
    oseg = executor.OracleSegment(seg)
    for name, dt, vals in cols:
        if name == "INT_COL":
            continue
        assert seg.columns[name].forward[20:24] == CHUNK_COMPRESSION[codec].to_bytes(4, "big")
        got = oseg.values(name)
        want = np.asarray(vals, dtype=dt.numpy).astype(got.dtype)
        assert np.array_equal(got, want), (codec, name)


def test_v4_chunks_are_power_of_two():
    """FixedByteChunkForwardIndexWriter.normalizeDocsPerChunk (:93-98): v4 / v5 round the chunk up to a power of
    two, and the v4 header is what FixedBytePower2ChunkSVForwardIndexReader reads (ForwardIndexReaderFactory:113-117)."""
    for ver, want in ((3, 1000), (4, 1024), (5, 1024)):
        seg, _ = _segment(5000, "LZ4", docs_per_chunk=1000, version=ver)
        hdr = np.frombuffer(seg.columns["L"].forward[:28], dtype=">i4")
        assert hdr[0] == ver and hdr[2] == want and hdr[1] == -(-5000 // want)
    with pytest.raises(ValueError):
        _segment(100, "LZ4", version=6)


# ------------------------------------------------------------------------------------------ GPU
QUERIES = (
    "SELECT SUM(L), MIN(L), MAX(L), SUM(I), SUM(LC), COUNT(*) FROM t",
    "SELECT SUM(D), MIN(F), MAX(D), SUM(L) FROM t WHERE INT_COL > 5 AND INT_COL < 1499",
    "SELECT COUNT(*), SUM(I) FROM t WHERE L BETWEEN -100000000000 AND 300000000000",
    "SELECT COUNT(*), SUM(L) FROM t WHERE LC IN (2000, 5000) AND INT_COL >= 100",
)


@pytest.mark.gpu
@pytest.mark.parametrize("codec", CODECS + ENTROPY)
def test_gpu_compressed_raw_columns(gpu_lib, codec):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tests.test_gpu_parity import _assert_intermediates_equal
    segs, gsegs = [], []
    try:
        for seed, dpc, ver in ((3, 1000, 3), (4, 7, 2), (5, 4096, 3), (6, 1000, 4), (7, 300, 5)):
            s, _ = _segment(123_457 if dpc != 7 else 20_001, codec, seed=seed, docs_per_chunk=dpc, version=ver)
            segs.append(s)
            gsegs.append(GpuSegment(s))
        for q in QUERIES:
            qc = parse(q)
            blk = GpuInstancePlanMaker().make_instance_plan(qc, gsegs).next_block()
            oblk, ex = executor.execute(qc, segs)
            _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
    finally:
        for g in gsegs:
            g.destroy()


@pytest.mark.gpu
def test_gpu_compressed_equals_pass_through_large(gpu_lib):
    """6M rows (one SSB-sized segment), LZ4: every aggregate equals the PASS_THROUGH copy of the same
    values and the exact int64 sum of the source (size-independent check; the oracle is not run here)."""
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    rng = np.random.default_rng(9)
    n = 6_000_000
    v = rng.integers(0, 10_000, n) * 97 - 3
    res = {}
    for codec in ("LZ4", "PASS_THROUGH"):
        c = SegmentCreator(codec, no_dictionary_columns=["M"], raw_compression={"M": codec})
        c.add_column("M", DataType.LONG, v)
        g = GpuSegment(c.build())
        try:
            qc = parse("SELECT SUM(M), MIN(M), MAX(M), COUNT(*) FROM t WHERE M > 5000")
            res[codec] = GpuInstancePlanMaker().make_instance_plan(qc, [g]).next_block().results
        finally:
            g.destroy()
    assert res["LZ4"] == res["PASS_THROUGH"]
    sel = v[v > 5000]
    assert res["LZ4"][0] == int(sel.sum()) and res["LZ4"][3] == len(sel)


@pytest.mark.gpu
def test_gpu_rejects_malformed_and_unsupported_chunks(gpu_lib):
    from pinot_amd import _lib
    from pinot_amd.engine.segment import GpuSegment
    rng = np.random.default_rng(1)
    n = 5000
    c = SegmentCreator("bad", no_dictionary_columns=["M"], raw_compression={"M": "LZ4"})
    c.add_column("M", DataType.LONG, rng.integers(0, 3, n))
    seg = c.build()
    fwd = bytearray(seg.columns["M"].forward)
    # the second chunk's first match offset -> 0xFFFF (beyond its decoded prefix)
    off1 = int.from_bytes(fwd[28 + 8:28 + 16], "big")
    tok, p = fwd[off1], off1 + 1
    lit = tok >> 4
    if lit == 15:
        while fwd[p] == 255:
            lit, p = lit + 255, p + 1
        lit, p = lit + fwd[p], p + 1
    p += lit
    fwd[p:p + 2] = b"\xff\xff"
    seg.columns["M"].forward = bytes(fwd)
    with pytest.raises(_lib.PhipError, match="malformed compressed chunk"):
        GpuSegment(seg)
    for codec in ENTROPY:  # a flipped byte in the last chunk: libzstd / zlib would throw, so the load fails
        z = SegmentCreator(codec, no_dictionary_columns=["M"], raw_compression={"M": codec})
        z.add_column("M", DataType.LONG, rng.integers(0, 3, n))
        zs = z.build()
        f = bytearray(zs.columns["M"].forward)
        nchunks = int.from_bytes(f[4:8], "big")
        last = int.from_bytes(f[28 + 8 * (nchunks - 1):28 + 8 * nchunks], "big")  # v3: long offsets
        f[last] ^= 0x5A  # the last chunk's zstd magic / zlib CMF byte
        zs.columns["M"].forward = bytes(f)
        with pytest.raises(_lib.PhipError, match="malformed compressed chunk"):
            GpuSegment(zs)
