"""Immutable segment writer for the encodings the hot path reads.

Produces, per column, the same index buffers Pinot's segment creator writes (and its loader
maps), so the C-ABI receives exactly what ``ImmutableSegmentLoader`` would hand it:

* dictionary     sorted distinct values, big-endian fixed width
                 (SegmentDictionaryCreator; read by BaseImmutableDictionary.java:124-246;
                 strings padded with '\\0' to the longest UTF-8 length)
* forward index  - unsorted dict column: bit-packed dict ids, MSB-first big-endian,
                   ceil(N*b/8) bytes, b = getNumBitsPerValue(card-1)
                   (FixedBitSVForwardIndexWriter.java:39-50, PinotDataBitSet.java:61-72,
                   SegmentColumnarIndexCreator.java:589)
                 - sorted dict column: card x (startDocId, endDocId) BE int32, inclusive
                   (SortedIndexReaderImpl.java:114-116)
                 - raw (no-dictionary) fixed-width column: chunk format v2..v5, any ChunkCompressionType
                   (BaseChunkForwardIndexWriter.java:40-160)
                 - raw STRING column: var-byte chunks v2 / v3 (VarByteChunkForwardIndexWriter.java:37-158)
* inverted index (card+1) BE u32 absolute offsets + portable Roaring bitmaps
                 (BitmapInvertedIndexWriter.java:35-156)
"""
import ctypes
import os
import subprocess
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from .. import spi
from ..spi import DataType
from . import roaring


_HERE = os.path.dirname(os.path.abspath(__file__))
_INVIDX_SO = os.path.join(_HERE, "libinvidx.so")
_invidx = None


def build_native():
    """Compile invidx.c (the native inverted-index writer; byte-identical to the Python path)."""
    src = os.path.join(_HERE, "invidx.c")
    if not os.path.exists(_INVIDX_SO) or os.path.getmtime(_INVIDX_SO) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-o", _INVIDX_SO, src])


def _native():
    global _invidx
    if _invidx is None:
        build_native()
        L = ctypes.CDLL(_INVIDX_SO)
        for f in (L.phip_invidx_size, L.phip_invidx_write):
            f.restype = ctypes.c_int64
        L.phip_invidx_size.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
        L.phip_invidx_write.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_int64]
        L.phip_pack_bits.restype = None
        L.phip_pack_bits.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
        _invidx = L
    return _invidx


def inverted_index_bytes(ids: np.ndarray, card: int, run_optimize: bool = True, native: bool = True) -> bytes:
    """Bitmap inverted index of dict ids (BitmapInvertedIndexWriter layout): native writer, or the
    Python restatement (``native=False``; kept as the reference the native one is tested against)."""
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    if native:
        L = _native()
        size = L.phip_invidx_size(ids.ctypes.data, len(ids), card, int(run_optimize))
        if size < 0:
            raise ValueError("invalid dict ids for the inverted index")
        out = np.empty(size, dtype=np.uint8)
        if L.phip_invidx_write(ids.ctypes.data, len(ids), card, int(run_optimize), out.ctypes.data, size) != size:
            raise RuntimeError("inverted index writer failed")
        return out.tobytes()
    order = np.argsort(ids, kind="stable")
    bounds = np.searchsorted(ids[order], np.arange(card + 1), side="left")
    bitmaps = [roaring.serialize(order[bounds[d]:bounds[d + 1]], run_optimize) for d in range(card)]
    offsets = np.empty(card + 1, dtype=np.int64)
    pos = (card + 1) * 4
    for d, bm in enumerate(bitmaps):
        offsets[d] = pos
        pos += len(bm)
    offsets[card] = pos
    return offsets.astype(">u4").tobytes() + b"".join(bitmaps)


# FieldSpec's default null values of dimension fields (pinot-spi/.../data/FieldSpec.java:75-81)
DEFAULT_NULL_VALUES = {DataType.INT: -2 ** 31, DataType.LONG: -2 ** 63, DataType.FLOAT: float("-inf"),
                       DataType.DOUBLE: float("-inf"), DataType.STRING: "null"}


@dataclass
class ColumnMetadata:
    name: str
    data_type: DataType
    total_docs: int
    cardinality: int
    bits_per_element: int
    is_sorted: bool
    has_dictionary: bool
    has_inverted_index: bool
    string_width: int = 0  # bytes per padded STRING dictionary entry
    hll_log2m: int = 0     # > 0: a star-tree DISTINCTCOUNTHLL pair column -- per doc 2^log2m u8 HLL registers


@dataclass
class ColumnIndexes:
    metadata: ColumnMetadata
    forward: bytes
    dictionary: Optional[bytes] = None
    inverted: Optional[bytes] = None
    null_vector: Optional[bytes] = None  # portable Roaring bitmap of the null docs (NullValueVectorCreator), or None


@dataclass
class ImmutableSegment:
    name: str
    num_docs: int
    columns: Dict[str, ColumnIndexes] = field(default_factory=dict)
    star_trees: list = field(default_factory=list)  # startree.StarTree per StarTreeIndexConfig

    def column_names(self) -> List[str]:
        return list(self.columns.keys())


def pack_bits(dict_ids: np.ndarray, bits: int, native: bool = True) -> bytes:
    """MSB-first big-endian packing (FixedBitIntReaderWriter.writeInt semantics); native writer, or the
    numpy restatement (``native=False``) it is tested against."""
    ids = np.asarray(dict_ids, dtype=np.uint32)
    n = len(ids)
    if n == 0:
        return b""
    if native:
        L = _native()
        ids32 = np.ascontiguousarray(ids.view(np.int32))
        out = np.zeros((n * bits + 7) // 8, dtype=np.uint8)
        L.phip_pack_bits(ids32.ctypes.data, ctypes.c_int64(n), ctypes.c_int32(bits), out.ctypes.data)
        return out.tobytes()
    be = ids.astype(">u4").view(np.uint8).reshape(n, 4)
    allbits = np.unpackbits(be, axis=1)[:, 32 - bits:]
    packed = np.packbits(allbits.reshape(-1))
    nbytes = (n * bits + 7) // 8
    assert len(packed) == nbytes
    return packed.tobytes()


def _encode_dictionary(sorted_vals, dt: DataType):
    if dt == DataType.STRING:
        enc = [s.encode("utf-8") for s in sorted_vals]
        width = max([len(e) for e in enc] + [1])
        buf = b"".join(e + b"\0" * (width - len(e)) for e in enc)
        return buf, width
    return np.asarray(sorted_vals, dtype=dt.numpy_be).tobytes(), 0


def _sorted_unique(values: np.ndarray, dt: DataType):
    if dt == DataType.STRING:
        # Java String.compareTo order == code point order for BMP text
        uniq = sorted(set(values.tolist()))
        index = {v: i for i, v in enumerate(uniq)}
        ids = np.fromiter((index[v] for v in values.tolist()), dtype=np.int32, count=len(values))
        return uniq, ids
    uniq, ids = np.unique(values, return_inverse=True)
    return uniq, ids.astype(np.int32)


# ChunkCompressionType (pinot-segment-spi/.../compression/ChunkCompressionType.java:22)
CHUNK_COMPRESSION = {"PASS_THROUGH": 0, "SNAPPY": 1, "ZSTANDARD": 2, "LZ4": 3, "LZ4_LENGTH_PREFIXED": 4, "GZIP": 5}


def _compress_chunk(chunk: bytes, codec: int) -> bytes:
    """One chunk through the codec Pinot's writer uses (BaseChunkForwardIndexWriter.writeChunk,
    BaseChunkForwardIndexWriter.java:175-200). The reference binds lz4-java / snappy-java / zstd-jni /
    java.util.zip; here the same published formats come from Arrow's bundled liblz4 / libsnappy / libzstd
    ("lz4_raw" = LZ4 block format without a frame) and Python's zlib (the library java.util.zip wraps).
    LZ4_LENGTH_PREFIXED prepends the 4-byte little-endian original length (lz4-java LZ4CompressorWithLength)."""
    import pyarrow as pa
    if codec == 0:
        return chunk
    if codec == 1:
        return pa.compress(chunk, codec="snappy", asbytes=True)
    if codec in (3, 4):
        body = pa.compress(chunk, codec="lz4_raw", asbytes=True)
        return (len(chunk).to_bytes(4, "little") + body) if codec == 4 else body
    if codec == 2:  # zstd-jni Zstd.compress: one frame at the default level 3 (ZstandardCompressor.java)
        return pa.Codec("zstd", compression_level=3).compress(chunk, asbytes=True)
    if codec == 5:  # GzipCompressor.java:38-46: java.util.zip.Deflater (zlib, default level) + 4-byte BE length
        import zlib
        return zlib.compress(chunk) + len(chunk).to_bytes(4, "big")
    raise NotImplementedError(f"chunk compression {codec}")


def _chunk_forward(values: np.ndarray, dt: DataType, docs_per_chunk: int = 1000, version: int = 3,
                   compression: str = "PASS_THROUGH") -> bytes:
    """Fixed-byte chunk forward index (BaseChunkForwardIndexWriter.java:40-60,130-200): 7-int header,
    chunk offsets (int for v2, long from v3), then each chunk through its codec; offsets are absolute.
    Versions 4 / 5 (fixed-width only, BaseChunkForwardIndexWriter.java:91) round docs per chunk up to a power of
    two (FixedByteChunkForwardIndexWriter.normalizeDocsPerChunk :93-98), which the v4 reader
    (FixedBytePower2ChunkSVForwardIndexReader) turns into a shift."""
    if version not in (2, 3, 4, 5):
        raise ValueError(f"illegal chunk writer version {version} for fixed-byte values")
    if version >= 4 and docs_per_chunk & (docs_per_chunk - 1):
        docs_per_chunk = 1 << (docs_per_chunk - 1).bit_length()
    codec = CHUNK_COMPRESSION[compression]
    n = len(values)
    entry = np.dtype(dt.numpy_be).itemsize
    num_chunks = (n + docs_per_chunk - 1) // docs_per_chunk
    off_size = 4 if version == 2 else 8
    header_size = 7 * 4 + num_chunks * off_size
    header = np.array([version, num_chunks, docs_per_chunk, entry, n, codec, 7 * 4], dtype=">i4").tobytes()
    data = np.asarray(values, dtype=dt.numpy_be).tobytes()
    offsets, chunks = [], []
    pos = header_size
    for c in range(num_chunks):
        lo = c * docs_per_chunk * entry
        body = _compress_chunk(data[lo:lo + min(docs_per_chunk, n - c * docs_per_chunk) * entry], codec)
        offsets.append(pos)
        chunks.append(body)
        pos += len(body)
    offs = np.asarray(offsets, dtype=">i4" if version == 2 else ">i8").tobytes()
    return header + offs + b"".join(chunks)


def _var_byte_forward(values, docs_per_chunk: int = 1000, version: int = 3, compression: str = "PASS_THROUGH") -> bytes:
    """Var-byte chunk forward index of a raw STRING column (VarByteChunkForwardIndexWriter.java:37-158 over the
    BaseChunkForwardIndexWriter header): the 7-int header with lengthOfLongestEntry as the entry size, the chunk
    offsets, then per chunk -- through its codec -- numDocsPerChunk BE int start offsets (0 for the absent rows of a
    partial chunk) followed by the values' UTF-8 bytes. The chunk ends at its last value (the writer flips its buffer
    at the write position)."""
    if version not in (2, 3):
        raise ValueError(f"illegal chunk writer version {version} for variable-length values")
    codec = CHUNK_COMPRESSION[compression]
    enc = [str(s).encode("utf-8") for s in np.asarray(values).tolist()]
    n = len(enc)
    longest = max((len(e) for e in enc), default=0)
    num_chunks = (n + docs_per_chunk - 1) // docs_per_chunk
    off_size = 4 if version == 2 else 8
    header = np.array([version, num_chunks, docs_per_chunk, longest, n, codec, 7 * 4], dtype=">i4").tobytes()
    offsets, chunks = [], []
    pos = 7 * 4 + num_chunks * off_size
    for c in range(num_chunks):
        rows = enc[c * docs_per_chunk:(c + 1) * docs_per_chunk]
        starts = np.zeros(docs_per_chunk, dtype=">i4")
        p = docs_per_chunk * 4
        for j, e in enumerate(rows):
            starts[j] = p
            p += len(e)
        body = _compress_chunk(starts.tobytes() + b"".join(rows), codec)
        offsets.append(pos)
        chunks.append(body)
        pos += len(body)
    offs = np.asarray(offsets, dtype=">i4" if version == 2 else ">i8").tobytes()
    return header + offs + b"".join(chunks)


class SegmentCreator:
    """Builds an ImmutableSegment from column arrays (``SegmentIndexCreationDriverImpl`` role)."""

    def __init__(self, name: str, inverted_index_columns: Sequence[str] = (),
                 no_dictionary_columns: Sequence[str] = (), run_optimize_bitmaps: bool = True,
                 raw_compression=None, docs_per_chunk: int = 1000, raw_version: int = 3,
                 star_tree_configs: Sequence = ()):
        """raw_compression: column -> ChunkCompressionType name for no-dictionary columns
        (PASS_THROUGH when absent, the METRIC default of ForwardIndexType.java:144-150)."""
        self.name = name
        self.compression = dict(raw_compression or {})
        self.docs_per_chunk = docs_per_chunk
        self.raw_version = raw_version
        self.inverted = set(inverted_index_columns)
        self.raw = set(no_dictionary_columns)
        self.run_optimize = run_optimize_bitmaps
        self.star_tree_configs = list(star_tree_configs)
        self._cols = []
        self._ids = {}
        self._nulls = {}

    def add_column(self, name: str, data_type: DataType, values, nulls=None, null_value=None):
        """nulls: optional bool mask of the docs whose value is null. Those docs store the field's default null value
        (``null_value``, else FieldSpec's dimension default: Integer.MIN_VALUE, Long.MIN_VALUE, -inf, "null";
        FieldSpec.java:75-81) in every index, and the column gets a null value vector (NullValueVectorCreator: the
        Roaring bitmap of the null doc ids, written only when some doc is null, :83-92)."""
        if data_type == DataType.STRING:
            arr = np.asarray(values, dtype=object if nulls is not None else np.str_)
        else:
            arr = np.asarray(values, dtype=object if nulls is not None else data_type.numpy)
        if nulls is not None:
            mask = np.asarray(nulls, dtype=bool)
            if len(mask) != len(arr):
                raise ValueError(f"column {name}: {len(mask)} null flags for {len(arr)} values")
            fill = null_value if null_value is not None else DEFAULT_NULL_VALUES[data_type]
            arr = np.where(mask, fill, arr)
            arr = np.asarray(arr, dtype=np.str_ if data_type == DataType.STRING else data_type.numpy)
            if mask.any():
                self._nulls[name] = np.nonzero(mask)[0]
        self._cols.append((name, data_type, arr))
        return self

    def build(self) -> ImmutableSegment:
        if not self._cols:
            raise ValueError("no columns")
        n = len(self._cols[0][2])
        seg = ImmutableSegment(self.name, n)
        for name, dt, vals in self._cols:
            if len(vals) != n:
                raise ValueError(f"column {name}: {len(vals)} values, expected {n}")
            seg.columns[name] = self._build_column(name, dt, vals, n)
            if name in self._nulls:
                seg.columns[name].null_vector = roaring.serialize(self._nulls[name], self.run_optimize)
        if self.star_tree_configs:
            from .startree import build_star_tree
            raw = {name: vals for name, _, vals in self._cols}
            for i, cfg in enumerate(self.star_tree_configs):
                dims = list(cfg.dimensions_split_order)
                for d in dims:
                    if d not in self._ids:
                        raise ValueError(f"star-tree dimension {d} must be a dictionary-encoded column")
                seg.star_trees.append(build_star_tree(cfg, [self._ids[d] for d in dims], [seg.columns[d] for d in dims],
                                                      raw, f"{self.name}.startree{i}",
                                                      {name: dt for name, dt, _ in self._cols}))
        return seg

    def _build_column(self, name, dt, vals, n) -> ColumnIndexes:
        if name in self.raw:
            meta = ColumnMetadata(name, dt, n, 0, 0, False, False, False)
            if dt == DataType.STRING:
                return ColumnIndexes(meta, _var_byte_forward(vals, self.docs_per_chunk, min(self.raw_version, 3),
                                                             self.compression.get(name, "PASS_THROUGH")))
            return ColumnIndexes(meta, _chunk_forward(vals, dt, self.docs_per_chunk, self.raw_version,
                                                      self.compression.get(name, "PASS_THROUGH")))
        uniq, ids = _sorted_unique(vals, dt)
        self._ids[name] = ids
        card = len(uniq)
        dict_bytes, width = _encode_dictionary(uniq, dt)
        is_sorted = bool(n == 0 or np.all(np.diff(ids) >= 0))
        bits = spi.num_bits_per_value(card - 1)
        if is_sorted:
            starts = np.searchsorted(ids, np.arange(card), side="left")
            ends = np.searchsorted(ids, np.arange(card), side="right") - 1
            pairs = np.empty(2 * card, dtype=">i4")
            pairs[0::2] = starts
            pairs[1::2] = ends
            fwd = pairs.tobytes()
        else:
            fwd = pack_bits(ids, bits)
        inv = None
        if name in self.inverted and not is_sorted:
            inv = inverted_index_bytes(ids, card, self.run_optimize)
        meta = ColumnMetadata(name, dt, n, card, bits, is_sorted, True, inv is not None, width)
        return ColumnIndexes(meta, fwd, dict_bytes, inv)
