"""On-disk segment directories: the read side ImmutableSegmentLoader maps, and a writer for tests.

The loader's job on the path is to find, per column, the forward index, the
dictionary and the inverted index buffers and hand them to ``phip_segment_load`` unchanged (big-endian
bytes, exactly as Pinot wrote them). Two directory layouts exist:

* v1 / v2 (FilePerIndexDirectory, pinot-segment-local/.../segment/store/FilePerIndexDirectory.java:184-199):
  one file per index, named by V1Constants (pinot-segment-spi/.../V1Constants.java:34-45):
  ``<col>.dict``, ``<col>.sv.unsorted.fwd`` (fixed-bit dict ids), ``<col>.sv.sorted.fwd`` (doc ranges),
  ``<col>.sv.raw.fwd`` (fixed-byte chunks), ``<col>.bitmap.inv`` (Roaring inverted index), ``<col>.bitmap.nullvalue``
  (the null value vector: one Roaring bitmap, NullValueVectorCreator.java:83-92);
* v3 (SingleFileIndexDirectory.java:72-73,165-185,225-310): ``v3/columns.psf`` holds every buffer,
  each preceded by the 8-byte magic 0xdeadbeefdeafbead; ``v3/index_map`` records
  ``<col>.<index>.startOffset`` / ``.size`` (size includes the magic) for the index ids
  ``dictionary``, ``forward_index``, ``inverted_index``, ``nullvalue_vector``.

Column metadata comes from ``metadata.properties`` (ColumnMetadataImpl.fromPropertiesConfiguration,
pinot-segment-spi/.../index/metadata/ColumnMetadataImpl.java:200-260): cardinality, bitsPerElement,
dataType, isSorted, hasDictionary, lengthOfEachEntry (STRING dictionary entry width). Like the reference,
a segment whose ``segment.padding.character`` is not ``\\0`` is rejected (ColumnMetadataImpl.java:250-253:
"Only support zero padding"), which covers both padded legacy layouts in the reference's test data.
"""
import os
import struct
from typing import Dict

from ..spi import DataType
from .creator import ColumnIndexes, ColumnMetadata, ImmutableSegment

MAGIC_MARKER = 0xDEADBEEFDEAFBEAD
_EXT = {"dictionary": ".dict", "sorted": ".sv.sorted.fwd", "unsorted": ".sv.unsorted.fwd", "raw": ".sv.raw.fwd",
        "inverted": ".bitmap.inv", "nullvalue": ".bitmap.nullvalue"}
# v3 index ids (StandardIndexes.java: "dictionary", "forward_index", "inverted_index", "nullvalue_vector")
_INDEX_ID = {"dictionary": "dictionary", "inverted": "inverted_index", "nullvalue": "nullvalue_vector"}
_TYPES = {"INT": DataType.INT, "LONG": DataType.LONG, "FLOAT": DataType.FLOAT, "DOUBLE": DataType.DOUBLE,
          "STRING": DataType.STRING}


def _unescape_java(v: str) -> str:
    out, i = [], 0
    while i < len(v):
        c = v[i]
        if c == "\\" and i + 1 < len(v):
            n = v[i + 1]
            if n == "u" and i + 5 < len(v):
                out.append(chr(int(v[i + 2:i + 6], 16)))
                i += 6
                continue
            out.append({"t": "\t", "n": "\n", "r": "\r", "\\": "\\"}.get(n, n))
            i += 2
            continue
        out.append(c)
        i += 1
    return "".join(out)


def read_properties(path: str) -> Dict[str, str]:
    """java.util.Properties / commons-configuration text: ``key = value``, '#' comments, \\-escapes."""
    props = {}
    with open(path, encoding="latin-1") as f:
        for line in f:
            line = line.strip()
            if not line or line[0] in "#!":
                continue
            k, sep, v = line.partition("=")
            if not sep:
                continue
            props[k.strip()] = _unescape_java(v.strip())
    return props


def _columns(props):
    names = []
    for key in ("segment.dimension.column.names", "segment.metric.column.names", "segment.time.column.name",
                "segment.datetime.column.names", "segment.complex.column.names"):
        for c in props.get(key, "").split(","):
            c = c.strip()
            if c and c not in names and f"column.{c}.dataType" in props:
                names.append(c)
    return names


def _as_bool(v: str) -> bool:
    return str(v).strip().lower() == "true"


def read_segment_dir(path: str) -> ImmutableSegment:
    """ImmutableSegmentLoader.load (ImmutableSegmentLoader.java:155-190,222-280) for the hot path's indexes."""
    seg_dir = os.path.join(path, "v3") if os.path.isdir(os.path.join(path, "v3")) else path
    props = read_properties(os.path.join(seg_dir, "metadata.properties"))
    pad = props.get("segment.padding.character")
    pad = _unescape_java(pad) if pad is not None else None  # StringEscapeUtils.unescapeJava, as the reference
    if pad != "\0":
        raise ValueError(f"Got non-zero string padding: {pad!r}")  # ColumnMetadataImpl.java:250-253
    num_docs = int(props["segment.total.docs"])
    seg = ImmutableSegment(props.get("segment.name", os.path.basename(path.rstrip("/"))), num_docs)
    psf = os.path.join(seg_dir, "columns.psf")
    if os.path.exists(psf):
        imap = read_properties(os.path.join(seg_dir, "index_map"))
        with open(psf, "rb") as f:
            blob = f.read()

        def buf(col, kind):
            index = _INDEX_ID.get(kind, "forward_index")
            start = imap.get(f"{col}.{index}.startOffset")
            if start is None:
                return None
            start, size = int(start), int(imap[f"{col}.{index}.size"])
            if struct.unpack(">Q", blob[start:start + 8])[0] != MAGIC_MARKER:
                raise ValueError(f"missing magic marker for {col}.{index} at {start}")
            return blob[start + 8:start + size]
    else:
        def buf(col, kind):
            p = os.path.join(seg_dir, col + _EXT[kind])
            if not os.path.exists(p):
                return None
            with open(p, "rb") as f:
                return f.read()

    for col in _columns(props):
        key = f"column.{col}."
        dt = _TYPES[props[key + "dataType"].upper()]
        has_dict = _as_bool(props.get(key + "hasDictionary", "true"))
        is_sorted = _as_bool(props.get(key + "isSorted", "false"))
        card = int(props.get(key + "cardinality", "0"))
        bits = int(props.get(key + "bitsPerElement", "0"))
        width = int(props.get(key + "lengthOfEachEntry", "0")) if dt == DataType.STRING else 0
        if not _as_bool(props.get(key + "isSingleValues", "true")):
            raise NotImplementedError(f"multi-value column {col} is outside the hot path")
        if not has_dict:
            fwd = buf(col, "raw")
            meta = ColumnMetadata(col, dt, num_docs, 0, 0, False, False, False)
            seg.columns[col] = ColumnIndexes(meta, fwd, null_vector=buf(col, "nullvalue"))
            continue
        dictionary = buf(col, "dictionary")
        fwd = buf(col, "sorted") if is_sorted else buf(col, "unsorted")
        if fwd is None:  # a sorted column written as an unsorted forward index, or the reverse
            fwd = buf(col, "unsorted") if is_sorted else buf(col, "sorted")
        inv = buf(col, "inverted")
        meta = ColumnMetadata(col, dt, num_docs, card, bits, is_sorted, True, inv is not None, width)
        seg.columns[col] = ColumnIndexes(meta, fwd, dictionary, inv, buf(col, "nullvalue"))
    return seg


def write_segment_dir(seg: ImmutableSegment, path: str, version: int = 3) -> str:
    """The columns of ``seg`` as a Pinot segment directory (v1: one file per index; v3: columns.psf +
    index_map with magic markers), plus metadata.properties with the keys read_segment_dir uses."""
    seg_dir = os.path.join(path, "v3") if version == 3 else path
    os.makedirs(seg_dir, exist_ok=True)
    lines = [f"segment.name = {seg.name}", f"segment.total.docs = {seg.num_docs}",
             "segment.padding.character = \\\\u0000",  # as Pinot writes it: \\u0000
             "segment.dimension.column.names = " + ",".join(seg.columns)]
    psf, imap = bytearray(), []
    for col, ci in seg.columns.items():
        m = ci.metadata
        key = f"column.{col}."
        lines += [key + f"dataType = {m.data_type.name}", key + f"cardinality = {m.cardinality}",
                  key + f"bitsPerElement = {m.bits_per_element}", key + f"isSorted = {str(m.is_sorted).lower()}",
                  key + f"hasDictionary = {str(m.has_dictionary).lower()}", key + "isSingleValues = true",
                  key + f"hasInvertedIndex = {str(m.has_inverted_index).lower()}",
                  key + f"lengthOfEachEntry = {m.string_width}", key + f"totalDocs = {m.total_docs}"]
        parts = [("raw" if not m.has_dictionary else ("sorted" if m.is_sorted else "unsorted"), ci.forward)]
        if ci.dictionary is not None:
            parts.append(("dictionary", ci.dictionary))
        if ci.inverted is not None:
            parts.append(("inverted", ci.inverted))
        if ci.null_vector is not None:
            parts.append(("nullvalue", ci.null_vector))
        for kind, data in parts:
            if version == 3:
                index = _INDEX_ID.get(kind, "forward_index")
                imap.append(f"{col}.{index}.startOffset = {len(psf)}")
                imap.append(f"{col}.{index}.size = {len(data) + 8}")
                psf += struct.pack(">Q", MAGIC_MARKER) + data
            else:
                with open(os.path.join(seg_dir, col + _EXT[kind]), "wb") as f:
                    f.write(data)
    if version == 3:
        with open(os.path.join(seg_dir, "columns.psf"), "wb") as f:
            f.write(bytes(psf))
        with open(os.path.join(seg_dir, "index_map"), "w") as f:
            f.write("\n".join(imap) + "\n")
    with open(os.path.join(seg_dir, "metadata.properties"), "w") as f:
        f.write("\n".join(lines) + "\n")
    return path
