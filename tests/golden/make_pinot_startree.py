"""Copies the Pinot-WRITTEN star-tree the reference keeps as test data, and the raw rows it was built from, into
tests/golden/pinot_startree/.

Run in the build container (the reference is not on the GPU box); the outputs are committed data files:
  star_tree_index, star_tree_index_map, metadata.properties
      pinot-segment-local/src/test/resources/data/startree/segment/ -- an OffHeapStarTree (magic
      0xBADDA55B00DAD00D, OffHeapStarTree.java:38-79) over AirlineID / Origin / Dest with count__* and
      max__ArrDelay, 1004 star-tree docs, maxLeafRecords 10 (metadata.properties startree.v2.0.*), used by the
      reference's StarTreeIndexSeparatorTest.java:43. The segment's columns.psf is not in the reference, so its
      dictionaries are rebuilt from the raw rows below.
  airline_2014_01_15.npz
      AirlineID / Origin / Dest / ArrDelay of pinot-tools/src/main/resources/examples/batch/airlineStats/rawdata/
      2014/01/15/airlineStats_data_2014-01-15.avro, the day of that segment (airlineStats_OFFLINE_16085_16085_0:
      DaysSinceEpoch 16085 = 2014-01-15, segment.total.docs = 313). A null ArrDelay is stored as the INT
      dimension default null value Integer.MIN_VALUE (FieldSpec.DEFAULT_DIMENSION_NULL_VALUE_OF_INT; the
      segment's column.ArrDelay.minValue = -2147483648 records it).
"""
import json
import os
import shutil

import numpy as np

SRC = "/root/reference/pinot-segment-local/src/test/resources/data/startree/segment"
AVRO = ("/root/reference/pinot-tools/src/main/resources/examples/batch/airlineStats/rawdata/2014/01/15/"
        "airlineStats_data_2014-01-15.avro")
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pinot_startree")
INT_MIN = -2 ** 31


class _Buf:
    def __init__(self, data):
        self.d = data
        self.p = 0

    def read(self, n):
        out = self.d[self.p:self.p + n]
        self.p += n
        return out

    def long(self):  # zig-zag varint
        shift = acc = 0
        while True:
            b = self.d[self.p]
            self.p += 1
            acc |= (b & 0x7F) << shift
            if not b & 0x80:
                break
            shift += 7
        return (acc >> 1) ^ -(acc & 1)


def _value(buf, t):
    """One Avro value of schema type t (the subset this file uses: unions, int/long, string, arrays)."""
    if isinstance(t, list):
        return _value(buf, t[buf.long()])
    if isinstance(t, dict):
        assert t["type"] == "array", t
        out = []
        while True:
            n = buf.long()
            if n == 0:
                return out
            if n < 0:
                n = -n
                buf.long()
            out.extend(_value(buf, t["items"]) for _ in range(n))
    if t in ("int", "long"):
        return buf.long()
    if t == "string":
        return buf.read(buf.long()).decode("utf-8")
    if t == "null":
        return None
    raise ValueError(t)


def read_avro(path, want):
    with open(path, "rb") as f:
        buf = _Buf(f.read())
    assert buf.read(4) == b"Obj\x01"
    meta = {}
    while True:
        n = buf.long()
        if n == 0:
            break
        if n < 0:
            n = -n
            buf.long()
        for _ in range(n):
            k = buf.read(buf.long()).decode()
            meta[k] = buf.read(buf.long())
    assert meta.get("avro.codec", b"null") == b"null"
    schema = json.loads(meta["avro.schema"])
    sync = buf.read(16)
    rows = {w: [] for w in want}
    while buf.p < len(buf.d):
        count, size = buf.long(), buf.long()
        end = buf.p + size
        for _ in range(count):
            for fld in schema["fields"]:
                v = _value(buf, fld["type"])
                if fld["name"] in rows:
                    rows[fld["name"]].append(v)
        assert buf.p == end
        assert buf.read(16) == sync
    return rows


def main():
    os.makedirs(DST, exist_ok=True)
    for name in ("star_tree_index", "star_tree_index_map", "metadata.properties"):
        shutil.copyfile(os.path.join(SRC, name), os.path.join(DST, name))
    rows = read_avro(AVRO, ("DaysSinceEpoch", "AirlineID", "Origin", "Dest", "ArrDelay"))
    assert set(rows["DaysSinceEpoch"]) == {16085}, set(rows["DaysSinceEpoch"])
    np.savez_compressed(os.path.join(DST, "airline_2014_01_15.npz"),
                        AirlineID=np.array(rows["AirlineID"], np.int32),
                        Origin=np.array(rows["Origin"]), Dest=np.array(rows["Dest"]),
                        ArrDelay=np.array([INT_MIN if v is None else v for v in rows["ArrDelay"]], np.int32))
    print(len(rows["AirlineID"]), "rows")


if __name__ == "__main__":
    main()
