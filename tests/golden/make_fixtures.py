"""Generate the committed golden fixtures from the reference's own test data.

Runs ONLY in the build container (needs /root/reference); its outputs are committed under
tests/golden/ so that nothing at test time (CPU or GPU box) reads the reference.

Inputs (reference test data, read as bytes, nothing executed):
  pinot-core/src/test/resources/data/test_data-sv.avro  (30,000 rows, Avro null codec)
    used by BaseSingleValueQueriesTest.java:75 ("data/test_data-sv.avro"), which selects the
    11 columns listed at BaseSingleValueQueriesTest.java:49-62.

Outputs:
  test_data_sv.npz   the 11 selected columns (int32 / unicode), no pickled objects
  expected.json      reference known answers transcribed from the reference tests (file:line)

The Avro container is decoded with a small reader written from the public Avro 1.x spec
(object container file: magic 'Obj\\x01', metadata map, 16-byte sync, blocks of
(count, size, data)); records are the union-of-null fields declared in the embedded schema.
"""
import json
import os
import sys

import numpy as np

REF = "/root/reference"
AVRO = os.path.join(REF, "pinot-core/src/test/resources/data/test_data-sv.avro")
HERE = os.path.dirname(os.path.abspath(__file__))

# BaseSingleValueQueriesTest.java:49-62 (name, Pinot data type)
SELECTED = [
    ("column1", "INT"), ("column3", "INT"), ("column5", "STRING"), ("column6", "INT"),
    ("column7", "INT"), ("column9", "INT"), ("column11", "STRING"), ("column12", "STRING"),
    ("column17", "INT"), ("column18", "INT"), ("daysSinceEpoch", "INT"),
]


class _Buf:
    def __init__(self, data):
        self.d = data
        self.p = 0

    def read(self, n):
        out = self.d[self.p:self.p + n]
        self.p += n
        return out

    def long(self):
        # zig-zag varint
        shift = 0
        acc = 0
        while True:
            b = self.d[self.p]
            self.p += 1
            acc |= (b & 0x7F) << shift
            if not b & 0x80:
                break
            shift += 7
        return (acc >> 1) ^ -(acc & 1)

    def bytes_(self):
        return self.read(self.long())


def read_avro(path):
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
            k = buf.bytes_().decode()
            meta[k] = buf.bytes_()
    codec = meta.get("avro.codec", b"null").decode()
    assert codec == "null", codec
    schema = json.loads(meta["avro.schema"])
    sync = buf.read(16)
    fields = []
    for fld in schema["fields"]:
        t = fld["type"]
        assert isinstance(t, list) and t[0] == "null", t
        fields.append((fld["name"], t[1]))
    rows = {name: [] for name, _ in fields}
    while buf.p < len(buf.d):
        count = buf.long()
        size = buf.long()
        end = buf.p + size
        for _ in range(count):
            for name, typ in fields:
                branch = buf.long()
                if branch == 0:
                    rows[name].append(None)
                elif typ == "int" or typ == "long":
                    rows[name].append(buf.long())
                elif typ == "string":
                    rows[name].append(buf.bytes_().decode("utf-8"))
                else:
                    raise ValueError(typ)
        assert buf.p == end
        assert buf.read(16) == sync
    return rows


def main():
    rows = read_avro(AVRO)
    n = len(rows["column1"])
    out = {}
    for name, typ in SELECTED:
        vals = rows[name]
        assert all(v is not None for v in vals), f"nulls in {name}"
        if typ == "INT":
            out[name] = np.asarray(vals, dtype=np.int32)
        else:
            out[name] = np.asarray(vals, dtype=np.str_)
    np.savez_compressed(os.path.join(HERE, "test_data_sv.npz"), **out)
    print("rows", n, {k: (v.dtype, len(np.unique(v))) for k, v in out.items()})




# ------------------------------------------------------------------------------------------------
# Known answers transcribed from the reference's tests (path, line). "rows" is the broker result
# table; "stats" = (numDocsScanned, numEntriesScannedPostFilter, numTotalDocs) as asserted by
# QueriesTestUtils.testInterSegmentsResult (numEntriesScannedInFilter is strategy dependent and
# excluded).
# ------------------------------------------------------------------------------------------------
AGG = "pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentAggregationSingleValueQueriesTest.java"
GBY = "pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentGroupBySingleValueQueriesTest.java"
FILTER = (" WHERE column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000 AND column5 = 'gFuH'"
          " AND (column6 < 500000000 OR column11 NOT IN ('t', 'P')) AND daysSinceEpoch = 126164076")
GB1 = " GROUP BY column9 ORDER BY v1 DESC, v2 DESC LIMIT 1"


def _agg_cases():
    c = []
    q = "SELECT COUNT(*) FROM testTable"
    c += [(f"{AGG}:52", q, [[120000]], (120000, 0, 120000)),
          (f"{AGG}:57", q + FILTER, [[24516]], (24516, 0, 120000)),
          (f"{AGG}:62", q + " GROUP BY column9 ORDER BY COUNT(*) DESC LIMIT 1", [[64420]], (120000, 120000, 120000)),
          (f"{AGG}:66", q + FILTER + " GROUP BY column9 ORDER BY COUNT(*) DESC LIMIT 1", [[17080]], (24516, 24516, 120000))]
    for fn, ln, rows in (
            ("MAX", (101, 106, 111, 116), ([2146952047.0, 2147419555.0], [2146952047.0, 999813884.0],
                                           [2146952047.0, 2146630496.0], [2146952047.0, 999813884.0])),
            ("MIN", (130, 135, 141, 146), ([240528.0, 17891.0], [101116473.0, 20396372.0], [240528.0, 17891.0],
                                           [101116473.0, 91804599.0])),
            ("SUM", (158, 163, 168, 173), ([129268741751388.0, 129156636756600.0], [27503790384288.0, 12429178874916.0],
                                           [69526727335224.0, 69225631719808.0], [19058003631876.0, 8606725456500.0])),
            ("AVG", (185, 190, 196, 201), ([1077239514.5949, 1076305306.305], [1121871038.68037, 506982332.96280],
                                           [2142595699.0, 334963174.0], [2142595699.0, 334963174.0])),
            ("MINMAXRANGE", (215, 220, 225, 230), ([2146711519.0, 2147401664.0], [2045835574.0, 979417512.0],
                                                   [2146711519.0, 2146612605.0], [2044094181.0, 979417512.0])),
            ("DISTINCTCOUNTHLL", (270, 274, 278, 282), ([5977, 23825], [1886, 4492], [3592, 11889], [1324, 3197])),
            ("DISTINCTCOUNTRAWHLL", (324, 329, 334, 339), ([5977, 23825], [1886, 4492], [3592, 11889], [1324, 3197])),
    ):
        q = f"SELECT {fn}(column1) AS v1, {fn}(column3) AS v2 FROM testTable"
        nonscan = fn in ("MAX", "MIN", "MINMAXRANGE", "DISTINCTCOUNTHLL", "DISTINCTCOUNTRAWHLL")
        gb = GB1 if fn not in ("MIN",) else " GROUP BY column9 ORDER BY v1, v2 LIMIT 1"
        c += [(f"{AGG}:{ln[0]}", q, [rows[0]], (120000, 0 if nonscan else 240000, 120000)),
              (f"{AGG}:{ln[1]}", q + FILTER, [rows[1]], (24516, 49032, 120000)),
              (f"{AGG}:{ln[2]}", q + gb, [rows[2]], (120000, 360000, 120000)),
              (f"{AGG}:{ln[3]}", q + FILTER + gb, [rows[3]], (24516, 73548, 120000))]
    return c


def _gby_cases():
    s11 = [["", 5935285005452.0], ["P", 88832999206836.0], ["gFuH", 63202785888.0], ["o", 18105331533948.0],
           ["t", 16331923219264.0]]
    two = [["", "HEuxNvH", 3789390396216.0], ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0],
           ["", "MaztCmmxxgguBUxPti", 1333941430664.0], ["", "dJWwFk", 55470665124.0],
           ["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["P", "HEuxNvH", 21998672845052.0],
           ["P", "KrNxpdycSiwoRohEiTIlLqDHnx", 18069909216728.0], ["P", "MaztCmmxxgguBUxPti", 27177029040008.0],
           ["P", "TTltMtFiRqUjvOG", 4462670055540.0], ["P", "XcBNHe", 120021767504.0]]
    two15 = two + [["P", "dJWwFk", 6224665921376.0], ["P", "fykKFqiw", 1574451324140.0], ["P", "gFuH", 860077643636.0],
                   ["P", "oZgnrlDEtjjVpUoFLol", 8345501392852.0], ["gFuH", "HEuxNvH", 29872400856.0]]
    c = [
        (f"{GBY}:66", "SELECT column11, SUM(column1) FROM testTable GROUP BY column11 ORDER BY column11", s11, 240000),
        (f"{GBY}:74", "SELECT column11, sum(column1) FROM testTable GROUP BY column11 ORDER BY column11 DESC",
         list(reversed(s11)), 240000),
        (f"{GBY}:80", "SELECT column11, Sum(column1) FROM testTable GROUP BY column11 ORDER BY column11 LIMIT 3",
         s11[:3], 240000),
        (f"{GBY}:87", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
                      "ORDER BY column11, column12", two, 360000),
        (f"{GBY}:102", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
                       "ORDER BY column11, column12 LIMIT 15", two15, 360000),
        (f"{GBY}:135", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
                       "ORDER BY SUM(column1) DESC LIMIT 3",
         [["P", "MaztCmmxxgguBUxPti", 27177029040008.0], ["P", "HEuxNvH", 21998672845052.0],
          ["P", "KrNxpdycSiwoRohEiTIlLqDHnx", 18069909216728.0]], 360000),
        (f"{GBY}:160", "SELECT sum(column1), MIN(column6) FROM testTable GROUP BY column11 ORDER BY column11",
         [[5935285005452.0, 2.96467636E8], [88832999206836.0, 1689277.0], [63202785888.0, 2.96467636E8],
          [18105331533948.0, 2.96467636E8], [16331923219264.0, 1980174.0]], 360000),
        (f"{GBY}:206", "SELECT column12, MIN(column6) FROM testTable GROUP BY column12 "
                       "ORDER BY Min(column6) DESC, SUM(column1) LIMIT 3",
         [["XcBNHe", 329467557.0], ["gFuH", 296467636.0], ["fykKFqiw", 296467636.0]], 360000),
        (f"{GBY}:215", "select column17, count(*) from testTable group by column17 order by column17 limit 15",
         [[83386499, 2924], [217787432, 3892], [227908817, 6564], [402773817, 7304], [423049234, 6556],
          [561673250, 7420], [635942547, 3308], [638936844, 3816], [939479517, 3116], [984091268, 3824],
          [1230252339, 5620], [1284373442, 7428], [1555255521, 2900], [1618904660, 2744], [1670085862, 3388]],
         120000),
        (f"{GBY}:244", "SELECT column11, AVG(column6) FROM testTable GROUP BY column11  ORDER BY column11",
         [["", 296467636.0], ["P", 909380310.3521485], ["gFuH", 296467636.0], ["o", 296467636.0],
          ["t", 526245333.3900426]], 240000),
    ]
    return [(ref, q, rows, (120000, post, 120000)) for ref, q, rows, post in c]


FFC = "pinot-core/src/test/java/org/apache/pinot/queries/FastFilteredCountTest.java"


def _fast_count_cases():
    # FastFilteredCountTest.java:104-114 data (1000 records) and :146-310 cases (TEXT/JSON cases are out of scope)
    n, b = 1000, 8
    bc, bcc, lo, hi = n // b, n - n // b, 20, n - 20
    allb = "(" + ", ".join(str(i) for i in range(b)) + ")"
    two = "(0, 7)"
    T = "testTable"
    cases = [
        ("select count(*) from " + T, n),
        (f"select count(*) from {T} where class = 1", bc),
        (f"select count(*) from {T} where sorted = 1", 1),
        (f"select count(*) from {T} where sorted between {lo} and {hi}", hi - lo + 1),
        (f"select count(*) from {T} where sorted not between {lo} and {hi}", n - (hi - lo + 1)),
        (f"select count(*) from {T} where sorted in {allb}", b),
        (f"select count(*) from {T} where sorted in {allb} and class in {allb}", b),
        (f"select count(*) from {T} where class <> 1", bcc),
        (f"select count(*) from {T} where class in {two}", 2 * bc),
        (f"select count(*) from {T} where class not in {two}", n - 2 * bc),
        (f"select count(*) from {T} where class in {two} and sorted < {n // 2}", bc),
        (f"select count(*) from {T} where sorted = 1 and class = 1", 1),
        (f"select count(*) from {T} where sorted = 1 and class <> 1", 0),
        (f"select count(*) from {T} where sorted = 1 and class <> 0", 1),
        (f"select count(*) from {T} where sorted <> 1 and class = 1", bc - 1),
        (f"select count(*) from {T} where sorted >= 0 and class = 1", bc),
        (f"select count(*) from {T} where sorted > 1 and class = 1", bc - 1),
        (f"select count(*) from {T} where sorted >= 0 and class <> 1", bcc),
        (f"select count(*) from {T} where sorted >= 0 or class <> 0", n),
        (f"select count(*) from {T} where sorted < {bc} and class <> 0", bc - bc // b - 1),
        (f"select count(*) from {T} where sorted >= {bc} and class <> 0", bcc - bcc // b),
        (f"select count(*) from {T} where sorted < {b - 1} and class = {b - 1}", 0),
        (f"select count(*) from {T} where sorted >= {b - 2} and class = {b - 2}", bc),
        (f"select count(*) from {T} where sorted >= {lo} and sorted < {hi} and class = 0", bc - (lo + n - hi) // b),
        (f"select count(*) from {T} where intRangeCol >= {lo} and intRangeCol < {hi}", hi - lo),
        (f"select count(*) from {T} where intRangeCol < {hi}", hi - 1),
        (f"select count(*) from {T} where intRangeCol not between {lo} and {hi}", n - hi + lo - 1),
        (f"select count(*) from {T} where intRangeCol between {lo} and {hi} and class = 0", bc - (lo + n - hi) // b),
        (f"select count(*) from {T} where intRangeCol not between {lo} and {hi} and class = 0", (lo + n - hi) // b),
    ]
    return [(f"{FFC}:146-310", q, [[v]], None) for q, v in cases]


SEL = "pinot-core/src/test/java/org/apache/pinot/queries/InnerSegmentSelectionSingleValueQueriesTest.java"


def _selection_cases():
    """Selection-only known answers over the ONE test_data-sv segment of the inner-segment tests: row count, the
    first row's asserted columns, the schema's size and asserted types, (numDocsScanned,
    numEntriesScannedPostFilter). numEntriesScannedInFilter depends on the lazy scan stopping at LIMIT (48204 at
    :148) and is excluded."""
    star, sel = "SELECT * FROM testTable", "SELECT column1, column5, column11 FROM testTable"
    types = {"column1": "INT", "column11": "STRING"}
    return [
        {"ref": f"{SEL}:47-66", "query": star + " LIMIT 0", "num_rows": 0, "first": {}, "schema_size": 11,
         "types": types, "stats": [0, 0]},
        {"ref": f"{SEL}:68-83", "query": star + FILTER + " LIMIT 0", "num_rows": 0, "first": {}, "schema_size": 11,
         "types": types, "stats": [0, 0]},
        {"ref": f"{SEL}:119-141", "query": star, "num_rows": 10, "first": {"column1": 1578964907, "column11": "P"},
         "schema_size": 11, "types": types, "stats": [10, 110]},
        {"ref": f"{SEL}:143-164", "query": star + FILTER, "num_rows": 10,
         "first": {"column1": 351823652, "column11": "t"}, "schema_size": 11, "types": types, "stats": [10, 110]},
        {"ref": f"{SEL}:168-190", "query": sel, "num_rows": 10, "first": {"column1": 1578964907, "column11": "P"},
         "schema_size": 3, "types": types, "stats": [10, 30]},
        {"ref": f"{SEL}:192-212", "query": sel + FILTER, "num_rows": 10,
         "first": {"column1": 351823652, "column11": "t"}, "schema_size": 3, "types": types, "stats": [10, 30]},
    ]


DOCSETS = "pinot-core/src/test/java/org/apache/pinot/core/operator/filter/"


def _docset_cases():
    a = [2, 3, 10, 15, 16, 28]
    b = [3, 6, 8, 20, 28]
    a3 = [2, 3, 6, 10, 15, 16, 28]
    c3 = [1, 2, 3, 6, 30]
    return [
        {"ref": DOCSETS + "AndFilterOperatorTest.java:34-49", "num_docs": 40, "op": "AND", "sets": [a, b],
         "expected": [3, 28]},
        {"ref": DOCSETS + "AndFilterOperatorTest.java:52-69", "num_docs": 40, "op": "AND", "sets": [a3, b, c3],
         "expected": [3, 6]},
        {"ref": DOCSETS + "AndFilterOperatorTest.java:72-93", "num_docs": 40, "op": "AND(AND,x)",
         "sets": [a3, b, c3], "expected": [3, 6]},
        {"ref": DOCSETS + "OrFilterOperatorTest.java:37-57", "num_docs": 40, "op": "OR", "sets": [a, b],
         "expected": sorted(set(a) | set(b))},
        {"ref": DOCSETS + "OrFilterOperatorTest.java:59-82", "num_docs": 40, "op": "OR", "sets": [a3, b, c3],
         "expected": sorted(set(a3) | set(b) | set(c3))},
        {"ref": DOCSETS + "OrFilterOperatorTest.java:84-111", "num_docs": 40, "op": "OR(OR,x)", "sets": [a3, b, c3],
         "expected": sorted(set(a3) | set(b) | set(c3))},
        {"ref": DOCSETS + "OrFilterOperatorTest.java:129-143", "num_docs": 10, "op": "OR", "sets": [[1, 2, 3], [0, 1, 2]],
         "expected": [0, 1, 2, 3]},
    ]


def write_expected():
    cases = []
    for ref, q, rows, stats in _agg_cases() + _gby_cases():
        cases.append({"ref": ref, "data": "test_data_sv", "query": q, "rows": rows, "stats": stats})
    for ref, q, rows, stats in _fast_count_cases():
        cases.append({"ref": ref, "data": "fast_filtered_count", "query": q, "rows": rows, "stats": stats})
    out = {"queries": cases, "docsets": _docset_cases(), "selections": _selection_cases(),
           "note": "known answers transcribed from the reference's tests; see make_fixtures.py"}
    with open(os.path.join(HERE, "expected.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(cases), "query cases")


if __name__ == "__main__":
    if os.path.exists(AVRO):
        main()
    write_expected()
