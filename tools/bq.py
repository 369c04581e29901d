"""Config C1: pinot-perf BenchmarkQueries-style offline segments.

Schema and table config follow pinot-perf/src/main/java/org/apache/pinot/perf/BenchmarkQueries.java
(:81-117): SORTED_COL (sorted, numRows - i), INT_COL (dictionary + inverted index), NO_INDEX_INT_COL
(dictionary, no index), RAW_INT_COL (no dictionary: PASS_THROUGH raw chunks), LOW_CARDINALITY_STRING_COL
("value" + i % 10, inverted index). Values come from Distribution EXP(lambda) over java.util.Random(42)
(tools/bqgen.c restates both). RAW_STRING_COL / NO_INDEX_STRING_COL (random UUIDs) and TSTMP_COL are
not generated: no query of the GPU subset reads them. The reference table's star-tree (split order SORTED_COL,
INT_COL; SUM__RAW_INT_COL; maxLeafRecords Integer.MAX_VALUE, :99-104) is built with ``star_tree=True`` (the
STARTREE_* queries then take the star-tree path, as in the reference benchmark); the range index is not (an
alternative to the scan leaf with identical results).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libbqgen.so")
_lib = None

SCENARIOS = {"EXP(0.001)": 0.001, "EXP(0.5)": 0.5, "EXP(0.999)": 0.999}

# BenchmarkQueries' query constants that fall inside the GPU subset (same text; MyTable)
QUERIES = {
    "SUM_QUERY": "SELECT SUM(RAW_INT_COL) FROM MyTable",
    "FILTERED_QUERY": "SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 123 AND INT_COL < 599999),"
                      "MAX(INT_COL) FILTER(WHERE INT_COL > 123 AND INT_COL < 599999) "
                      "FROM MyTable WHERE NO_INDEX_INT_COL > 5 AND NO_INDEX_INT_COL < 1499999",
    "FILTERED_MIXED": "SELECT COUNT(*), SUM(RAW_INT_COL) FILTER(WHERE LOW_CARDINALITY_STRING_COL IN ('value1', 'value7')), "
                      "MIN(NO_INDEX_INT_COL) FILTER(WHERE INT_COL BETWEEN 10 AND 20), "
                      "COUNT(*) FILTER(WHERE INT_COL BETWEEN 10 AND 20) FROM MyTable WHERE NO_INDEX_INT_COL >= 3 OR INT_COL < 50",
    "RAW_COLUMN_SUMMARY_STATS": "SELECT MIN(RAW_INT_COL), MAX(RAW_INT_COL), COUNT(*) FROM MyTable",
    "FILTERED_SCAN_SUM": "SELECT SUM(INT_COL), MAX(INT_COL) FROM MyTable "
                         "WHERE NO_INDEX_INT_COL > 5 AND NO_INDEX_INT_COL < 1499999",
    "FILTERING_SCAN_QUERY": "SELECT SUM(RAW_INT_COL) FROM MyTable WHERE RAW_INT_COL BETWEEN 1 AND 10",
    "FILTERING_BITMAP_SCAN_COUNT": "SELECT COUNT(*) FROM MyTable WHERE INT_COL = 1 AND RAW_INT_COL IN (0, 1, 2)",
    "COUNT_RANGE_SCAN": "SELECT COUNT(*) FROM MyTable WHERE NO_INDEX_INT_COL BETWEEN 10 AND 2000",
    "COUNT_OVER_BITMAP_INDEX_IN": "SELECT COUNT(*) FROM MyTable WHERE INT_COL IN (0, 1, 2, 3, 4, 5, 7, 9, 10)",
    "COUNT_OVER_BITMAP_INDEX_EQUALS": "SELECT COUNT(*) FROM MyTable WHERE LOW_CARDINALITY_STRING_COL = 'value1'",
    "COUNT_OVER_BITMAP_INDEXES": "SELECT COUNT(*) FROM MyTable WHERE INT_COL IN (0, 1, 2, 3, 4, 5, 7, 9, 10) "
                                 "AND LOW_CARDINALITY_STRING_COL = 'value1' ",
    "COUNT_OVER_BITMAP_AND_SORTED_INDEXES": "SELECT COUNT(*) FROM MyTable WHERE INT_COL IN (0, 1, 2, 3, 4, 5, 7, 9, 10) "
                                            "AND LOW_CARDINALITY_STRING_COL = 'value1' "
                                            "AND SORTED_COL BETWEEN 10 and 50",
    "STARTREE_SUM_QUERY": "SELECT INT_COL, SORTED_COL, SUM(RAW_INT_COL) from MyTable "
                          "GROUP BY INT_COL, SORTED_COL ORDER BY SORTED_COL, INT_COL ASC",
    "STARTREE_FILTER_QUERY": "SELECT INT_COL, SORTED_COL, SUM(RAW_INT_COL) FROM MyTable "
                             "WHERE INT_COL = 0 and SORTED_COL = 1 "
                             "GROUP BY INT_COL, SORTED_COL ORDER BY SORTED_COL, INT_COL ASC",
    "GROUP_BY_LOW_CARD": "SELECT LOW_CARDINALITY_STRING_COL, COUNT(*), SUM(RAW_INT_COL), MAX(NO_INDEX_INT_COL) "
                         "FROM MyTable WHERE INT_COL < 600 GROUP BY LOW_CARDINALITY_STRING_COL",
}


def build():
    src = os.path.join(_HERE, "bqgen.c")
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-o", _SO, src, "-lm"])


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_SO)
        L.bq_seed_scramble.argtypes = [ctypes.c_int64]
        L.bq_seed_scramble.restype = ctypes.c_int64
        L.bq_generate.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_double, ctypes.c_int64,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.bq_generate.restype = None
        L.c4_generate.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
        L.c4_generate.restype = None
        L.bq_doubles.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        L.bq_doubles.restype = None
        _lib = L
    return _lib


def java_random_doubles(seed: int, n: int) -> np.ndarray:
    """First n java.util.Random(seed).nextDouble() values (known-answer check of the restated LCG)."""
    L = lib()
    out = np.empty(n, np.float64)
    L.bq_doubles(seed, n, out.ctypes.data)
    return out


def generate(num_rows: int, num_segments: int, scenario: str = "EXP(0.001)", seed: int = 42):
    """Column arrays of every segment, in build order (the supplier continues across segments)."""
    L = lib()
    lam = SCENARIOS[scenario]
    st = ctypes.c_int64(L.bq_seed_scramble(seed))
    out = []
    for _ in range(num_segments):
        a = np.empty(num_rows, np.int32)
        b = np.empty(num_rows, np.int32)
        c = np.empty(num_rows, np.int32)
        L.bq_generate(ctypes.byref(st), lam, num_rows, a.ctypes.data, b.ctypes.data, c.ctypes.data)
        out.append({"INT_COL": a, "NO_INDEX_INT_COL": b, "RAW_INT_COL": c})
    return out


def make_segments(num_rows: int, num_segments: int = 1, scenario: str = "EXP(0.001)", seed: int = 42,
                  star_tree: bool = False):
    from pinot_amd.segment.creator import SegmentCreator
    from pinot_amd.segment.startree import StarTreeIndexConfig
    from pinot_amd.spi import DataType
    st = [StarTreeIndexConfig(["SORTED_COL", "INT_COL"], ["SUM__RAW_INT_COL"], max_leaf_records=2 ** 31 - 1)] \
        if star_tree else []
    low = np.array([f"value{i}" for i in range(10)])
    segs = []
    for k, cols in enumerate(generate(num_rows, num_segments, scenario, seed)):
        c = SegmentCreator(f"testSegment{k}", inverted_index_columns=["INT_COL", "LOW_CARDINALITY_STRING_COL"],
                           no_dictionary_columns=["RAW_INT_COL"], star_tree_configs=st)
        c.add_column("SORTED_COL", DataType.INT, num_rows - np.arange(num_rows, dtype=np.int64))
        c.add_column("INT_COL", DataType.INT, cols["INT_COL"])
        c.add_column("NO_INDEX_INT_COL", DataType.INT, cols["NO_INDEX_INT_COL"])
        c.add_column("RAW_INT_COL", DataType.INT, cols["RAW_INT_COL"])
        c.add_column("LOW_CARDINALITY_STRING_COL", DataType.STRING, low[np.arange(num_rows) % 10])
        segs.append(c.build())
    return segs
