"""Segments built from the committed golden fixtures (tests/golden/)."""
import functools
import json
import os

import numpy as np

from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# BaseSingleValueQueriesTest.java:49-62 schema; inverted indexes at :87-91
SV_SCHEMA = [("column1", DataType.INT), ("column3", DataType.INT), ("column5", DataType.STRING),
             ("column6", DataType.INT), ("column7", DataType.INT), ("column9", DataType.INT),
             ("column11", DataType.STRING), ("column12", DataType.STRING), ("column17", DataType.INT),
             ("column18", DataType.INT), ("daysSinceEpoch", DataType.INT)]
SV_INVERTED = ["column6", "column7", "column11", "column17", "column18"]


@functools.lru_cache(maxsize=None)
def expected():
    with open(os.path.join(GOLDEN, "expected.json")) as f:
        return json.load(f)


@functools.lru_cache(maxsize=None)
def test_data_sv_segment():
    data = np.load(os.path.join(GOLDEN, "test_data_sv.npz"))
    c = SegmentCreator("testTable_126164076_167572854", inverted_index_columns=SV_INVERTED)
    for name, dt in SV_SCHEMA:
        c.add_column(name, dt, data[name])
    return c.build()


@functools.lru_cache(maxsize=None)
def fast_filtered_count_segment():
    # FastFilteredCountTest.java:104-114 (TEXT/JSON columns out of scope); inverted on class & sorted (:127-128)
    n, b = 1000, 8
    i = np.arange(n)
    c = SegmentCreator("testSegment", inverted_index_columns=["class", "sorted"])
    c.add_column("sorted", DataType.INT, i)
    c.add_column("class", DataType.INT, i % b)
    c.add_column("intRangeCol", DataType.INT, n - i)
    return c.build()


def segment_for(name):
    return {"test_data_sv": test_data_sv_segment, "fast_filtered_count": fast_filtered_count_segment}[name]()


def docset_segment(sets, num_docs):
    """One INT column per doc-id set: value 1 on the set's docs, 0 elsewhere (TestFilterOperator stand-in).
    Column s{k} has an inverted index, column t{k} is scanned."""
    c = SegmentCreator("docsets", inverted_index_columns=[f"s{k}" for k in range(len(sets))])
    for k, s in enumerate(sets):
        v = np.zeros(num_docs, dtype=np.int32)
        v[np.asarray(s, dtype=np.int64)] = 1
        c.add_column(f"s{k}", DataType.INT, v)
        c.add_column(f"t{k}", DataType.INT, v)
    return c.build()


def docset_filter(op, nsets, prefix):
    p = [f"{prefix}{k} = 1" for k in range(nsets)]
    if op == "AND":
        return " AND ".join(p)
    if op == "OR":
        return " OR ".join(p)
    if op == "AND(AND,x)":
        return f"({p[0]} AND {p[1]}) AND {p[2]}"
    if op == "OR(OR,x)":
        return f"({p[0]} OR {p[1]}) OR {p[2]}"
    raise ValueError(op)


def rows_match(actual, expected, rel=1e-9):
    if len(actual) != len(expected):
        return False
    for ra, re_ in zip(actual, expected):
        if len(ra) != len(re_):
            return False
        for a, e in zip(ra, re_):
            if isinstance(e, float) or isinstance(a, float):
                if not (a == e or abs(a - e) <= rel * max(abs(a), abs(e))):
                    return False
            elif a != e:
                return False
    return True
