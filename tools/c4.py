"""Config C4: inverted-index-heavy workload.

Segments of 10M rows with five dictionary-encoded INT columns C1..C5, each with a bitmap inverted
index, cardinalities 10 / 100 / 1K / 10K / 100K, values uniform (seeded splitmix64, tools/bqgen.c),
plus a dictionary metric M (card 1000, no index). Dictionary ids equal the values (every value occurs).
The predicate template is

    C1 IN (S1) AND (C2 = v OR C3 IN (S3)) AND NOT C4 = w AND C5 BETWEEN lo AND hi

with the set sizes and the range chosen so the expected selectivity is the target (0.01 % .. 50 %).
As in the reference (FilterOperatorUtils.java:98-131), the IN / EQ / NOT leaves are served by the
inverted index (Roaring containers decoded on the GPU) and the RANGE leaf by a scan of the forward index.
"""
import numpy as np

from pinot_amd.segment.creator import (ColumnIndexes, ColumnMetadata, ImmutableSegment, inverted_index_bytes,
                                       pack_bits)
from pinot_amd.spi import DataType, num_bits_per_value

from . import bq

CARDS = {"C1": 10, "C2": 100, "C3": 1000, "C4": 10_000, "C5": 100_000, "M": 1000}
INVERTED = ("C1", "C2", "C3", "C4", "C5")
SELECTIVITIES = (0.0001, 0.001, 0.01, 0.1, 0.5)
# (|S1|, |S3|) per target; the C5 range closes the gap to the target
_SETS = {0.0001: (1, 1), 0.001: (1, 20), 0.01: (2, 100), 0.1: (5, 300), 0.5: (9, 700)}


def query(sel: float, agg: str = "COUNT(*)") -> str:
    s1, s3 = _SETS[sel]
    p1 = s1 / 10
    p23 = 1 - (1 - 1 / 100) * (1 - s3 / 1000)
    p4 = 1 - 1 / 10_000
    width = int(round(sel / (p1 * p23 * p4) * 100_000))
    width = max(1, min(100_000, width))
    lo = 1000
    hi = min(99_999, lo + width - 1)
    S1 = ", ".join(str(v) for v in range(s1))
    S3 = ", ".join(str(v) for v in range(s3))
    return (f"SELECT {agg} FROM c4 WHERE C1 IN ({S1}) AND (C2 = 7 OR C3 IN ({S3})) AND NOT C4 = 4242 "
            f"AND C5 BETWEEN {lo} AND {hi}")


def expected_selectivity(sel: float) -> float:
    s1, s3 = _SETS[sel]
    q = query(sel)
    lo, hi = [int(x) for x in q.split("BETWEEN ")[1].split(" AND ")]
    return (s1 / 10) * (1 - (1 - 1 / 100) * (1 - s3 / 1000)) * (1 - 1 / 10_000) * ((hi - lo + 1) / 100_000)


def make_segment(index: int, num_rows: int = 10_000_000, seed: int = 7) -> ImmutableSegment:
    L = bq.lib()
    seg = ImmutableSegment(f"c4_{index}", num_rows)
    for j, (name, card) in enumerate(CARDS.items()):
        ids = np.empty(num_rows, np.int32)
        L.c4_generate(seed * 1000 + j, index * num_rows, num_rows, card, ids.ctypes.data)
        bits = num_bits_per_value(card - 1)
        inv = inverted_index_bytes(ids, card) if name in INVERTED else None
        meta = ColumnMetadata(name, DataType.INT, num_rows, card, bits, False, True, inv is not None)
        seg.columns[name] = ColumnIndexes(meta, pack_bits(ids, bits), np.arange(card, dtype=">i4").tobytes(), inv)
    return seg
