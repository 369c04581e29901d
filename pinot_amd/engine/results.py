"""Results blocks and execution statistics (the output contract of the hot path).

  AggregationResultsBlock  pinot-core/.../operator/blocks/results/AggregationResultsBlock.java:54-155
  GroupByResultsBlock      pinot-core/.../operator/blocks/results/GroupByResultsBlock.java:68-106
  SelectionResultsBlock    pinot-core/.../operator/blocks/results/SelectionResultsBlock.java (DataSchema + rows)
  ExecutionStatistics      pinot-core/.../operator/ExecutionStatistics.java:42-45

Intermediate results follow each function's intermediate type:
  count -> int, sum -> float (int when every input is INT/LONG: exact), min/max ->
  float, avg -> (sum, count), minmaxrange -> (min, max), distinctcounthll -> uint8 registers.
"""
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np


class JavaDoubleKey(float):
    """A FLOAT / DOUBLE group-key value that Python's float equality would merge with another: -0.0 (== 0.0 in
    Python) and NaN (!= itself). The reference keys raw real group values by their bits (Double2IntOpenHashMap /
    Float2IntOpenHashMap hash and compare doubleToLongBits / floatToIntBits, the Key's Double.equals in the
    IndexedTable), so -0.0 and 0.0 are two groups and every NaN is one; so do the device tables (keys.hip) and so
    does this wrapper: equal only to a -0.0 (resp. a NaN), hashed by the bits. Every other key stays a plain float."""
    __slots__ = ()

    def __eq__(self, o):
        if not isinstance(o, float):
            return NotImplemented
        x = float(o)  # (plain float comparisons: o may be a JavaDoubleKey too)
        if math.isnan(self):
            return math.isnan(x)
        return x == 0.0 and math.copysign(1.0, x) < 0

    def __ne__(self, o):
        r = self.__eq__(o)
        return r if r is NotImplemented else not r

    def __hash__(self):
        return hash(0x7FF8000000000000) if math.isnan(self) else hash(-0x8000000000000000)

    def __reduce__(self):
        return (JavaDoubleKey, (float(self),))


def java_double_key(x):
    """x as a group-key value with Java's Double.equals semantics (JavaDoubleKey for -0.0 and NaN)."""
    if isinstance(x, float) and (x != x or (x == 0.0 and math.copysign(1.0, x) < 0)):
        return JavaDoubleKey(x)
    return x


def key_column_list(col, key_type=None):
    """A key column (numpy array) as a list of group-key values: real columns (a float array, or an object array
    of floats and None null keys when `key_type` is FLOAT / DOUBLE) wrap their -0.0 / NaN entries."""
    out = col.tolist() if isinstance(col, np.ndarray) else list(col)
    if isinstance(col, np.ndarray) and col.dtype.kind == "f":
        odd = np.nonzero(np.isnan(col) | ((col == 0) & np.signbit(col)))[0]
        for i in odd.tolist():
            out[i] = JavaDoubleKey(out[i])
    elif key_type in ("FLOAT", "DOUBLE"):
        out = [java_double_key(v) for v in out]
    return out


@dataclass
class ExecutionStatistics:
    num_docs_scanned: int = 0
    num_entries_scanned_in_filter: int = 0
    num_entries_scanned_post_filter: int = 0
    num_total_docs: int = 0
    num_segments_processed: int = 0
    num_segments_matched: int = 0

    def merge(self, o: "ExecutionStatistics"):
        self.num_docs_scanned += o.num_docs_scanned
        self.num_entries_scanned_in_filter += o.num_entries_scanned_in_filter
        self.num_entries_scanned_post_filter += o.num_entries_scanned_post_filter
        self.num_total_docs += o.num_total_docs
        self.num_segments_processed += o.num_segments_processed
        self.num_segments_matched += o.num_segments_matched


@dataclass
class AggregationResultsBlock:
    aggregations: list                 # AggregationInfo per function
    results: List[object]              # intermediate result per function
    stats: ExecutionStatistics = field(default_factory=ExecutionStatistics)
    device_ms: float = 0.0
    scan_kernel_ms: float = 0.0


@dataclass
class GroupByResultsBlock:
    aggregations: list
    group_by: list                     # group-by expressions
    groups: Dict[Tuple, List[object]]  # key values tuple -> intermediates
    stats: ExecutionStatistics = field(default_factory=ExecutionStatistics)
    num_groups_limit_reached: bool = False
    device_ms: float = 0.0
    scan_kernel_ms: float = 0.0
    key_types: Optional[List[str]] = None  # stored types of the group-by columns (column metadata: INT / LONG / ...)

    def set_columns(self, key_columns, prim_columns, mapping):
        """A columnar block (the GPU decode): per group-by column an array of the groups' key values, per primitive
        (plan_aggregations) an array of the groups' values (HLL: [groups][registers] u8), and the functions' mapping
        onto primitives. `groups` -- the {key tuple: intermediates} view -- is built from them on first access."""
        self.__dict__.pop("groups", None)
        self.key_columns, self.prim_columns, self._mapping = key_columns, prim_columns, mapping

    @property
    def num_groups(self) -> int:
        if "groups" in self.__dict__ or not hasattr(self, "key_columns"):
            return len(self.groups)
        return len(self.key_columns[0]) if self.key_columns else (len(self.prim_columns[0]) if self.prim_columns else 0)

    def __getattr__(self, name):
        # (only reached when `groups` is not set: a columnar block builds its dict view once)
        if name != "groups" or "prim_columns" not in self.__dict__:
            raise AttributeError(name)
        prim = [[row.copy() for row in c] if c.ndim == 2 else c.tolist() for c in self.prim_columns]
        fcols = [list(zip(prim[sl[0]], prim[sl[1]])) if fn in ("avg", "minmaxrange") else prim[sl]
                 for fn, sl in self._mapping]
        kt = self.__dict__.get("key_types") or [None] * len(self.key_columns)
        cols = [key_column_list(c, t) for c, t in zip(self.key_columns, kt)]
        n = self.num_groups
        gkeys = list(zip(*cols)) if cols else [()] * n
        g = dict(zip(gkeys, map(list, zip(*fcols)))) if fcols else {k: [] for k in gkeys}
        self.groups = g
        return g


@dataclass
class SelectionResultsBlock:
    """Rows of a selection query: the DataSchema's column names are the select expressions' strings, its types the
    columns' stored types (DOUBLE for arithmetic, the transform functions' result type). The values are held
    column-wise (numpy arrays, or lists of str) -- a multi-stage leaf ships millions of rows -- and `rows` builds
    the row lists on demand."""
    column_names: List[str]
    column_types: List[str]
    columns: List[object]
    stats: ExecutionStatistics = field(default_factory=ExecutionStatistics)
    device_ms: float = 0.0
    scan_kernel_ms: float = 0.0

    @property
    def num_rows(self) -> int:
        return len(self.columns[0]) if self.columns else 0

    @property
    def rows(self) -> List[list]:
        cols = [c.tolist() if isinstance(c, np.ndarray) else list(c) for c in self.columns]
        return [list(r) for r in zip(*cols)] if cols else []


def merge_intermediate(function: str, a, b):
    """AggregationFunction.merge for the functions on the path. None is a null intermediate result (enableNullHandling:
    no non-null value aggregated); merging it keeps the other side (SumAggregationFunction.merge under null handling,
    :240-250, and the other nullable functions alike)."""
    if a is None:
        return b
    if b is None:
        return a
    if function == "count":
        return a + b
    if function == "sum":
        return a + b
    if function == "min":
        return min(a, b)
    if function == "max":
        return max(a, b)
    if function == "avg":
        return (a[0] + b[0], a[1] + b[1])
    if function == "minmaxrange":
        return (min(a[0], b[0]), max(a[1], b[1]))
    if function in ("distinctcounthll", "distinctcountrawhll"):
        return np.maximum(a, b)
    raise NotImplementedError(function)
