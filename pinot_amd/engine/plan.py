"""GPU plan maker and operators (host mirror of the reference's operator surface).

  GpuInstancePlanMaker   InstancePlanMakerImplV2 (pinot-core/.../plan/maker/InstancePlanMakerImplV2.java:172-308)
                         selected when the query option ``useGpu`` is set; builds ONE combine-level
                         GPU operator over all segments instead of per-segment plan nodes.
  filter compilation     FilterPlanNode.constructPhysicalOperator (pinot-core/.../plan/FilterPlanNode.java:195-320):
                         per segment, constant-folds always-true/false predicates, then picks the leaf
                         like FilterOperatorUtils.DefaultImplementation (…/operator/filter/FilterOperatorUtils.java:98-131):
                         sorted index > inverted index > scan.
  GpuCombineOperator     replaces AggregationOperator / GroupByOperator per segment plus the
                         CombineOperator merge (…/operator/combine/BaseSingleBlockCombineOperator.java:58-162)
                         with one phip_query call.
"""
import contextvars
import ctypes
import dataclasses
import math
import os
import re
import struct
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Union

import numpy as np

from .. import _lib
from ..query import predicate as predeval
from ..query.context import (UNBOUNDED, AggregationInfo, FilterContext, Function, Identifier, Literal, Predicate,
                             QueryContext, columns_of)
from ..query.sql import parse
from ..spi import (DEFAULT_GROUPBY_TRIM_THRESHOLD, DEFAULT_MIN_SEGMENT_GROUP_TRIM_SIZE,
                   DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE, DEFAULT_NUM_GROUPS_LIMIT, MAX_TRIM_THRESHOLD, DataType)
from .results import (AggregationResultsBlock, ExecutionStatistics, GroupByResultsBlock, SelectionResultsBlock,
                      merge_intermediate)
from .segment import GpuSegment


from .._lib import QueryCancelledError, QueryTimeoutError, UnsupportedOnGpu  # noqa: E402,F401 (re-exported)


# ------------------------------------------------------------------------------ filter trees
@dataclass
class _Leaf:
    kind: int
    column: Optional[str] = None
    lo: int = 0
    hi: int = 0
    exclusive: bool = False
    ids: Optional[np.ndarray] = None  # int32


@dataclass
class _Node:
    op: int
    children: list = field(default_factory=list)


_TRUE = _Leaf(_lib.LEAF_MATCH_ALL)
_FALSE = _Leaf(_lib.LEAF_MATCH_NONE)


def _is_const(n, which):
    return isinstance(n, _Leaf) and n.kind == which.kind and n.column is None


def _doc_ranges_for(seg: GpuSegment, column: str, ev: predeval.DictPredicateEvaluation) -> np.ndarray:
    """Sorted column: matching dict ids -> merged inclusive doc ranges (SortedIndexBasedFilterOperator.java:52-132)."""
    card = seg.column_metadata(column).cardinality
    ids = ev.matching_dict_ids(card)
    ranges = []
    for d in ids:
        s, e = seg.sorted_doc_range(column, d)
        if ranges and ranges[-1][1] + 1 == s:
            ranges[-1][1] = e
        else:
            ranges.append([s, e])
    return np.asarray(ranges, dtype=np.int32).reshape(-1)


RAW_SET_MAX = 1 << 20  # values of a raw IN list (the descriptor blob carries them)


def _raw_string_predicate(column, pred):
    """Value-based leaf on a raw STRING column (RangePredicateEvaluatorFactory's StringRawValueBasedRange-
    PredicateEvaluator: String.compareTo against the bounds; the raw EQ / IN evaluators: equality). Literals become
    their string form; the payload layouts are pinot_hip.h's RAW_STRING_RANGE / RAW_STRING_SET (the library sorts
    and deduplicates the set)."""
    def words(b: bytes) -> np.ndarray:
        return np.frombuffer(b + b"\0" * (-len(b) % 4), dtype=np.int32).copy()

    if pred.type == "RANGE":
        lo = None if pred.lower == UNBOUNDED else str(pred.lower).encode("utf-8")
        hi = None if pred.upper == UNBOUNDED else str(pred.upper).encode("utf-8")
        head = np.array([-1 if lo is None else len(lo), -1 if hi is None else len(hi),
                         int(bool(pred.lower_inclusive)), int(bool(pred.upper_inclusive))], dtype=np.int32)
        return _Leaf(_lib.LEAF_RAW_STRING_RANGE, column, ids=np.concatenate([head, words((lo or b"") + (hi or b""))]))
    exclusive = pred.type in ("NOT_EQ", "NOT_IN")
    vals = sorted({str(v).encode("utf-8") for v in pred.values})
    if len(vals) > RAW_SET_MAX:
        raise UnsupportedOnGpu(f"raw IN list longer than {RAW_SET_MAX} values")
    if not vals:
        return _TRUE if exclusive else _FALSE
    offs = np.zeros(len(vals) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(v) for v in vals])
    if offs[-1] >= 1 << 31:
        raise UnsupportedOnGpu("raw STRING IN list over 2 GiB")
    head = np.concatenate([[len(vals)], offs]).astype(np.int32)
    return _Leaf(_lib.LEAF_RAW_STRING_SET, column, exclusive=exclusive, ids=np.concatenate([head, words(b"".join(vals))]))


def _raw_predicate(column, dt: DataType, pred):
    """Value-based leaf on a raw column (RawValueBasedPredicateEvaluatorFactory + ScanBasedFilterOperator):
    literals converted to the column type first (FLOAT literals rounded to float32, as Float.parseFloat);
    integral ranges folded to closed integer intervals."""
    if dt == DataType.STRING:
        return _raw_string_predicate(column, pred)
    real = dt in (DataType.FLOAT, DataType.DOUBLE)

    def conv(v):
        x = float(v)
        return float(np.float32(x)) if dt == DataType.FLOAT else x

    if pred.type == "RANGE":
        rr = _lib.RawRange()
        rr.lo_int, rr.hi_int = -(1 << 63), (1 << 63) - 1
        rr.lo_real, rr.hi_real = -math.inf, math.inf
        rr.lo_inclusive = rr.hi_inclusive = 1
        if pred.lower != UNBOUNDED:
            x = conv(pred.lower)
            if real:
                rr.lo_real, rr.lo_inclusive = x, int(pred.lower_inclusive)
            else:
                v = pred.lower
                lo = (math.ceil(x) if pred.lower_inclusive else math.floor(x) + 1) if not isinstance(v, int) else \
                    (v if pred.lower_inclusive else v + 1)
                rr.lo_int = max(lo, -(1 << 63))
        if pred.upper != UNBOUNDED:
            x = conv(pred.upper)
            if real:
                rr.hi_real, rr.hi_inclusive = x, int(pred.upper_inclusive)
            else:
                v = pred.upper
                hi = (math.floor(x) if pred.upper_inclusive else math.ceil(x) - 1) if not isinstance(v, int) else \
                    (v if pred.upper_inclusive else v - 1)
                rr.hi_int = min(hi, (1 << 63) - 1)
        if not real and rr.lo_int > rr.hi_int:
            return _FALSE
        words = np.frombuffer(bytes(rr), dtype=np.int32).copy()
        return _Leaf(_lib.LEAF_RAW_RANGE, column, ids=words)
    exclusive = pred.type in ("NOT_EQ", "NOT_IN")
    vals = []
    for v in pred.values:
        x = conv(v)
        if real:
            vals.append(x)
        elif float(x).is_integer():
            vals.append(int(v) if isinstance(v, int) else int(x))
    # the device binary-searches the list: sorted, distinct, no NaN (IEEE equality never matches it)
    arr = np.unique(np.asarray(vals, dtype=np.float64 if real else np.int64))
    if real:
        arr = arr[~np.isnan(arr)]
    if len(arr) > RAW_SET_MAX:
        raise UnsupportedOnGpu(f"raw IN list longer than {RAW_SET_MAX} values")
    if not len(arr):
        return _TRUE if exclusive else _FALSE
    return _Leaf(_lib.LEAF_RAW_SET, column, exclusive=exclusive, ids=arr.view(np.int32).copy())


INVERTED_COST_RATIO = 0.5  # decode bytes allowed per forward-index byte (measured: tools/configs_bench.py C4)


def _null_leaf(seg: GpuSegment, column: str, exclusive: bool = False):
    """IS NULL (exclusive: IS NOT NULL) over the column's null value vector: BitmapBasedFilterOperator on
    NullValueVectorReader.getNullBitmap(), or EmptyFilterOperator / MatchAllFilterOperator for a column without one
    (FilterPlanNode.java:294-307)."""
    if seg.has_null_vector(column):
        return _Leaf(_lib.LEAF_NULL, column, exclusive=exclusive)
    return _TRUE if exclusive else _FALSE


def compile_predicate(seg: GpuSegment, pred) -> object:
    column = pred.column
    if pred.type in ("IS_NULL", "IS_NOT_NULL"):
        return _null_leaf(seg, column, pred.type == "IS_NOT_NULL")
    m = seg.column_metadata(column)
    if not m.has_dictionary:
        return _raw_predicate(column, m.data_type, pred)
    ev = predeval.evaluate(pred, seg.dictionary(column))
    if ev.always_false:
        return _FALSE
    if ev.always_true:
        return _TRUE
    if m.is_sorted:
        return _Leaf(_lib.LEAF_DOC_RANGES, column, ids=_doc_ranges_for(seg, column, ev))
    if m.has_inverted_index and pred.type != "RANGE":
        # FilterOperatorUtils picks the inverted index for EQ / IN / NOT_EQ / NOT_IN (:118-131). The GPU
        # planner keeps that choice unless decoding the selected bitmaps would move more bytes than
        # streaming the forward index (inverted_cost_ratio x forward bytes): a scan leaf of the same
        # dict ids gives the identical doc set. PINOT_AMD_INVERTED=always restores the reference choice.
        ids = (np.arange(ev.start, ev.end, dtype=np.int32) if ev.kind == "range"
               else np.asarray(ev.ids, dtype=np.int32))
        fwd = (seg.num_docs * m.bits_per_element + 7) // 8
        inv_ok = os.environ.get("PINOT_AMD_INVERTED", "") == "always"
        if not inv_ok:
            ratio = float(os.environ.get("PINOT_AMD_INVERTED_RATIO", INVERTED_COST_RATIO))  # (measurement override)
            inv_ok = seg.inverted_bytes(column, ids) <= ratio * fwd
        if inv_ok:
            if ev.kind == "range":
                return _Leaf(_lib.LEAF_INVERTED, column, ids=ids)
            return _Leaf(_lib.LEAF_INVERTED, column, exclusive=ev.exclusive, ids=ids)
    if ev.kind == "range":
        return _Leaf(_lib.LEAF_DICT_RANGE, column, lo=ev.start, hi=ev.end)
    return _Leaf(_lib.LEAF_DICT_SET, column, exclusive=ev.exclusive, ids=np.asarray(ev.ids, dtype=np.int32))


def _fold_and(kids):
    if any(_is_const(k, _FALSE) for k in kids):
        return _FALSE
    kids = [k for k in kids if not _is_const(k, _TRUE)]
    if not kids:
        return _TRUE
    return kids[0] if len(kids) == 1 else _Node(_lib.NODE_AND, kids)


def _fold_or(kids):
    if any(_is_const(k, _TRUE) for k in kids):
        return _TRUE
    kids = [k for k in kids if not _is_const(k, _FALSE)]
    if not kids:
        return _FALSE
    return kids[0] if len(kids) == 1 else _Node(_lib.NODE_OR, kids)


def _fold_not(k):
    if _is_const(k, _TRUE):
        return _FALSE
    if _is_const(k, _FALSE):
        return _TRUE
    if isinstance(k, _Leaf) and k.kind in (_lib.LEAF_DICT_SET, _lib.LEAF_INVERTED, _lib.LEAF_RAW_SET, _lib.LEAF_NULL):
        return _Leaf(k.kind, k.column, k.lo, k.hi, not k.exclusive, k.ids)
    return _Node(_lib.NODE_NOT, [k])


def _three_valued(seg: GpuSegment, fc: FilterContext):
    """(trues, falses, nulls) trees of a filter under enableNullHandling (nulls None = EmptyDocIdSet):
      column leaf      BaseColumnFilterOperator: trues = p AND NOT null(c), nulls = null(c), falses = NOT(trues OR
                       nulls) = NOT p AND NOT null(c) (BaseColumnFilterOperator.java:45-80, BaseFilterOperator.java:
                       104-122); an always-true predicate is BitmapBasedFilterOperator(null bitmap, exclusive), an
                       always-false one EmptyFilterOperator (FilterOperatorUtils.java:75-88): no nulls of their own
      IS [NOT] NULL    BitmapBasedFilterOperator: no nulls
      AND / OR         trues = AND / OR of the trues; falses = NOT(AND / OR of (trues_i OR nulls_i)); no nulls
                       (AndFilterOperator.java:60-86, OrFilterOperator.java:59-85)
      NOT              trues = the child's falses, falses = its trues (NotFilterOperator.java:52-60)"""
    if fc.type == "CONSTANT":
        t = _TRUE if fc.constant else _FALSE
        return t, _fold_not(t), None
    if fc.type == "PREDICATE":
        pred = fc.predicate
        p = compile_predicate(seg, pred)
        if pred.type in ("IS_NULL", "IS_NOT_NULL") or not seg.has_null_vector(pred.column):
            return p, _fold_not(p), None
        n, nn = _null_leaf(seg, pred.column), _null_leaf(seg, pred.column, True)
        if not seg.column_metadata(pred.column).has_dictionary:
            # raw-value evaluators are never always-true / always-false (BaseRawValueBasedPredicateEvaluator.java:
            # 37-44): the scan operator keeps the null bitmap as its nulls even when p folded to a constant here
            return _fold_and([p, nn]), _fold_and([_fold_not(p), nn]), n
        if _is_const(p, _FALSE):
            return _FALSE, _TRUE, None
        if _is_const(p, _TRUE):
            return nn, n, None
        return _fold_and([p, nn]), _fold_and([_fold_not(p), nn]), n
    if fc.type == "NOT":
        t, f, _ = _three_valued(seg, fc.children[0])
        return f, t, None
    parts = [_three_valued(seg, c) for c in fc.children]
    either = [t if nl is None else _fold_or([t, nl]) for t, _, nl in parts]
    if fc.type == "AND":
        return _fold_and([t for t, _, _ in parts]), _fold_not(_fold_and(either)), None
    if fc.type == "OR":
        return _fold_or([t for t, _, _ in parts]), _fold_not(_fold_or(either)), None
    raise ValueError(fc.type)


def null_handling_enabled(query: QueryContext) -> bool:
    """QueryContext.isNullHandlingEnabled (the enableNullHandling query option, QueryContext.java:597)."""
    return str(query.options.get("enableNullHandling", "false")).strip().lower() == "true"


def compile_filter(seg: GpuSegment, fc: Optional[FilterContext], null_handling: bool = False):
    """FilterContext -> leaf/node tree for one segment, constants folded (FilterPlanNode.java:197-229).
    null_handling: the docs where the filter is TRUE under three-valued logic (_three_valued)."""
    if fc is None:
        return _TRUE
    if null_handling:
        return _three_valued(seg, fc)[0]
    if fc.type == "PREDICATE":
        return compile_predicate(seg, fc.predicate)
    if fc.type == "CONSTANT":
        return _TRUE if fc.constant else _FALSE
    if fc.type == "NOT":
        c = compile_filter(seg, fc.children[0])
        if _is_const(c, _TRUE):
            return _FALSE
        if _is_const(c, _FALSE):
            return _TRUE
        if isinstance(c, _Leaf) and c.kind in (_lib.LEAF_DICT_SET, _lib.LEAF_INVERTED, _lib.LEAF_RAW_SET, _lib.LEAF_NULL):
            return _Leaf(c.kind, c.column, c.lo, c.hi, not c.exclusive, c.ids)
        return _Node(_lib.NODE_NOT, [c])
    kids = [compile_filter(seg, c) for c in fc.children]
    if fc.type == "AND":
        if any(_is_const(k, _FALSE) for k in kids):
            return _FALSE
        kids = [k for k in kids if not _is_const(k, _TRUE)]
        if not kids:
            return _TRUE
        if len(kids) == 1:
            return kids[0]
        # evaluation order (FilterOperatorUtils :205-252): sorted < bitmap < scan
        prio = {_lib.LEAF_DOC_RANGES: 0, _lib.LEAF_INVERTED: 1, _lib.LEAF_DICT_RANGE: 3, _lib.LEAF_DICT_SET: 3,
                _lib.LEAF_RAW_RANGE: 3, _lib.LEAF_RAW_SET: 3}
        kids.sort(key=lambda k: prio.get(k.kind, 2) if isinstance(k, _Leaf) else (4 if k.op == _lib.NODE_AND else 5))
        return _Node(_lib.NODE_AND, kids)
    if fc.type == "OR":
        if any(_is_const(k, _TRUE) for k in kids):
            return _TRUE
        # (only EQ / IN predicates merge: MergeEqInFilterOptimizer leaves ranges as separate scan operators)
        eq_in = [c.type == "PREDICATE" and c.predicate.type in ("EQ", "IN") for c in fc.children]
        kept = [(k, m) for k, m in zip(kids, eq_in) if not _is_const(k, _FALSE)]
        kids = _merge_or_leaves([k for k, _ in kept], [m for _, m in kept])
        if not kids:
            return _FALSE
        if len(kids) == 1:
            return kids[0]
        return _Node(_lib.NODE_OR, kids)
    raise ValueError(fc.type)


def _leaf_ids(leaf):
    if leaf.kind == _lib.LEAF_DICT_RANGE:
        return np.arange(leaf.lo, leaf.hi, dtype=np.int32)
    return np.asarray(leaf.ids, dtype=np.int32)


def _merge_or_leaves(kids, mergeable=None):
    """OR of EQ / IN leaves on one dictionary column -> one leaf over the union of their dict ids, as the reference's
    broker rewrites an OR of EQ / IN predicates on one column into one IN (MergeEqInFilterOptimizer,
    pinot-core/.../query/optimizer/filter/MergeEqInFilterOptimizer.java:40-120): a scan leaf (DICT_SET; the library
    turns a contiguous id set into a range) when every merged leaf scans, an inverted leaf when every one reads the
    inverted index. Exclusive (NOT_EQ / NOT_IN) leaves and leaves of other predicates (mergeable[i] False: ranges,
    which the optimizer leaves alone, so numEntriesScannedInFilter counts one scan per range) stay apart. The doc set
    is the OR's."""
    scan = (_lib.LEAF_DICT_RANGE, _lib.LEAF_DICT_SET)
    groups, order = {}, []
    for i, k in enumerate(kids):
        fam = None
        if isinstance(k, _Leaf) and k.column is not None and not k.exclusive and (mergeable is None or mergeable[i]):
            fam = "scan" if k.kind in scan else ("inv" if k.kind == _lib.LEAF_INVERTED else None)
        key = (k.column, fam) if fam else id(k)
        if key not in groups:
            groups[key] = []
            order.append(key)
        groups[key].append(k)
    out = []
    for key in order:
        g = groups[key]
        if len(g) == 1 or not isinstance(key, tuple):
            out.extend(g)
            continue
        ids = np.unique(np.concatenate([_leaf_ids(k) for k in g])).astype(np.int32)
        out.append(_Leaf(_lib.LEAF_DICT_SET if key[1] == "scan" else _lib.LEAF_INVERTED, key[0], ids=ids))
    return out


def _flatten(tree, col_index, out, keep):
    if isinstance(tree, _Leaf):
        n = _lib.FilterNode()
        n.op = _lib.NODE_LEAF
        n.leaf_kind = tree.kind
        n.column = col_index[tree.column] if tree.column is not None else -1
        n.lo, n.hi = tree.lo, tree.hi
        n.exclusive = int(tree.exclusive)
        if tree.ids is not None:
            ids = np.ascontiguousarray(tree.ids, dtype=np.int32)
            keep.append(ids)
            n.count = len(ids) // 2 if tree.kind == _lib.LEAF_DOC_RANGES else len(ids)  # RAW_*: int32 words
            n.ids = ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        out.append(n)
        return
    n = _lib.FilterNode()
    n.op = tree.op
    n.num_children = len(tree.children)
    out.append(n)
    for c in tree.children:
        _flatten(c, col_index, out, keep)


def _leaf_columns(tree, acc):
    if isinstance(tree, _Leaf):
        if tree.column is not None and tree.column not in acc:
            acc.append(tree.column)
    else:
        for c in tree.children:
            _leaf_columns(c, acc)


# ------------------------------------------------------------------------------ aggregations
def _strip_cast(e):
    while isinstance(e, Function) and e.name == "cast":
        e = e.args[0]
    return e


def _gpu_expr(e):
    """Aggregation argument -> (PHIP_EXPR_*, col_a, col_b)."""
    e = _strip_cast(e)
    if isinstance(e, Identifier):
        return _lib.EXPR_COLUMN, e.name, None
    if isinstance(e, Function) and e.name in ("times", "minus", "plus") and len(e.args) == 2:
        a, b = _strip_cast(e.args[0]), _strip_cast(e.args[1])
        if isinstance(a, Identifier) and isinstance(b, Identifier):
            op = {"times": _lib.EXPR_MUL, "minus": _lib.EXPR_SUB, "plus": _lib.EXPR_ADD}[e.name]
            return op, a.name, b.name
    raise UnsupportedOnGpu(f"aggregation argument {e} is outside the GPU expression subset")


def plan_aggregations(aggs: Sequence[AggregationInfo], programs: Optional[Sequence[int]] = None):
    """Query aggregations -> GPU primitives (deduplicated) + per-function slot mapping. ``programs``: per
    aggregation, the filter program it reads (several programs in one pass); primitives of different programs
    never merge."""
    prims = []  # (function, expr, col_a, col_b, log2m, program)
    mapping = []

    for j, ag in enumerate(aggs):
        prog = programs[j] if programs is not None else 0

        def slot(p):
            p = p + (prog,)
            if p not in prims:
                prims.append(p)
            return prims.index(p)

        f = ag.function
        if f == "count":
            mapping.append(("count", slot((_lib.AGG_COUNT, 0, None, None, 0))))
            continue
        expr = _gpu_expr(ag.argument)
        if f == "sum":
            mapping.append(("sum", slot((_lib.AGG_SUM,) + expr + (0,))))
        elif f == "min":
            mapping.append(("min", slot((_lib.AGG_MIN,) + expr + (0,))))
        elif f == "max":
            mapping.append(("max", slot((_lib.AGG_MAX,) + expr + (0,))))
        elif f == "avg":
            mapping.append(("avg", (slot((_lib.AGG_SUM,) + expr + (0,)), slot((_lib.AGG_COUNT, 0, None, None, 0)))))
        elif f == "minmaxrange":
            mapping.append(("minmaxrange", (slot((_lib.AGG_MIN,) + expr + (0,)), slot((_lib.AGG_MAX,) + expr + (0,)))))
        elif f in ("distinctcounthll", "distinctcountrawhll"):
            # (over an expression: its DOUBLE values hashed on the device, as the reference offers a transform's result)
            mapping.append((f, slot((_lib.AGG_HLL,) + expr + (ag.log2m,))))
        else:
            raise UnsupportedOnGpu(f"aggregation {f} is not on the GPU path")
    return prims, mapping


# ------------------------------------------------------------------------------ operators
class GpuCombineOperator:
    """One operator over all segments of the query (the all-segment GPU variant of SURVEY.md §8b)."""

    null_keys = 0  # phip_query_desc.null_group_by (set per instance under enableNullHandling)

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int,
                 segment_filters=None, programs=None):
        """segment_filters: optional per-segment (FilterContext or None, inclusive doc ranges or None) replacing
        query.filter -- the star-tree path's matched documents AND remaining predicates.
        programs: optional (filters, agg_programs) -- k filters (None = every doc) evaluated in one pass, and per
        query aggregation the index of the filter whose docs it aggregates (phip_query_desc.num_filter_programs;
        query.filter is then unused)."""
        self.query = query
        self.segments = list(segments)
        self.num_groups_limit = num_groups_limit
        for e in query.group_by:
            if not isinstance(e, Identifier):
                raise UnsupportedOnGpu(f"group-by expression {e}")
        self.num_programs = len(programs[0]) if programs is not None else 1
        self.stats_programs = 0  # phip_query_desc.stats_programs: 0 = every program's scans count
        self.prims, self.mapping = plan_aggregations(query.aggregations, programs[1] if programs is not None else None)
        nh = null_handling_enabled(query)
        # enableNullHandling: the group-by columns whose null docs key as the null key (phip_query_desc.null_group_by;
        # NoDictionary*GroupKeyGenerator with null handling, DefaultGroupByExecutor.java:106-116)
        self.null_keys = 0
        if nh:
            for k, e in enumerate(query.group_by):
                if isinstance(e, Identifier) and any(s.has_column(e.name) and s.has_null_vector(e.name)
                                                     for s in self.segments):
                    self.null_keys |= 1 << k
        if programs is not None:
            # program-major, as filter_offsets lays them out: program p of segment s at p * nseg + s
            self.trees = [compile_filter(s, f, nh) for f in programs[0] for s in self.segments]
        elif segment_filters is None:
            self.trees = [compile_filter(s, query.filter, nh) for s in self.segments]
        else:
            self.trees = []
            for s, (flt, ranges) in zip(self.segments, segment_filters):
                t = compile_filter(s, flt, nh)
                if ranges is not None:
                    if len(ranges) == 0 or _is_const(t, _FALSE):
                        t = _FALSE
                    else:
                        leaf = _Leaf(_lib.LEAF_DOC_RANGES, None, ids=np.asarray(ranges, dtype=np.int32))
                        t = leaf if _is_const(t, _TRUE) else _Node(_lib.NODE_AND, [leaf, t])
                self.trees.append(t)
        cols = []
        for t in self.trees:
            _leaf_columns(t, cols)
        for p in self.prims:
            for c in (p[2], p[3]):
                if c is not None and c not in cols:
                    cols.append(c)
        for e in query.group_by:
            if e.name not in cols:
                cols.append(e.name)
        self.columns = cols
        for s in self.segments:
            for c in cols:
                if not s.has_column(c):
                    raise KeyError(f"segment {s.name} has no column {c}")

    def _desc(self, keep):
        col_index = {c: i for i, c in enumerate(self.columns)}
        q = _lib.QueryDesc()
        names = (ctypes.c_char_p * max(len(self.columns), 1))(*[c.encode() for c in self.columns])
        keep.append(names)
        q.num_columns = len(self.columns)
        q.columns = names
        handles = (ctypes.c_uint64 * len(self.segments))(*[s.handle for s in self.segments])
        keep.append(handles)
        q.num_segments = len(self.segments)
        q.segments = handles
        nodes = []
        offsets = [0]
        for t in self.trees:
            if not _is_const(t, _TRUE):
                _flatten(t, col_index, nodes, keep)
            offsets.append(len(nodes))
        offs = (ctypes.c_int32 * len(offsets))(*offsets)
        keep.append(offs)
        q.filter_offsets = offs
        arr = (_lib.FilterNode * max(len(nodes), 1))(*nodes)
        keep.append(arr)
        q.filter_nodes = arr
        q.num_filter_programs = self.num_programs
        q.stats_programs = self.stats_programs
        aggs = (_lib.Aggregation * max(len(self.prims), 1))()
        for i, (f, expr, ca, cb, log2m, prog) in enumerate(self.prims):
            aggs[i].function = f
            aggs[i].expr = expr
            aggs[i].column_a = col_index[ca] if ca is not None else -1
            aggs[i].column_b = col_index[cb] if cb is not None else -1
            aggs[i].log2m = log2m
            aggs[i].program = prog
        keep.append(aggs)
        q.num_aggregations = len(self.prims)
        q.aggregations = aggs
        gb = (ctypes.c_int32 * max(len(self.query.group_by), 1))(*[col_index[e.name] for e in self.query.group_by])
        keep.append(gb)
        q.num_group_by = len(self.query.group_by)
        q.group_by_columns = gb
        q.num_groups_limit = self.num_groups_limit
        q.null_group_by = self.null_keys
        q.order_by_aggregation, q.order_by_desc, q.trim_size, okeys, terms = self._trim_spec()
        if okeys:
            arr = (ctypes.c_int32 * len(okeys))(*okeys)
            keep.append(arr)
            q.num_order_by_keys = len(okeys)
            q.order_by_keys = arr
        if terms:
            arr = (_lib.OrderTerm * len(terms))(*[_lib.OrderTerm(*t) for t in terms])
            keep.append(arr)
            q.num_order_terms = len(terms)
            q.order_terms = arr
        return q

    def _trim_spec(self):
        """Server-level trim of GroupByUtils.createIndexedTableForCombineOperator (GroupByUtils.java:96-140):
        with ORDER BY the combine keeps trimSize = getTableCapacity(limit, minServerGroupTrimSize)
        = max(5 * limit, 5000) records (:55-58; default minServerGroupTrimSize 5000,
        InstancePlanMakerImplV2.java:92), ordered by the ORDER BY (TableResizer's extractors:
        group-by values, or aggregations' final results). Returns (order_by_aggregation, desc, trimSize,
        group-key order, general terms): a single SUM/MIN/MAX/COUNT or only group-by columns use the one-pass
        device orders, any other mix of group-by columns and SUM/MIN/MAX/COUNT/AVG/MINMAXRANGE goes as
        PHIP_ORDER_* terms (DISTINCTCOUNTHLL by its cardinality estimate, PHIP_ORDER_HLL); an ORDER BY outside that
        (DISTINCTCOUNTRAWHLL, post-aggregation expressions) returns every group (the broker's ORDER BY + LIMIT gives
        the same final rows)."""
        from .reduce import _agg_index
        q = getattr(self, "trim_query", None) or self.query
        none = (-1, 0, 0, [], [])
        if not q.group_by or not q.order_by or not getattr(self, "device_trim", True):
            return none
        seg_trim = getattr(self, "segment_trim", None)
        if seg_trim is not None:  # one segment's GroupByOperator trim (minSegmentGroupTrimSize > 0)
            min_trim = seg_trim
        else:
            min_trim = int(q.options.get("minServerGroupTrimSize", DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE))
        if min_trim <= 0:  # trim disabled (GroupByUtils.java:108)
            return none
        trim = min(max(5 * int(q.limit), min_trim), 2 ** 31 - 1)
        gb = [str(e) for e in q.group_by]
        if len(q.order_by) > 8 or len(gb) > 8:
            return none
        for ob in q.order_by:
            # the device orders a null key after every value (its id is the dictionary's cardinality): the reference's
            # default; an explicit NULLS FIRST ascending / NULLS LAST descending is left to the host's trim
            if str(ob.expression) in gb and (self.null_keys >> gb.index(str(ob.expression))) & 1 and \
                    ob.nulls_last is not None and ob.nulls_last != ob.ascending:
                return none
        if all(str(ob.expression) in gb for ob in q.order_by):
            keys = [(gb.index(str(ob.expression)) + 1) * (1 if ob.ascending else -1) for ob in q.order_by]
            return -1, 0, trim, keys, []
        terms = []
        for ob in q.order_by:
            desc = int(not ob.ascending)
            if str(ob.expression) in gb:
                terms.append((_lib.ORDER_GROUP_KEY, gb.index(str(ob.expression)), 0, desc))
                continue
            i = _agg_index(q, ob.expression)
            if i is None or (q.aggregations[i].filter is not None and self.num_programs == 1):
                return none
            f, sl = self.mapping[i]
            if f in ("sum", "min", "max", "count"):
                terms.append((_lib.ORDER_VALUE, int(sl), 0, desc))
            elif f == "avg":
                terms.append((_lib.ORDER_AVG, int(sl[0]), int(sl[1]), desc))
            elif f == "minmaxrange":
                terms.append((_lib.ORDER_RANGE, int(sl[0]), int(sl[1]), desc))
            elif f == "distinctcounthll":  # (its cardinality estimate, computed from the registers on the device)
                terms.append((_lib.ORDER_HLL, int(sl), 0, desc))
            else:
                return none
        if len(terms) == 1 and terms[0][0] == _lib.ORDER_VALUE:
            return terms[0][1], terms[0][3], trim, [], []
        return -1, 0, trim, [], terms

    def filter_bitmap(self) -> np.ndarray:
        """BaseFilterOperator.getTrues for a single segment, as 64-doc bitmap words."""
        if len(self.segments) != 1:
            raise ValueError("filter_bitmap takes one segment")
        keep = []
        q = self._desc(keep)
        nwords = (self.segments[0].num_docs + 63) // 64
        out = np.zeros(max(nwords, 1), dtype=np.uint64)
        _lib.check(_lib.load().phip_filter_bitmap(ctypes.byref(q), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                                  len(out)))
        return out[:nwords]

    def run_raw(self, prepare_only=False):
        """One execution of the prepared plan (phip_plan_create once per operator, then phip_plan_execute:
        InstancePlanMakerImplV2's Plan run by GlobalPlanImplV0.execute)."""
        lib = getattr(self, "_lib", None) or _lib.load()  # (the loaded library, kept once the plan exists)
        if getattr(self, "_plan", None) is None:
            keep = []
            q = self._desc(keep)
            h = ctypes.c_uint64(0)
            _lib.check(lib.phip_plan_create(ctypes.byref(q), ctypes.byref(h)))
            self._plan = h.value
            self._lib = lib
        if prepare_only:
            return None
        self._apply_deadline(lib)
        res = ctypes.POINTER(_lib.Result)()
        _lib.check(lib.phip_plan_execute(self._plan, ctypes.byref(res)))
        return res

    def _apply_deadline(self, lib):
        """The running query's end time to the prepared plan (phip_plan_set_deadline; 0 = none), when it changed."""
        end = _END_TIME_MS.get()
        d = int(end) if end is not None else 0
        if d != getattr(self, "_deadline_set", 0):
            _lib.check(lib.phip_plan_set_deadline(self._plan, d))
            self._deadline_set = d

    def exchange(self):
        """(devices, exchange kind) of the prepared plan (phip_plan_exchange): a plan over segments on several devices
        is a node plan whose sub-plans' partials meet in an RCCL reduce (_lib.EXCHANGE_RCCL), a peer merge
        (EXCHANGE_PEER), a hash-table insert on the root device (EXCHANGE_HASH) or the host record merge
        (EXCHANGE_RECORDS); (1, EXCHANGE_NONE) for one device."""
        if getattr(self, "_plan", None) is None:
            return 1, _lib.EXCHANGE_NONE
        parts, kind = ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.check(_lib.load().phip_plan_exchange(self._plan, ctypes.byref(parts), ctypes.byref(kind)))
        return parts.value, kind.value

    def close(self):
        """Release the prepared plan (and with it the last references to unloaded segments)."""
        if getattr(self, "_plan", None):
            self._lib.phip_plan_destroy(self._plan)
            self._plan = None
        self._str_dicts = None  # (decoded entries of the destroyed plan's dictionaries)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- NonScanBasedAggregationOperator (AggregationPlanNode.java:107-118, isFitForNonScanBasedPlan :165-190)
    _NON_SCAN = ("count", "min", "max", "minmaxrange", "distinctcounthll", "distinctcountrawhll")

    def _non_scan_fit(self):
        if self.query.group_by or not all(_is_const(t, _TRUE) for t in self.trees):
            return False
        nh = null_handling_enabled(self.query)
        for ag in self.query.aggregations:
            if ag.function not in self._NON_SCAN:
                return False
            if nh and ag.argument is not None and (not isinstance(ag.argument, Identifier) or any(
                    s.has_null_vector(ag.argument.name) for s in self.segments)):
                return False  # (AggregationPlanNode.hasNullValues, :104,125-150)
            if ag.function == "count":
                continue
            if not isinstance(ag.argument, Identifier):
                return False
            for s in self.segments:
                if not s.column_metadata(ag.argument.name).has_dictionary:
                    return False
        return True

    def _non_scan_block(self):
        from . import hll
        results = None
        stats = ExecutionStatistics()
        for s in self.segments:
            seg_res = []
            for ag in self.query.aggregations:
                if ag.function == "count":
                    seg_res.append(s.num_docs)
                    continue
                d = s.dictionary(ag.argument.name)
                if ag.function == "min":
                    seg_res.append(float(d.get(0)))
                elif ag.function == "max":
                    seg_res.append(float(d.get(len(d) - 1)))
                elif ag.function == "minmaxrange":
                    seg_res.append((float(d.get(0)), float(d.get(len(d) - 1))))
                else:
                    seg_res.append(hll.registers_of_hashes(hll.hash_values(d.values, d.data_type), ag.log2m))
            if results is None:
                results = seg_res
            else:
                from .results import merge_intermediate
                results = [merge_intermediate(ag.function, a, b) for ag, a, b in zip(self.query.aggregations, results, seg_res)]
            stats.merge(ExecutionStatistics(s.num_docs, 0, 0, s.num_docs, 1, 1 if s.num_docs else 0))
        return AggregationResultsBlock(self.query.aggregations, results, stats)

    def next_block(self):
        fit = self.__dict__.get("_non_scan")  # (a function of the query and the segments: decided once)
        if fit is None:
            fit = self._non_scan = self._non_scan_fit()
        if fit:
            return self._non_scan_block()
        return self._block_from_result(self.run_raw())

    # -- multi-GPU servers (include/pinot_hip.h "multi-GPU servers"; engine/distributed.py) -------------
    def execute_partial(self):
        """Runs the plan up to this GPU's dense partial group table (phip_plan_execute_partial). Returns the
        _lib.Partial (device pointers), or None when the plan cannot hand one out (hash-table key space,
        numGroupsLimit reached on this GPU; an aggregation the non-scan operator answers from dictionaries, whose
        statistics differ) -- the caller then merges records instead. Aggregation-only plans hand out a one-group
        table (rows + statistics + u8 HLL registers in device memory, include/pinot_hip.h)."""
        if not self.query.group_by and self._non_scan_fit():
            return None
        lib = _lib.load()
        self.run_raw(prepare_only=True)
        self._apply_deadline(lib)
        part = _lib.Partial()
        rc = lib.phip_plan_execute_partial(self._plan, ctypes.byref(part))
        if rc == _lib.PHIP_ERR_UNSUPPORTED:
            return None
        _lib.check(rc)
        return part

    def abandon_partial(self):
        """Hands a pending partial table back unfinished (phip_plan_abandon_partial): the ranks agreed to merge
        records instead, and the next execution of this plan rewrites the table."""
        if getattr(self, "_plan", None):
            _lib.check(_lib.load().phip_plan_abandon_partial(self._plan))

    def finish(self, merged):
        """Result block of the (merged) partial table: compaction, server-level trim, statistics of `merged`."""
        lib = _lib.load()
        res = ctypes.POINTER(_lib.Result)()
        _lib.check(lib.phip_plan_finish(self._plan, ctypes.byref(merged), ctypes.byref(res)))
        return self._block_from_result(res)

    def _aggregation_block(self, res):
        """One-row results (aggregation only, no HLL) from one read of the result's scalars and its three short
        arrays (_lib.RESULT_IMAGE): a ctypes field read costs ~0.1 us and the general path makes ~30 per query.
        None: the general path applies."""
        f = _lib.RESULT_IMAGE.unpack(ctypes.string_at(res, _lib.RESULT_IMAGE.size))
        na, ng, nhll = f[7], f[8], f[10]
        if ng != 1 or nhll:
            return None
        dec = self.__dict__.get("_agg_dec")
        if dec is None or dec[0] != na:  # (per operator: the slots' structs and each primitive's kind)
            kinds = [0 if p[0] == _lib.AGG_COUNT else (1 if p[0] == _lib.AGG_SUM else 2) for p in self.prims]
            pairs = [fn in ("avg", "minmaxrange") for fn, _ in self.mapping]
            dec = self._agg_dec = (na, struct.Struct(f"<{na}d"), struct.Struct(f"<{na}q"), struct.Struct(f"<{na}i"),
                                   kinds, pairs)
        _, sd, sq, si, kinds, pairs = dec
        vals = sd.unpack(ctypes.string_at(f[11], 8 * na)) if na else ()
        longs = sq.unpack(ctypes.string_at(f[12], 8 * na)) if na else ()
        exact = si.unpack(ctypes.string_at(f[19], 4 * na)) if na else ()
        pv = [longs[i] if k == 0 or (k == 1 and exact[i]) else vals[i] for i, k in enumerate(kinds)]
        out = [(pv[s[0]], pv[s[1]]) if pr else pv[s] for pr, (_, s) in zip(pairs, self.mapping)]
        blk = AggregationResultsBlock(self.query.aggregations, out, ExecutionStatistics(*f[0:6]))
        blk.scan_kernel_ms, blk.device_ms = f[15], f[16]
        blk.fused = bool(f[18])
        blk.filter_kernel_ms, blk.agg_kernel_ms = f[20], f[21]
        blk.filter_bytes, blk.agg_bytes = f[22], f[23]
        blk.stream_bytes = f[30]
        blk.segment_docs_matched = None
        return blk

    def _key_values(self, k, dv, ids):
        """Values of group-by column k's keys (`ids` into the result's query-global dictionary) as an array; under
        enableNullHandling the null key (id == the dictionary's cardinality) is None."""
        if (self.null_keys >> k) & 1:
            ids = np.asarray(ids)
            isnull = ids >= dv.cardinality
            if isnull.any():
                out = np.empty(len(ids), dtype=object)
                nn = ~isnull
                if nn.any():
                    vals = self._key_values_plain(k, dv, ids[nn])
                    out[nn] = [v.item() if hasattr(v, "item") else v for v in vals]
                out[isnull] = None
                return out
        return self._key_values_plain(k, dv, ids)

    def _key_values_plain(self, k, dv, ids):
        if DataType(dv.data_type) == DataType.STRING and dv.string_width > 0 and len(ids):
            cache = self.__dict__.get("_str_dicts")
            if cache is None:
                cache = self._str_dicts = {}
            return _string_cache_lookup(cache, k, dv, ids)
        return _dictionary_array(dv, ids)

    def key_types(self):
        """Stored types of the group-by columns, from the column metadata (the group-by block's DataSchema)."""
        return [_STORED[self.segments[0].column_metadata(e.name).data_type] for e in self.query.group_by] \
            if self.segments else None

    def _block_from_result(self, res):
        lib = getattr(self, "_lib", None) or _lib.load()
        if not self.query.group_by:
            blk = self._aggregation_block(res)
            if blk is not None:
                lib.phip_result_free(res)
                return blk
        try:
            r = res.contents
            stats = ExecutionStatistics(r.num_docs_scanned, r.num_entries_scanned_in_filter,
                                        r.num_entries_scanned_post_filter, r.num_total_docs,
                                        r.num_segments_processed, r.num_segments_matched)
            na = r.num_aggregations
            ng = r.num_groups
            plan = getattr(self, "_decode_plan", None)
            if plan is None:  # per operator, once: HLL width and slots (the server loop decodes every execution)
                hs = {}
                for i, p in enumerate(self.prims):
                    if p[0] == _lib.AGG_HLL:
                        hs[i] = len(hs)
                plan = self._decode_plan = (1 << max([p[4] for p in self.prims if p[0] == _lib.AGG_HLL] + [0]), hs)
            m, hll_slot = plan
            # (no groups: the library's arrays may be null)
            if not self.query.group_by and ng == 1:
                # one row: read its few slots through the pointers (a numpy view + copy costs ~6 us per array,
                # on every query of the server loop)
                vals = [[r.values[i] for i in range(na)]]
                longs = [[r.long_values[i] for i in range(na)]]
            elif not self.query.group_by:
                vals = (np.ctypeslib.as_array(r.values, shape=(ng * na,)).reshape(ng, na).tolist() if ng * na
                        else [[0.0] * na for _ in range(ng)])
                longs = (np.ctypeslib.as_array(r.long_values, shape=(ng * na,)).reshape(ng, na).tolist() if ng * na
                         else [[0] * na for _ in range(ng)])
            else:
                # (ng, na) arrays: the group-by decode below takes whole columns of them
                vals = (np.ctypeslib.as_array(r.values, shape=(ng * na,)).reshape(ng, na) if ng * na
                        else np.zeros((ng, na), np.float64))
                longs = (np.ctypeslib.as_array(r.long_values, shape=(ng * na,)).reshape(ng, na) if ng * na
                         else np.zeros((ng, na), np.int64))
            hll = None
            if r.num_hll and ng:
                hll = np.ctypeslib.as_array(r.hll_registers, shape=(ng * r.num_hll * m,)).reshape(ng, r.num_hll, m).copy()
            # long_exact[a]: the library kept an exact int64 sum (else it summed in double: int64 overflow bound)
            exact = [bool(r.long_exact[i]) for i in range(na)] if na else []

            def prim_value(g, i):
                f = self.prims[i][0]
                if f == _lib.AGG_COUNT:
                    return int(longs[g][i])
                if f == _lib.AGG_SUM:
                    return int(longs[g][i]) if exact[i] else float(vals[g][i])
                if f in (_lib.AGG_MIN, _lib.AGG_MAX):
                    return float(vals[g][i])
                return hll[g, hll_slot[i], :1 << self.prims[i][4]].copy()  # (slots hold 2^max-log2m bytes)

            def intermediates(g):
                out = []
                for f, s in self.mapping:
                    if f in ("avg", "minmaxrange"):
                        out.append((prim_value(g, s[0]), prim_value(g, s[1])))
                    else:
                        out.append(prim_value(g, s))
                return out

            if not self.query.group_by:
                blk = AggregationResultsBlock(self.query.aggregations, intermediates(0), stats)
            else:
                nk = r.num_group_by
                keys = np.ctypeslib.as_array(r.group_keys, shape=(max(ng * nk, 1),))[:ng * nk].reshape(ng, nk) if ng else np.zeros((0, nk), np.int32)
                # The block is columnar (the reference's DataTable keeps dictionary-encoded columns too): per group-by
                # column the groups' key values as one array, per primitive one value array -- copied out of the
                # library's result here; the {key tuple: intermediates} view is built on first access
                # (GroupByResultsBlock.groups), as one list per column zipped into the groups' lists.
                cols = []  # per group-by column: the values of the groups' keys (only the ids that occur)
                key_space = 1  # the query-global key space: the union of the segments' values per column
                for k in range(nk):
                    dv = _lib.DictionaryView()
                    _lib.check(lib.phip_result_dictionary(res, k, ctypes.byref(dv)))
                    key_space *= max(int(dv.cardinality) + ((self.null_keys >> k) & 1), 1)
                    cols.append(self._key_values(k, dv, keys[:, k]) if ng else np.zeros(0, np.int64))
                prim_arrays = []
                for i, p in enumerate(self.prims):
                    f = p[0]
                    if f == _lib.AGG_COUNT or (f == _lib.AGG_SUM and exact[i]):
                        prim_arrays.append(longs[:, i].copy())
                    elif f in (_lib.AGG_SUM, _lib.AGG_MIN, _lib.AGG_MAX):
                        prim_arrays.append(vals[:, i].copy())
                    else:
                        mi = 1 << self.prims[i][4]
                        prim_arrays.append(hll[:, hll_slot[i], :mi] if hll is not None  # (hll is a copy)
                                           else np.zeros((0, mi), np.uint8))
                blk = GroupByResultsBlock(self.query.aggregations, list(self.query.group_by), None, stats,
                                          bool(r.num_groups_limit_reached))
                blk.set_columns(cols, prim_arrays, self.mapping)
                blk.num_groups_trimmed = bool(r.num_groups_trimmed)
                blk.key_space = key_space
                blk.key_types = self.key_types()
            blk.device_ms = r.device_ms
            blk.scan_kernel_ms = r.scan_kernel_ms
            nseg = r.num_segments_processed
            blk.segment_docs_matched = ((np.ctypeslib.as_array(r.segment_docs_matched, shape=(nseg,)).tolist() if nseg
                                         else []) if self.query.group_by and r.segment_docs_matched else None)
            blk.program_docs_matched = ([int(r.program_docs_matched[p]) for p in range(self.num_programs)]
                                        if self.query.group_by and r.program_docs_matched else None)
            blk.filter_kernel_ms, blk.agg_kernel_ms = r.filter_kernel_ms, r.agg_kernel_ms
            blk.filter_bytes, blk.agg_bytes = int(r.filter_bytes), int(r.agg_bytes)
            blk.stream_bytes = int(r.stream_bytes)
            blk.fused = bool(r.fused)
            return blk
        finally:
            lib.phip_result_free(res)


def _string_cache_lookup(cache, k, dv, ids):
    """STRING group keys through a per-operator cache of decoded dictionary entries: the query-global dictionary of
    a dictionary column is the plan's own (stable while the plan lives), so each entry is decoded once per plan
    (lazily: only the ids some execution's groups use), not once per group and execution (Q4.3's 800 groups over two
    STRING keys: ~1600 decodes per query before)."""
    card, w = int(dv.cardinality), int(dv.string_width)
    key = (k, int(dv.values or 0), card, w)
    arr = cache.get(key)
    if arr is None:
        arr = cache[key] = np.empty(card, dtype=object)
    ids = np.asarray(ids, dtype=np.int64)
    uniq = np.unique(ids)
    todo = uniq[np.equal(arr[uniq], None)]
    if len(todo):
        raw = np.ctypeslib.as_array(ctypes.cast(dv.values, ctypes.POINTER(ctypes.c_uint8)), shape=(card * w,))
        for i, v in zip(todo.tolist(), raw.view(f"S{w}")[todo].tolist()):
            arr[i] = v.decode("utf-8")
    return arr[ids]


def _dictionary_array(dv, ids):
    """_dictionary_lookup as a numpy array (object array for STRING)."""
    if DataType(dv.data_type) == DataType.STRING:
        return np.array(_dictionary_lookup(dv, ids), dtype=object)
    ids = np.asarray(ids, dtype=np.int64)
    t = DataType(dv.data_type)
    dt = {DataType.INT: np.int32, DataType.LONG: np.int64, DataType.FLOAT: np.float32, DataType.DOUBLE: np.float64}[t]
    arr = np.ctypeslib.as_array(ctypes.cast(dv.values, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                shape=(max(int(dv.cardinality), 1),))
    return arr[ids]  # (fancy indexing copies: the result's dictionary may go with the result)


def _dictionary_lookup(dv, ids):
    """Values of the dictionary entries `ids` (a result's group keys), without converting the whole dictionary."""
    ids = np.asarray(ids, dtype=np.int64)
    card = dv.cardinality
    t = DataType(dv.data_type)
    if t == DataType.STRING:
        w = dv.string_width
        if w == 0 or len(ids) == 0:
            return [""] * len(ids)
        raw = np.ctypeslib.as_array(ctypes.cast(dv.values, ctypes.POINTER(ctypes.c_uint8)), shape=(card * w,))
        # fixed-width NUL-padded entries as numpy bytes ("S<w>": items come back without the trailing NULs), ~5x
        # faster than a bytes() + rstrip per row
        return [v.decode("utf-8") for v in raw.view(f"S{w}")[ids].tolist()]
    dt = {DataType.INT: np.int32, DataType.LONG: np.int64, DataType.FLOAT: np.float32, DataType.DOUBLE: np.float64}[t]
    arr = np.ctypeslib.as_array(ctypes.cast(dv.values, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(card,))
    return arr[ids].tolist()


_STORED = {DataType.INT: "INT", DataType.LONG: "LONG", DataType.FLOAT: "FLOAT", DataType.DOUBLE: "DOUBLE",
           DataType.STRING: "STRING"}


class GpuSelectionOperator(GpuCombineOperator):
    """SelectionOnlyOperator (pinot-core/.../operator/query/SelectionOnlyOperator.java:40-170) over every segment,
    with SelectionOnlyCombineOperator's merge (…/operator/combine/SelectionOnlyCombineOperator.java:30-70): per
    segment the first LIMIT matched docs in doc order, projected to the select expressions; the segments' rows
    concatenated in segment order up to LIMIT (the reference merges in completion order; which rows a LIMIT below
    the matches keeps is thread-timing dependent there, segment order here). One filter launch, then the selection
    kernels (select.hip) rank the matched docs and gather the columns; STRING columns come back as ids in a
    query-global dictionary. Statistics as the reference's: numDocsScanned = the rows each segment kept,
    numEntriesScannedPostFilter = that x the projected columns. numEntriesScannedInFilter is the full filter scan
    (the reference's lazy scan stops at LIMIT; the known answers exclude it). LIMIT 0 is EmptySelectionOperator:
    the schema, no rows, zero statistics. ORDER BY (SelectionOrderByOperator) is outside this operator."""

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int = 0):
        if query.order_by and query.limit > 0:
            raise UnsupportedOnGpu("selection ORDER BY (SelectionOrderByOperator)")
        if not segments:
            raise UnsupportedOnGpu("selection over no segments")
        self.exprs = query.select_expressions(list(segments[0].segment.columns))
        self.sel = []
        for e in self.exprs:
            e2 = _strip_cast(e)
            if isinstance(e2, Identifier):
                self.sel.append((_lib.EXPR_COLUMN, e2.name, None))
            else:
                self.sel.append(_gpu_expr(e2))
        if len(self.sel) > 16:
            raise UnsupportedOnGpu("selection of more than 16 expressions")
        super().__init__(query, segments, num_groups_limit)
        for _, a, b in self.sel:
            for c in (a, b):
                if c is not None and c not in self.columns:
                    self.columns.append(c)
        for s in self.segments:
            for c in self.columns:
                if not s.has_column(c):
                    raise KeyError(f"segment {s.name} has no column {c}")
        self.names = [str(e) for e in self.exprs]
        self.types = []
        for expr, a, _ in self.sel:
            m = self.segments[0].column_metadata(a)
            if expr == _lib.EXPR_COLUMN:
                self.types.append(_STORED[m.data_type])
            else:
                self.types.append("DOUBLE")

    def _desc(self, keep):
        q = super()._desc(keep)
        col_index = {c: i for i, c in enumerate(self.columns)}
        arr = (_lib.SelectExpr * len(self.sel))()
        for i, (expr, a, b) in enumerate(self.sel):
            arr[i].expr = expr
            arr[i].column_a = col_index[a]
            arr[i].column_b = col_index[b] if b is not None else -1
        keep.append(arr)
        q.num_select = len(self.sel)
        q.select = arr
        q.select_limit = int(self.query.limit)
        return q

    def next_block(self):
        if self.query.limit <= 0:  # EmptySelectionOperator: the data schema only
            stats = ExecutionStatistics(0, 0, 0, sum(s.num_docs for s in self.segments), len(self.segments), 0)
            return SelectionResultsBlock(self.names, self.types, [[] for _ in self.names], stats)
        lib = _lib.load()
        res = self.run_raw()
        try:
            r = res.contents
            stats = ExecutionStatistics(r.num_docs_scanned, r.num_entries_scanned_in_filter,
                                        r.num_entries_scanned_post_filter, r.num_total_docs,
                                        r.num_segments_processed, r.num_segments_matched)
            n, k = int(r.num_rows), int(r.num_select)
            raw = (np.ctypeslib.as_array(r.select_values, shape=(k * n,)).reshape(k, n).copy() if n * k
                   else np.zeros((k, 0), dtype=np.uint64))
            cols = []
            for j, t in enumerate(self.types):
                v = raw[j]
                if t in ("INT", "LONG"):
                    cols.append(v.view(np.int64).astype(np.int32 if t == "INT" else np.int64))
                elif t == "FLOAT":
                    cols.append(v.view(np.float64).astype(np.float32))
                elif t == "DOUBLE":
                    cols.append(v.view(np.float64))
                else:
                    dv = _lib.DictionaryView()
                    _lib.check(lib.phip_result_select_dictionary(res, j, ctypes.byref(dv)))
                    cols.append(_dictionary_lookup(dv, v.view(np.int64)) if n else [])
            blk = SelectionResultsBlock(self.names, list(self.types), cols, stats)
            blk.device_ms = r.device_ms
            blk.filter_kernel_ms, blk.agg_kernel_ms = r.filter_kernel_ms, r.agg_kernel_ms
            blk.filter_bytes, blk.agg_bytes = int(r.filter_bytes), int(r.agg_bytes)
            blk.fused = False
            return blk
        finally:
            lib.phip_result_free(res)


def _stats_mask(keys, stats_filters) -> int:
    """phip_query_desc.stats_programs for programs keyed by ``keys`` (their FILTER clauses, in program order)."""
    if stats_filters is None:
        return 0
    return sum(1 << p for p, k in enumerate(keys) if k in stats_filters) or (1 << 31)  # (no program 31: none)


def _run_parts(parts):
    """The per-info operators of a filtered query, in info order (FilteredAggregationOperator runs its infos one
    after another too). Running them on concurrent execution lanes from a thread pool was measured slower on C1
    FILTERED_MIXED (0.48 -> 0.56 ms p50, profiles/r02c_configs_c1.jsonl): each info's device work is ~50 us and the
    host side of an execution does not overlap under the GIL."""
    out = []
    for _, op in parts:
        check_deadline("between filtered-aggregation plans")
        out.append(op.next_block())
    return out


class GpuFilteredAggregationOperator:
    """FilteredAggregationOperator (pinot-core/.../operator/query/FilteredAggregationOperator.java:67-113)
    over all segments: the aggregations are grouped by their FILTER clause (unfiltered ones under the
    main filter), as AggregationFunctionUtils.buildFilteredAggregationInfos does, and every group's filter --
    main AND its FILTER -- becomes one filter program of a single GPU plan: one filter launch evaluates all
    programs into one tile mask each and one aggregation launch applies every function to its own program's
    docs (phip_query_desc.num_filter_programs). Results return in query order; numDocsScanned and the entries
    scanned are summed over the programs, like the reference operator's statistics. More than
    kMaxPrograms (8) groups, or more than 8 primitive slots, run as one plan per group."""

    _MAX_PROGRAMS = 8  # device.h kMaxPrograms
    _MAX_SLOTS = 8     # device.h kMaxAggs
    _TIMES = ("device_ms", "scan_kernel_ms", "filter_kernel_ms", "agg_kernel_ms", "filter_bytes", "agg_bytes")

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int,
                 stats_filters=None):
        """stats_filters: the FILTER clauses (None = unfiltered) whose programs count in numEntriesScannedInFilter
        (default: all) -- GpuCaseAggregationOperator's original filters, not its CASE-branch programs."""
        if query.group_by:
            raise UnsupportedOnGpu("FILTER clause with GROUP BY (FilteredGroupByOperator)")
        self.query = query
        self.segments = list(segments)
        groups = {}
        for i, ag in enumerate(query.aggregations):
            groups.setdefault(ag.filter, []).append(i)
        filters = []
        for flt in groups:
            if flt is None:
                filters.append(query.filter)
            elif query.filter is None:
                filters.append(flt)
            else:
                filters.append(FilterContext.AND(query.filter, flt))
        self.one_pass = None
        self.parts = []
        if 1 < len(filters) <= self._MAX_PROGRAMS:
            order = list(groups)
            sub = QueryContext(query.table, [], [ag.unfiltered() for ag in query.aggregations], None, [],
                               limit=query.limit, options=dict(query.options))
            op = GpuCombineOperator(sub, self.segments, num_groups_limit,
                                    programs=(filters, [order.index(ag.filter) for ag in query.aggregations]))
            op.stats_programs = _stats_mask(order, stats_filters)
            if len(op.prims) <= self._MAX_SLOTS:
                self.one_pass = op
                return
        self.part_counts = []
        for (key, idxs), f in zip(groups.items(), filters):
            sub = QueryContext(query.table, [], [query.aggregations[i].unfiltered() for i in idxs], f, [],
                               limit=query.limit, options=dict(query.options))
            self.parts.append((idxs, GpuCombineOperator(sub, self.segments, num_groups_limit)))
            self.part_counts.append(stats_filters is None or key in stats_filters)

    def next_block(self):
        if self.one_pass is not None:
            blk = self.one_pass.next_block()
            out = AggregationResultsBlock(self.query.aggregations, blk.results, blk.stats)
            for k in self._TIMES:
                setattr(out, k, getattr(blk, k, 0))
            return out
        results = [None] * len(self.query.aggregations)
        stats = ExecutionStatistics()
        times = dict.fromkeys(self._TIMES, 0)
        for (idxs, op), blk, counts in zip(self.parts, _run_parts(self.parts), self.part_counts):
            for j, i in enumerate(idxs):
                results[i] = blk.results[j]
            s = blk.stats
            stats.num_docs_scanned += s.num_docs_scanned
            stats.num_entries_scanned_in_filter += s.num_entries_scanned_in_filter if counts else 0
            stats.num_entries_scanned_post_filter += s.num_entries_scanned_post_filter
            stats.num_total_docs = s.num_total_docs
            stats.num_segments_processed = s.num_segments_processed
            stats.num_segments_matched = max(stats.num_segments_matched, s.num_segments_matched)
            for k in self._TIMES:
                times[k] += getattr(blk, k, 0) or 0
        blk = AggregationResultsBlock(self.query.aggregations, results, stats)
        for k, v in times.items():
            setattr(blk, k, v)
        return blk

    def close(self):
        if self.one_pass is not None:
            self.one_pass.close()
        for _, op in self.parts:
            op.close()


_HOLDER_DEFAULTS = {"count": 0, "min": float("inf"), "max": float("-inf"), "avg": (0.0, 0),
                    "minmaxrange": (float("inf"), float("-inf"))}


def _holder_default(ag, sample):
    """The value GroupByResultHolder.ensureCapacity leaves in a group no doc of the function's filter reached
    (DoubleGroupByResultHolder: the function's default -- 0.0 for SUM, +/-inf for MIN/MAX; count 0; an empty
    HLL). ``sample`` is another group's intermediate of the same function, to keep its type (exact int sums)."""
    f = ag.function
    if f == "sum":
        return 0 if isinstance(sample, int) else 0.0
    if f in ("distinctcounthll", "distinctcountrawhll"):
        return np.zeros(1 << ag.log2m, dtype=np.uint8)
    return _HOLDER_DEFAULTS[f]


class GpuFilteredGroupByOperator:
    """FilteredGroupByOperator (pinot-core/.../operator/query/FilteredGroupByOperator.java:110-176) over all
    segments. The infos of AggregationFunctionUtils.buildFilteredAggregationInfos (:312-400) -- one per distinct
    FILTER (main AND filter), then the main filter with the non-filtered functions, which a group-by always gets
    so every group of the main filter exists (unless ``filteredAggregationsSkipEmptyGroups``) -- become the
    filter programs of ONE GPU plan: one filter launch writes a tile mask per info, one aggregation launch keys
    every info's docs into one shared dense key space (the shared DictionaryBasedGroupKeyGenerator) and applies
    each function to its own info's docs only (phip_aggregation.program; COUNTs count their info's docs in their
    own table row). A group's presence is the union over the infos; a function whose filter never reached a group
    keeps its holder default (0 / +inf / -inf / empty registers, read back from the untouched table rows).
    numDocsScanned / post-filter entries sum over the infos (each projects the group-by columns plus its
    functions' arguments). The server-level trim runs on the device over the complete groups.

    numGroupsLimit: the shared generator numbers groups first-seen over info 0's docs, then info 1's, ... per
    segment; the device limit pass orders (segment, key) entries by (info, doc) exactly so. The info order is
    the reference's for one filtered info (filtered infos first, the main info last); with several filtered
    infos the reference iterates a HashMap of FilterContexts, so which keys survive a reached limit is not defined
    by the query: such an execution raises UnsupportedOnGpu (the plan maker's CPU operator answers it).

    More than 8 infos or more than 8 primitive slots run one GPU group-by per info, merged by key on the host
    (the round-2 path); that path raises UnsupportedOnGpu when an info reaches numGroupsLimit."""

    _MAX_PROGRAMS = 8  # device.h kMaxPrograms
    _MAX_SLOTS = 8     # device.h kMaxAggs

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int,
                 device_trim: bool = True, stats_filters=None):
        self.query = query
        self.segments = list(segments)
        self.num_groups_limit = num_groups_limit
        self.device_trim = device_trim
        main, infos = [], {}
        for i, ag in enumerate(query.aggregations):
            if ag.filter is None:
                main.append(i)
            else:
                infos.setdefault(ag.filter, []).append(i)
        order = list(infos.items())
        self.num_filtered_infos = len(order)
        skip = str(query.options.get("filteredAggregationsSkipEmptyGroups", "false")).lower() == "true"
        if main or not skip:
            order.append((None, main))
        filters = []
        for flt, _ in order:
            if flt is None:
                filters.append(query.filter)
            elif query.filter is None:
                filters.append(flt)
            else:
                filters.append(FilterContext.AND(query.filter, flt))
        self.one_pass = None
        self.parts = []
        self.part_counts = []
        if len(order) <= self._MAX_PROGRAMS:
            prog_of = {}
            for p, (_, idxs) in enumerate(order):
                for i in idxs:
                    prog_of[i] = p
            sub = QueryContext(query.table, [], [ag.unfiltered() for ag in query.aggregations], None,
                               list(query.group_by), list(query.order_by), limit=query.limit,
                               options=dict(query.options))
            op = GpuCombineOperator(sub, self.segments, num_groups_limit,
                                    programs=(filters, [prog_of[i] for i in range(len(query.aggregations))]))
            op.stats_programs = _stats_mask([flt for flt, _ in order], stats_filters)
            if len(op.prims) <= self._MAX_SLOTS:
                op.device_trim = device_trim
                op.trim_query = query  # ORDER BY resolves against the FILTER'ed functions
                self.one_pass = op
                return
            op.close()
        for (flt, idxs), f in zip(order, filters):
            # an info without functions still generates its groups: a COUNT rides along and is dropped
            aggs = [query.aggregations[i].unfiltered() for i in idxs] or [AggregationInfo("count", None)]
            sub = QueryContext(query.table, [], aggs, f, list(query.group_by), limit=query.limit,
                               options=dict(query.options))
            op = GpuCombineOperator(sub, self.segments, num_groups_limit)
            op.device_trim = False
            self.parts.append((idxs, op))
            self.part_counts.append(stats_filters is None or flt in stats_filters)

    def _wrap(self, blk):
        out = GroupByResultsBlock(self.query.aggregations, list(self.query.group_by), blk.groups, blk.stats,
                                  blk.num_groups_limit_reached)
        out.num_groups_trimmed = getattr(blk, "num_groups_trimmed", False)
        out.key_types = getattr(blk, "key_types", None)
        for k in GpuFilteredAggregationOperator._TIMES + ("fused",):
            setattr(out, k, getattr(blk, k, 0))
        out.segment_docs_matched = getattr(blk, "segment_docs_matched", None)
        return out

    def next_block(self):
        if self.one_pass is not None:
            blk = self.one_pass.next_block()
            if blk.num_groups_limit_reached and self.num_filtered_infos >= 2:
                # which keys a segment keeps past the limit depends on the order the shared generator sees the infos
                # in, and the reference iterates a HashMap of FilterContexts: not defined by the query
                raise UnsupportedOnGpu("numGroupsLimit reached by a FILTER + GROUP BY query with two or more "
                                       "filtered infos (the reference's info order is HashMap order)")
            return self._wrap(blk)
        from .reduce import trim_groups
        na = len(self.query.aggregations)
        stats = ExecutionStatistics()
        per_part = []
        keys = {}
        device_ms = 0.0
        for (idxs, op), blk, counts in zip(self.parts, _run_parts(self.parts), self.part_counts):
            if blk.num_groups_limit_reached:
                raise UnsupportedOnGpu("numGroupsLimit reached by a FILTER + GROUP BY query of more than 8 infos")
            per_part.append((idxs, blk.groups))
            for k in blk.groups:
                keys.setdefault(k, None)
            s = blk.stats
            stats.num_docs_scanned += s.num_docs_scanned
            stats.num_entries_scanned_in_filter += s.num_entries_scanned_in_filter if counts else 0
            stats.num_entries_scanned_post_filter += s.num_entries_scanned_post_filter
            stats.num_total_docs = s.num_total_docs
            stats.num_segments_processed = s.num_segments_processed
            stats.num_segments_matched = max(stats.num_segments_matched, s.num_segments_matched)
            device_ms += getattr(blk, "device_ms", 0.0) or 0.0
        groups = {k: [None] * na for k in keys}
        for idxs, pg in per_part:
            for j, i in enumerate(idxs):
                ag = self.query.aggregations[i]
                sample = next(iter(pg.values()))[j] if pg else None
                dflt = _holder_default(ag, sample)
                for k, vals in groups.items():
                    v = pg.get(k)
                    vals[i] = v[j] if v is not None else (dflt.copy() if isinstance(dflt, np.ndarray) else dflt)
        blk = GroupByResultsBlock(self.query.aggregations, list(self.query.group_by), groups, stats, False)
        blk.num_groups_trimmed = False
        blk.key_types = self.parts[0][1].key_types() if self.parts else None
        if self.device_trim:
            blk = trim_groups(self.query, blk, getattr(self, "segment_trim", None))
        blk.device_ms = device_ms
        blk.segment_docs_matched = None  # (summed per info below it: the checks take the segments' docs instead)
        return blk

    # -- multi-GPU servers: the one-pass plan hands out its dense partial table like any group-by
    def execute_partial(self):
        return self.one_pass.execute_partial() if self.one_pass is not None else None

    def abandon_partial(self):
        if self.one_pass is not None:
            self.one_pass.abandon_partial()

    def finish(self, merged):
        return self._wrap(self.one_pass.finish(merged))

    def close(self):
        if self.one_pass is not None:
            self.one_pass.close()
        for _, op in self.parts:
            op.close()


def _is_case(e):
    return isinstance(_strip_cast(e), Function) and _strip_cast(e).name == "case"


def _and(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return FilterContext.AND(a, b)


class GpuCaseAggregationOperator:
    """Aggregations over ``CASE WHEN c1 THEN e1 [WHEN c2 THEN e2 ...] ELSE e END`` (the CASE-based sums of
    SURVEY.md §8f f1; CaseTransformFunction picks, per doc, the THEN of the first WHEN that holds, else the ELSE).

    The GPU never materialises the CASE column: branch k holds exactly the docs of
    ``c_k AND NOT (c_1 OR ... OR c_{k-1})`` (ELSE: ``NOT (c_1 OR ... OR c_n)``), so the aggregation splits into
    filtered aggregations of the branch values -- ``agg(e_k) FILTER(WHERE branch_k)`` for an expression,
    ``COUNT(*) FILTER(WHERE branch_k)`` for a literal -- which run through the filtered operators (one GPU pass
    per distinct filter) and are folded back per group: SUM = sum of branch sums + literal x branch count,
    MIN / MAX over the branch results (a literal counts when its branch has docs), AVG = that sum over
    COUNT(*), COUNT(CASE ...) = COUNT(*). The reference's statistics are those of ONE pass per original filter
    (an unfiltered CASE query is a plain AggregationOperator / GroupByOperator): hidden ``COUNT(*)`` per
    original filter give numDocsScanned and, times the columns that filter's functions project (CASE
    conditions included), numEntriesScannedPostFilter."""

    _FOLDABLE = ("sum", "min", "max", "avg", "minmaxrange", "count")

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int):
        self.query = query
        inner = []

        def slot(fn, arg, flt, log2m=8):
            a = AggregationInfo(fn, arg, log2m, flt)
            if a not in inner:
                inner.append(a)
            return inner.index(a)

        self.plan = []
        for ag in query.aggregations:
            if ag.argument is None or not _is_case(ag.argument):
                self.plan.append(("pass", slot(ag.function, ag.argument, ag.filter, ag.log2m)))
                continue
            if ag.function not in self._FOLDABLE:
                raise UnsupportedOnGpu(f"{ag.function} over CASE")
            if ag.function == "count":
                self.plan.append(("pass", slot("count", None, ag.filter)))
                continue
            case = _strip_cast(ag.argument)
            conds, vals = list(case.args[0:-1:2]), list(case.args[1:-1:2]) + [case.args[-1]]
            branches = []
            for k, v in enumerate(vals):
                prior = None
                if k:
                    prior = FilterContext.NOT(conds[0] if k == 1 else FilterContext.OR(*conds[:k]))
                cond = conds[k] if k < len(conds) else None
                bflt = _and(ag.filter, _and(cond, prior))
                v = _strip_cast(v)
                if isinstance(v, Literal):
                    if isinstance(v.value, str):
                        raise UnsupportedOnGpu("string literal in a CASE under an aggregation")
                    branches.append(("lit", v.value, slot("count", None, bflt)))
                else:
                    fn = "sum" if ag.function == "avg" else ag.function
                    branches.append(("expr", fn, slot(fn, v, bflt)))
            total = slot("count", None, ag.filter) if ag.function == "avg" else None
            self.plan.append(("case", ag.function, branches, total))
        # statistics: one pass per original filter (FilteredAggregationOperator / FilteredGroupByOperator infos)
        self.stats_slots = []
        gb_cols = set()
        for e in query.group_by:
            gb_cols.update(columns_of(e))
        per_filter = {}
        for ag in query.aggregations:
            cols = per_filter.setdefault(ag.filter, set(gb_cols))
            if ag.argument is not None:
                cols.update(columns_of(ag.argument))
        if query.group_by and None not in per_filter and \
                str(query.options.get("filteredAggregationsSkipEmptyGroups", "false")).lower() != "true":
            per_filter[None] = set(gb_cols)
        for flt, cols in per_filter.items():
            self.stats_slots.append((slot("count", None, flt), len(cols)))
        inner_options = dict(query.options)
        if all(ag.filter is None for ag in query.aggregations):
            inner_options.pop("filteredAggregationsSkipEmptyGroups", None)  # the CASE query's groups = main filter's
        self.inner_query = QueryContext(query.table, [], inner, query.filter, list(query.group_by), [],
                                        limit=query.limit, options=inner_options)
        # numEntriesScannedInFilter: the scans of the original filters' programs only (the hidden COUNT(*) slots'),
        # not those of the CASE-branch programs, which re-evaluate the filter AND a WHEN condition
        stats_filters = set(per_filter)
        if query.group_by:
            self.inner = GpuFilteredGroupByOperator(self.inner_query, segments, num_groups_limit,
                                                    stats_filters=stats_filters)
        else:
            self.inner = GpuFilteredAggregationOperator(self.inner_query, segments, num_groups_limit,
                                                        stats_filters=stats_filters)

    def _fold(self, vals):
        out = []
        for p in self.plan:
            if p[0] == "pass":
                out.append(vals[p[1]])
                continue
            _, fn, branches, total = p
            if fn in ("sum", "avg"):
                acc = 0
                for kind, x, s in branches:
                    acc = acc + (x * vals[s] if kind == "lit" else vals[s])
                if not all(isinstance(x, int) for kind, x, s in branches if kind == "lit") or \
                        not all(isinstance(vals[s], int) for kind, x, s in branches if kind == "expr"):
                    acc = float(acc)
                out.append(acc if fn == "sum" else (acc, int(vals[total])))
                continue
            lo, hi = float("inf"), float("-inf")
            for kind, x, s in branches:
                if kind == "lit":
                    if vals[s] > 0:
                        lo, hi = min(lo, float(x)), max(hi, float(x))
                elif fn == "minmaxrange":
                    lo, hi = min(lo, vals[s][0]), max(hi, vals[s][1])
                else:
                    lo, hi = min(lo, vals[s]), max(hi, vals[s])
            out.append(lo if fn == "min" else hi if fn == "max" else (lo, hi))
        return out

    def _stats(self, stats, counts):
        stats.num_docs_scanned = sum(int(c) for c, _ in counts)
        stats.num_entries_scanned_post_filter = sum(int(c) * ncols for c, ncols in counts)
        return stats

    def next_block(self):
        from .reduce import trim_groups
        blk = self.inner.next_block()
        if not self.query.group_by:
            counts = [(blk.results[s], n) for s, n in self.stats_slots]
            out = AggregationResultsBlock(self.query.aggregations, self._fold(blk.results), self._stats(blk.stats, counts))
            out.device_ms = getattr(blk, "device_ms", 0.0)
            return out
        counts = [(sum(v[s] for v in blk.groups.values()), n) for s, n in self.stats_slots]
        groups = {k: self._fold(v) for k, v in blk.groups.items()}
        out = GroupByResultsBlock(self.query.aggregations, list(self.query.group_by), groups,
                                  self._stats(blk.stats, counts), blk.num_groups_limit_reached)
        out.num_groups_trimmed = False
        out.key_types = getattr(blk, "key_types", None)
        out = trim_groups(self.query, out, getattr(self, "segment_trim", None))
        out.device_ms = getattr(blk, "device_ms", 0.0)
        out.segment_docs_matched = getattr(blk, "segment_docs_matched", None)
        return out

    def close(self):
        self.inner.close()


# ------------------------------------------------------------------------------ query options
class QueryOptionError(ValueError):
    """A malformed query option (QueryOptionsUtils's IllegalArgumentException: a BadQueryRequest)."""


_INT = re.compile(r"[+-]?[0-9]+\Z")


def _int_option(options, key, min_value=None):
    """QueryOptionsUtils.uncheckedParseInt / checkedParseInt (pinot-common/.../utils/config/QueryOptionsUtils.java:
    366-402): Integer.parseInt of the option, at least ``min_value`` when given; None when absent."""
    v = options.get(key)
    if v is None:
        return None
    v = str(v)
    if not _INT.match(v) or not -(1 << 31) <= int(v) < (1 << 31):
        raise QueryOptionError(f"{key} must be an integer, got: {v}")
    x = int(v)
    if min_value is not None and x < min_value:
        raise QueryOptionError(f"{key} must be a number between {min_value} and 2^31-1, got: {v}")
    return x


def _long_option_positive(options, key):
    """QueryOptionsUtils.checkedParseLongPositive (QueryOptionsUtils.java:410-430): Long.parseLong, at least 1."""
    v = options.get(key)
    if v is None:
        return None
    v = str(v)
    if not _INT.match(v) or not 1 <= int(v) < (1 << 63):
        raise QueryOptionError(f"{key} must be a number between 1 and 2^63-1, got: {v}")
    return int(v)


# The running query's end time (QueryContext.getEndTimeMs, wall-clock ms): set by the outermost operator for the
# length of its next_block (_DeadlineOperator), read by every plan execution under it and by the multi-plan
# operators between their plans (BaseSingleBlockCombineOperator.java:133-144 checks it between blocks).
_END_TIME_MS = contextvars.ContextVar("pinot_amd_end_time_ms", default=None)


def check_deadline(where: str):
    """QueryTimeoutError when the running query's end time has passed (a no-op without timeoutMs)."""
    end = _END_TIME_MS.get()
    if end is not None and time.time() * 1000.0 > end:
        raise QueryTimeoutError(_lib.PHIP_ERR_TIMEOUT, f"query timed out ({where})")


class _DeadlineOperator:
    """The outermost operator of a query with timeoutMs: each next_block runs under endTimeMs = its start +
    timeoutMs (the server's QueryContext end time), which every library execution under it receives
    (phip_plan_set_deadline) and the multi-plan operators check between plans."""

    def __init__(self, op, timeout_ms):
        self.op, self.timeout_ms = op, timeout_ms

    def next_block(self):
        token = _END_TIME_MS.set(time.time() * 1000.0 + self.timeout_ms)
        try:
            check_deadline("before execution")
            return self.op.next_block()
        finally:
            _END_TIME_MS.reset(token)

    def close(self):
        self.op.close()

    def __getattr__(self, name):
        if name == "op":
            raise AttributeError(name)
        return getattr(self.op, name)


def _bool_option(options, key) -> bool:
    """Boolean.parseBoolean of a query option (only a case-insensitive "true" is true)."""
    return str(options.get(key, "")).strip().lower() == "true"


def table_capacity(limit: int, min_num_groups: int) -> int:
    """GroupByUtils.getTableCapacity (pinot-core/.../util/GroupByUtils.java:55-58): max(limit * 5, minNumGroups)."""
    by_limit = int(limit) * 5
    return (1 << 31) - 1 if by_limit > (1 << 31) - 1 else max(by_limit, int(min_num_groups))


def indexed_table_trim_threshold(trim_size: int, trim_threshold: int) -> int:
    """GroupByUtils.getIndexedTableTrimThreshold (:60-70): trim disabled (Integer.MAX_VALUE) when the threshold is
    non-positive or above 10^9 or trimSize above 5 x 10^8; else max(threshold, 2 x trimSize)."""
    if trim_threshold <= 0 or trim_threshold > MAX_TRIM_THRESHOLD or trim_size > MAX_TRIM_THRESHOLD // 2:
        return (1 << 31) - 1
    return max(trim_threshold, 2 * trim_size)


def _source_segments(op):
    """The segments (GpuSegment) an operator's per-segment GroupByOperators key: the star-tree documents for a
    star-tree operator, the inner operator's for a CASE operator."""
    return list(op.segments) if hasattr(op, "segments") else list(op.inner.segments)


def _set_segment_trim(op, n):
    """Make ``op`` (an operator over ONE segment) trim its groups as that segment's GroupByOperator would with
    minSegmentGroupTrimSize = n: keep the top getTableCapacity(limit, n) by the ORDER BY."""
    op.segment_trim = n
    for attr in ("one_pass", "inner"):
        sub = getattr(op, attr, None)
        if isinstance(sub, GpuCombineOperator):
            sub.segment_trim = n


class GpuGroupByCombineOperator:
    """The result-changing group-by options of the combine, over any group-by operator of the plan maker:

      minSegmentGroupTrimSize  GroupByOperator.getNextBlock (pinot-core/.../operator/query/GroupByOperator.java:
                               118-133): with ORDER BY and a positive size, a segment holding more than
                               trimSize = getTableCapacity(limit, size) groups keeps only its top trimSize
                               (TableResizer.trimInSegmentResults) before the combine merges it.
      groupTrimThreshold       the combine's IndexedTable resizes to the server trimSize whenever it holds
                               getIndexedTableTrimThreshold(trimSize, threshold) records
                               (SimpleIndexedTable.upsert; GroupByUtils.java:60-70,130-145).

    The all-segment GPU operator answers first. Per segment s it reports the docs its filter passed; its group
    records are at most b_s = min(matched docs, key space, numGroupsLimit). When every b_s is within the segment
    trimSize no segment trims, and the one-launch answer is the reference's; otherwise the query runs once per
    segment (each plan trimming its own groups on the device, top trimSize by the ORDER BY) and the blocks merge
    on the host, as the combine merges them. A combine that can reach the trim threshold with records of two or
    more segments resizes mid-merge, and which partial values then survive depends on the order the reference's
    worker threads upsert in (ConcurrentIndexedTable): that query raises UnsupportedOnGpu so the plan maker
    answers it on the CPU (a one-segment combine holds every group once with its exact value, so its resizes keep
    the exact top trimSize: the GPU answers it)."""

    def __init__(self, query: QueryContext, inner, make_op):
        self.query = query
        self.inner = inner
        self.make_op = make_op
        self.segments = _source_segments(inner)
        o = query.options
        self.limit = int(o.get("numGroupsLimit", DEFAULT_NUM_GROUPS_LIMIT))
        min_seg = int(o.get("minSegmentGroupTrimSize", DEFAULT_MIN_SEGMENT_GROUP_TRIM_SIZE))
        self.min_seg = min_seg if (query.order_by and min_seg > 0) else None
        self.seg_trim = table_capacity(query.limit, min_seg) if self.min_seg else None
        min_srv = int(o.get("minServerGroupTrimSize", DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE))
        srv_trim = table_capacity(query.limit, min_srv) if min_srv > 0 else (1 << 31) - 1
        thr = int(o.get("groupTrimThreshold", DEFAULT_GROUPBY_TRIM_THRESHOLD))
        self.threshold = indexed_table_trim_threshold(srv_trim, thr) if query.order_by else (1 << 31) - 1
        self.key_space = []
        for seg in self.segments:
            ks = 1
            for e in query.group_by:
                m = seg.column_metadata(e.name)
                ks *= m.cardinality if m.has_dictionary else max(seg.num_docs, 1)
            self.key_space.append(ks)
        self.per_segment = None

    @staticmethod
    def needed(query: QueryContext) -> bool:
        """Whether either option can change the result of ``query`` (its options resolved by the plan maker)."""
        if not query.group_by or not query.order_by:
            return False
        o = query.options
        if int(o.get("minSegmentGroupTrimSize", DEFAULT_MIN_SEGMENT_GROUP_TRIM_SIZE)) > 0:
            return True
        min_srv = int(o.get("minServerGroupTrimSize", DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE))
        srv_trim = table_capacity(query.limit, min_srv) if min_srv > 0 else (1 << 31) - 1
        thr = int(o.get("groupTrimThreshold", DEFAULT_GROUPBY_TRIM_THRESHOLD))
        return indexed_table_trim_threshold(srv_trim, thr) < (1 << 31) - 1

    def _bounds(self, blk):
        docs = getattr(blk, "segment_docs_matched", None)
        if docs is None or len(docs) != len(self.segments):
            docs = [s.num_docs for s in self.segments]
        return [min(int(d), ks, self.limit) for d, ks in zip(docs, self.key_space)]

    def _check_threshold(self, records, distinct=None, key_space=None):
        """ConcurrentIndexedTable resizes once its map holds trimThreshold DISTINCT keys (ConcurrentIndexedTable.java:
        63-67), so the combine's bound is the per-segment records' sum capped by the distinct keys of the merged
        result (exact when the block is untrimmed) or by the query-global key space (the union of the segments'
        dictionaries)."""
        nonempty = sum(1 for r in records if r > 0)
        bound = sum(records)
        if distinct is not None:
            bound = min(bound, distinct)
        if key_space:
            bound = min(bound, key_space)
        if nonempty >= 2 and bound >= self.threshold:
            raise UnsupportedOnGpu(
                f"the combine can reach its trim threshold ({self.threshold} distinct records from {nonempty} "
                "segments): which partial groups survive depends on the reference's thread interleaving")

    def _run_per_segment(self):
        from .reduce import trim_groups
        if self.per_segment is None:
            self.per_segment = []
            for seg in self.segments:
                op = self.make_op([seg])
                _set_segment_trim(op, self.min_seg)
                self.per_segment.append(op)
        blocks = []
        for op in self.per_segment:  # (the combine checks the query's end time between its segments' blocks)
            check_deadline("between per-segment group-by plans")
            blocks.append(op.next_block())
        aggs = self.query.aggregations
        groups, stats, reached = {}, ExecutionStatistics(), False
        times = dict.fromkeys(GpuFilteredAggregationOperator._TIMES, 0)
        for b in blocks:  # GroupByCombineOperator: every segment's records upserted into one table
            for k, v in b.groups.items():
                groups[k] = v if k not in groups else [merge_intermediate(a.function, x, y)
                                                       for a, x, y in zip(aggs, groups[k], v)]
            stats.merge(b.stats)
            reached |= bool(b.num_groups_limit_reached)
            for k in times:
                times[k] += getattr(b, k, 0) or 0
        self._check_threshold([len(b.groups) for b in blocks], distinct=len(groups))
        out = GroupByResultsBlock(aggs, list(self.query.group_by), groups, stats, reached)
        out.key_types = getattr(blocks[0], "key_types", None) if blocks else None
        out.num_groups_trimmed = False
        out = trim_groups(self.query, out)  # the server-level trim of the combine
        for k, v in times.items():
            setattr(out, k, v)
        out.segment_trimmed = True
        return out

    def next_block(self):
        blk = self.inner.next_block()
        bounds = self._bounds(blk)
        if self.seg_trim is not None and any(b > self.seg_trim for b in bounds):
            return self._run_per_segment()
        if self.seg_trim is not None:
            bounds = [min(b, self.seg_trim) for b in bounds]
        # (num_groups: a columnar block's count without building its {key: intermediates} view, ~0.1 ms at 800 groups)
        distinct = None if getattr(blk, "num_groups_trimmed", True) else blk.num_groups
        self._check_threshold(bounds, distinct, getattr(blk, "key_space", None))
        return blk

    def close(self):
        self.inner.close()
        for op in self.per_segment or []:
            op.close()

    def __getattr__(self, name):
        # the inner operator's surface (execute_partial / finish for a multi-GPU server's merge, key_types, ...);
        # a multi-GPU merge applies neither check: its combine spans the GPUs
        if name == "inner":
            raise AttributeError(name)
        return getattr(self.inner, name)


class GpuPlanWithCpuFallback:
    """A GPU group-by operator whose execution may still refuse the query (UnsupportedOnGpu from next_block: the
    combine's trim threshold, numGroupsLimit reached under several FILTER infos): the configured CPU plan maker's
    operator answers it instead."""

    def __init__(self, gpu_op, cpu_plan_maker, query, segments):
        self.gpu_op, self.cpu_plan_maker, self.query, self.segments = gpu_op, cpu_plan_maker, query, segments

    def next_block(self):
        try:
            return self.gpu_op.next_block()
        except UnsupportedOnGpu:
            return self.cpu_plan_maker.make_instance_plan(self.query, self.segments).next_block()

    def close(self):
        self.gpu_op.close()

    def __getattr__(self, name):
        # the GPU operator's surface (execute_partial / finish for a multi-GPU merge, run_raw, key_types, ...)
        if name == "gpu_op":
            raise AttributeError(name)
        return getattr(self.gpu_op, name)


def use_gpu_option(query: QueryContext, default: bool) -> bool:
    """The ``useGpu`` query option (``SET useGpu = true;`` / queryOptions), parsed as Java's
    Boolean.parseBoolean (only a case-insensitive "true" is true); absent -> the plan maker's default."""
    v = query.options.get("useGpu")
    if v is None:
        return default
    return str(v).strip().lower() == "true"


def _query_columns(query: QueryContext):
    cols = set()
    if query.filter is not None:
        cols.update(query.filter.columns())
    for ag in query.aggregations:
        if ag.argument is not None:
            cols.update(columns_of(ag.argument))
        if ag.filter is not None:
            cols.update(ag.filter.columns())
    for e in query.group_by:
        cols.update(columns_of(e))
    for e, _ in query.select:
        cols.update(c for c in columns_of(e) if c != "*")
    return cols


def _has_nulls(query: QueryContext, segments) -> bool:
    """enableNullHandling with a null value vector on any column the query reads in any segment: the star-tree
    then stays unused, as StarTreeUtils.isFitForStarTree decides per segment (StarTreeUtils.java:380-400)."""
    if not null_handling_enabled(query):
        return False
    cols = _query_columns(query)
    return any(s.has_null_vector(c) for s in segments for c in cols if s.has_column(c))


_NULLABLE = ("sum", "min", "max", "avg", "minmaxrange", "count")  # NullableSingleInputAggregationFunction subclasses


def _null_handling_operator(query: QueryContext, segments, limit):
    """enableNullHandling (QueryContext.isNullHandlingEnabled). The filter side needs nothing here: every
    GpuCombineOperator compiles its programs three-valued (_three_valued) and keys null group-by docs as the null key
    (GpuCombineOperator.null_keys). This picks the aggregation side:
      * aggregation only -> GpuNullHandlingAggregationOperator;
      * group-by: GpuNullHandlingGroupByOperator when a nullable function's column has a null vector in some segment
        (per-group null results) or a function has a FILTER (a group its info never reached is null); else the
        regular operators (null keys, if any, come from the library). CASE with GROUP BY stays UnsupportedOnGpu;
      * selection: the selected columns must be null-free (the reference returns nulls for null values);
    None = the regular operators apply."""
    def null_cols(exprs):
        cols = set()
        for e in exprs:
            cols.update(c for c in columns_of(e) if c != "*")
        return {c for c in cols if any(s.has_column(c) and s.has_null_vector(c) for s in segments)}

    if any(ag.argument is not None and _is_case(ag.argument) for ag in query.aggregations):
        raise UnsupportedOnGpu("enableNullHandling with CASE aggregations")
    if query.is_selection:
        if null_cols([e for e, _ in query.select]):
            raise UnsupportedOnGpu("enableNullHandling: selected columns with null values")
        return None
    nullable_args = [ag.argument for ag in query.aggregations if ag.function in _NULLABLE and ag.argument is not None]
    if query.group_by:
        if any(ag.filter is not None for ag in query.aggregations):  # (unreached groups: null holders)
            return GpuNullHandlingGroupByOperator(query, segments, limit, null_cols(nullable_args))
        if null_cols(nullable_args):
            return GpuNullHandlingGroupByOperator(query, segments, limit, null_cols(nullable_args))
        return None
    return GpuNullHandlingAggregationOperator(query, segments, limit, null_cols(nullable_args))


class GpuNullHandlingGroupByOperator:
    """GROUP BY under enableNullHandling with nullable functions over columns that hold nulls (DefaultGroupByExecutor
    with null handling, DefaultGroupByExecutor.java:106-116: NoDictionary*GroupKeyGenerator keys the matched docs --
    null group-by docs as the null key -- and every NullableSingleInputAggregationFunction skips the docs where its
    argument is null, its group result null when none was left: SumAggregationFunction.aggregateGroupBySV under null
    handling, CountAggregationFunction for COUNT(col)).

    One GPU plan of filter programs over one shared key space: program 0 is the query's filter (every matched doc: it
    generates the groups and numbers them first-seen in doc order for numGroupsLimit, the library's limit pass
    ordering (segment, key) by (program, doc)), program p > 0 is ``filter AND c IS NOT NULL ...`` for one set of
    null-holding argument columns, carrying the functions over them plus a hidden COUNT(*) (their non-null docs per
    group: 0 = a null result; COUNT(col) is that count). Every program's docs are program 0's, so the groups are
    program 0's. The statistics are the reference's single pass: numDocsScanned = program 0's matched docs
    (phip_result.program_docs_matched), post-filter entries = those x the distinct projected columns, filter scans of
    program 0 only. The server-level trim runs on the host after the nulls are restored (the device would order a
    null result by its holder default).

    With FILTER clauses (FilteredGroupByOperator.java:110-176 under null handling) the infos of
    GpuFilteredGroupByOperator -- one per distinct FILTER, then the main filter's -- are programs 0..I-1 in that
    order (first-seen over info 0's docs, then info 1's, ...), each IS NOT NULL set a program ``info filter AND c IS
    NOT NULL ...`` after them, and every nullable function carries the non-null count of its own program: its holder
    is an ObjectGroupByResultHolder (SumAggregationFunction.createGroupByResultHolder :62-67), so a group its info
    never reached is null too. Statistics sum over the infos (each projecting the group-by columns plus its
    functions' arguments)."""

    _MAX_PROGRAMS = 8

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int, null_cols):
        self.query = query
        self.segments = list(segments)
        main, by_filter = [], {}
        for i, ag in enumerate(query.aggregations):
            if ag.filter is None:
                main.append(i)
            else:
                by_filter.setdefault(ag.filter, []).append(i)
        order = list(by_filter.items())
        self.num_filtered_infos = len(order)
        skip = str(query.options.get("filteredAggregationsSkipEmptyGroups", "false")).lower() == "true"
        if main or not skip or not order:
            order.append((None, main))
        filtered = self.num_filtered_infos > 0
        info_filters = [query.filter if flt is None else _and(query.filter, flt) for flt, _ in order]
        info_of = {i: p for p, (_, idxs) in enumerate(order) for i in idxs}
        keys = [(p, ()) for p in range(len(order))]  # programs 0..I-1: the infos (their docs: every group)
        aggs, progs = [], []
        counts = {}

        def program_of(p, cols):
            k = (p, tuple(sorted(cols)))
            if k not in keys:
                keys.append(k)
            return keys.index(k)

        def count_for(p):
            if p not in counts:
                counts[p] = len(aggs)
                aggs.append(AggregationInfo("count", None))
                progs.append(p)
            return counts[p]

        self.slots = []  # per original aggregation: (value index, non-null count index or None)
        for i, ag0 in enumerate(query.aggregations):
            ag = ag0.unfiltered()
            p = info_of[i]
            cols = [c for c in columns_of(ag.argument) if c in null_cols] if ag.argument is not None else []
            nullable = ag.function in _NULLABLE and ag.argument is not None
            if not nullable or (not cols and not filtered):
                self.slots.append((len(aggs), None))
                aggs.append(ag)
                progs.append(p)
                continue
            q = program_of(p, cols) if cols else p
            if ag.function == "count":
                self.slots.append((count_for(q), None))
                continue
            if ag.function == "avg":  # (its own count is the non-null count)
                self.slots.append((len(aggs), "avg"))
                aggs.append(ag)
                progs.append(q)
                continue
            ci = count_for(q)
            self.slots.append((len(aggs), ci))
            aggs.append(ag)
            progs.append(q)
        if len(keys) > self._MAX_PROGRAMS:
            raise UnsupportedOnGpu("enableNullHandling GROUP BY: more than 8 infos and sets of null-holding argument "
                                   "columns")
        filters = []
        for p, cols in keys:
            nn = [FilterContext.PRED(Predicate("IS_NOT_NULL", Identifier(c))) for c in cols]
            parts = ([info_filters[p]] if info_filters[p] is not None else []) + nn
            filters.append(None if not parts else parts[0] if len(parts) == 1 else FilterContext.AND(*parts))
        sub = QueryContext(query.table, [], aggs, None, list(query.group_by), [], limit=query.limit,
                           options=dict(query.options))
        self.op = GpuCombineOperator(sub, self.segments, num_groups_limit, programs=(filters, progs))
        if len(self.op.prims) > 8:  # (device.h kMaxAggs primitive slots: the functions plus their non-null counts)
            self.op.close()
            raise UnsupportedOnGpu("enableNullHandling GROUP BY: more than 8 aggregation slots with the non-null counts")
        self.num_infos = len(order)
        self.op.stats_programs = (1 << len(order)) - 1  # (the infos' filter scans: the reference's passes)
        self.op.device_trim = False
        gb = set()
        for e in query.group_by:
            gb.update(columns_of(e))
        self.info_projected = []  # per info: the group-by columns plus its functions' arguments
        for _, idxs in order:
            proj = set(gb)
            for i in (idxs if filtered else range(len(query.aggregations))):
                ag = query.aggregations[i]
                if ag.argument is not None:
                    proj.update(c for c in columns_of(ag.argument) if c != "*")
            self.info_projected.append(len(proj))
        self.num_projected = self.info_projected[-1]

    def next_block(self):
        from .reduce import trim_groups
        blk = self.op.next_block()
        if blk.num_groups_limit_reached and self.num_filtered_infos >= 2:
            raise UnsupportedOnGpu("numGroupsLimit reached by a FILTER + GROUP BY query with two or more filtered "
                                   "infos (the reference's info order is HashMap order)")
        groups = {}
        for key, vals in blk.groups.items():
            groups[key] = [None if (ci == "avg" and vals[vi][1] == 0) or (isinstance(ci, int) and vals[ci] == 0)
                           else vals[vi] for vi, ci in self.slots]
        stats = dataclasses.replace(blk.stats)
        if blk.program_docs_matched:
            docs = [int(blk.program_docs_matched[p]) for p in range(self.num_infos)]
        else:
            docs = [stats.num_docs_scanned]
        stats.num_docs_scanned = sum(docs)
        stats.num_entries_scanned_post_filter = sum(d * n for d, n in zip(docs, self.info_projected))
        out = GroupByResultsBlock(self.query.aggregations, list(self.query.group_by), groups, stats,
                                  blk.num_groups_limit_reached)
        out.key_types = getattr(blk, "key_types", None)
        for k in GpuFilteredAggregationOperator._TIMES + ("fused",):
            setattr(out, k, getattr(blk, k, 0))
        out.segment_docs_matched = None
        if self.query.order_by:
            out = trim_groups(self.query, out)
        return out

    def close(self):
        self.op.close()


class GpuNullHandlingAggregationOperator:
    """Aggregation-only query under enableNullHandling (AggregationOperator / FilteredAggregationOperator with
    NullableSingleInputAggregationFunction: SUM / MIN / MAX / AVG / MINMAXRANGE skip the null values of their
    argument -- of every column it reads, BaseTransformFunction's OR of the arguments' null bitmaps -- and their
    result is null when no non-null value was aggregated (SumAggregationFunction.java:55-160, AvgAggregationFunction
    .java:170-186); COUNT(col) counts the non-null values (CountAggregationFunction.java:44-160); COUNT(*) and
    DISTINCTCOUNTHLL (not nullable) are unchanged).

    On the GPU every nullable function over columns with null vectors becomes a filtered aggregation over
    ``its filter AND col IS NOT NULL ...`` plus a hidden COUNT(*) of the same program, and every original info gets a
    hidden COUNT(*) of its docs: one plan of filter programs (GpuFilteredAggregationOperator). A result whose count is
    0 is None. The statistics are the reference's: numDocsScanned and post-filter entries from the original infos'
    counts (each info projects its functions' input columns), filter scans of the original infos' programs only."""

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int, null_cols):
        self.query = query
        keys = []
        for ag in query.aggregations:
            if ag.filter not in keys:
                keys.append(ag.filter)
        aggs = []
        counts = {}

        def count_for(flt):
            if flt not in counts:
                counts[flt] = len(aggs)
                aggs.append(AggregationInfo("count", None, 8, flt))
            return counts[flt]

        self.info_count = {k: count_for(k) for k in keys}
        self.slots = []  # per original aggregation: (its value's index, the index of its non-null count or None)
        for ag in query.aggregations:
            if ag.function not in _NULLABLE or ag.argument is None:
                self.slots.append((len(aggs), None))
                aggs.append(ag)
                continue
            cols = [c for c in columns_of(ag.argument) if c in null_cols]
            flt = ag.filter
            if cols:
                nn = [FilterContext.PRED(Predicate("IS_NOT_NULL", Identifier(c))) for c in cols]
                parts = ([flt] if flt is not None else []) + nn
                flt = parts[0] if len(parts) == 1 else FilterContext.AND(*parts)
            if ag.function == "count":
                self.slots.append((count_for(flt), None))
                continue
            ci = count_for(flt)
            self.slots.append((len(aggs), ci))
            aggs.append(AggregationInfo(ag.function, ag.argument, ag.log2m, flt))
        sub = QueryContext(query.table, [], aggs, query.filter, [], limit=query.limit, options=dict(query.options))
        if any(a.filter is not None for a in aggs):
            self.op = GpuFilteredAggregationOperator(sub, segments, num_groups_limit, stats_filters=set(keys))
        else:
            self.op = GpuCombineOperator(sub, segments, num_groups_limit)
        self.proj = {}
        for ag in query.aggregations:
            cols = self.proj.setdefault(ag.filter, set())
            if ag.argument is not None:
                cols.update(columns_of(ag.argument))

    def next_block(self):
        blk = self.op.next_block()
        res = blk.results
        out = []
        for vi, ci in self.slots:
            out.append(None if ci is not None and res[ci] == 0 else res[vi])
        stats = dataclasses.replace(blk.stats)
        if not (isinstance(self.op, GpuCombineOperator) and self.op._non_scan_fit()):
            stats.num_docs_scanned = sum(int(res[i]) for i in self.info_count.values())
            stats.num_entries_scanned_post_filter = sum(int(res[i]) * len(self.proj[k])
                                                        for k, i in self.info_count.items())
        o = AggregationResultsBlock(self.query.aggregations, out, stats)
        for k in GpuFilteredAggregationOperator._TIMES:
            setattr(o, k, getattr(blk, k, 0))
        return o

    def close(self):
        self.op.close()


class GpuInstancePlanMaker:
    """``pinot.server.query.executor.plan.maker.class`` plug-in (INTEGRATION.md §3 is the Java
    twin, a subclass of InstancePlanMakerImplV2).

    Routing, as InstancePlanMakerImplV2.makeInstancePlan's override: the query option ``useGpu`` selects the GPU
    operators; ``useGpu=false`` -- or a query outside the GPU subset (UnsupportedOnGpu) -- goes to
    ``cpu_plan_maker.make_instance_plan`` (the reference's own CPU plan, ``super.makeInstancePlan``) when one
    is configured, and raises UnsupportedOnGpu otherwise (this process has no CPU operators of its own).
    ``default_use_gpu`` is the server-level default for queries that do not set the option: the Java twin
    keeps the reference's default (CPU) and a GPU server flips it in its config; this host mirror is built
    for GPU servers and defaults to True."""

    def __init__(self, num_groups_limit: int = DEFAULT_NUM_GROUPS_LIMIT, device_trim: bool = True,
                 cpu_plan_maker=None, default_use_gpu: bool = True,
                 min_segment_group_trim_size: int = DEFAULT_MIN_SEGMENT_GROUP_TRIM_SIZE,
                 min_server_group_trim_size: int = DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE,
                 group_trim_threshold: int = DEFAULT_GROUPBY_TRIM_THRESHOLD):
        """device_trim=False: return every group (a rank of a multi-GPU server, whose partial groups must
        meet in ``distributed.allreduce_block`` BEFORE the server-level trim, ``reduce.trim_groups``).
        The remaining arguments are the server's instance config (InstancePlanMakerImplV2.init,
        InstancePlanMakerImplV2.java:108-140): query options override them per query (applyQueryOptions)."""
        if group_trim_threshold <= 0:  # (InstancePlanMakerImplV2.java:133-134)
            raise ValueError(f"Invalid configurable: groupByTrimThreshold: {group_trim_threshold} must be positive")
        self.num_groups_limit = num_groups_limit
        self.device_trim = device_trim
        self.cpu_plan_maker = cpu_plan_maker
        self.default_use_gpu = default_use_gpu
        self.min_segment_group_trim_size = min_segment_group_trim_size
        self.min_server_group_trim_size = min_server_group_trim_size
        self.group_trim_threshold = group_trim_threshold

    def apply_query_options(self, query: QueryContext) -> QueryContext:
        """InstancePlanMakerImplV2.applyQueryOptions (pinot-core/.../plan/maker/InstancePlanMakerImplV2.java:
        230-300): for a group-by query, numGroupsLimit (a positive int), minSegmentGroupTrimSize,
        minServerGroupTrimSize and groupTrimThreshold from the query options, else the server's values, written into
        a copy of the query's options (the reference's QueryContext setters). A malformed option raises
        QueryOptionError (the reference's BadQueryRequest). Options whose semantics the GPU operators do not have
        raise UnsupportedOnGpu: the server-returns-final-result modes (their blocks carry final, not intermediate,
        results). enableNullHandling is _make_operator's (GpuNullHandlingAggregationOperator)."""
        o = query.options
        _bool_option(o, "enableNullHandling")  # (validated: the operators read it, null_handling_enabled)
        _long_option_positive(o, "timeoutMs")  # (validated: make_instance_plan applies it, _DeadlineOperator)
        for k in ("serverReturnFinalResult", "serverReturnFinalResultKeyUnpartitioned"):
            if _bool_option(o, k):
                raise UnsupportedOnGpu(f"{k}: the GPU operators return intermediate results")
        if not (query.aggregations and query.group_by):
            return query
        opts = dict(o)
        v = _int_option(o, "numGroupsLimit", 1)
        opts["numGroupsLimit"] = str(v if v is not None else self.num_groups_limit)
        v = _int_option(o, "minSegmentGroupTrimSize")
        opts["minSegmentGroupTrimSize"] = str(v if v is not None else self.min_segment_group_trim_size)
        v = _int_option(o, "minServerGroupTrimSize")
        opts["minServerGroupTrimSize"] = str(v if v is not None else self.min_server_group_trim_size)
        v = _int_option(o, "groupTrimThreshold")
        opts["groupTrimThreshold"] = str(v if v is not None else self.group_trim_threshold)
        return dataclasses.replace(query, options=opts)

    def make_instance_plan(self, query: Union[str, QueryContext], segments: Sequence[GpuSegment]):
        if isinstance(query, str):
            query = parse(query)
        timeout = _long_option_positive(query.options, "timeoutMs")
        op = self._make_instance_plan(query, segments)
        return _DeadlineOperator(op, timeout) if timeout is not None else op

    def _make_instance_plan(self, query: QueryContext, segments: Sequence[GpuSegment]):
        if not use_gpu_option(query, self.default_use_gpu):
            if self.cpu_plan_maker is None:
                raise UnsupportedOnGpu("useGpu=false: the query belongs to the CPU plan maker")
            return self.cpu_plan_maker.make_instance_plan(query, segments)
        if self.cpu_plan_maker is None:
            return self._make_gpu_plan(query, segments)
        try:
            op = self._make_gpu_plan(query, segments)
        except UnsupportedOnGpu:
            return self.cpu_plan_maker.make_instance_plan(query, segments)
        # (an execution may still refuse: the combine's trim threshold, several infos at the limit, or a shape the
        # library only rejects when it prepares the plan on first execution)
        return GpuPlanWithCpuFallback(op, self.cpu_plan_maker, query, segments)

    def _make_gpu_plan(self, query: QueryContext, segments: Sequence[GpuSegment]):
        query = self.apply_query_options(query)
        op = self._make_operator(query, segments)
        if self.device_trim and GpuGroupByCombineOperator.needed(query):
            op = GpuGroupByCombineOperator(query, op, lambda segs: self._make_operator(query, segs))
        return op

    def _make_operator(self, query: QueryContext, segments: Sequence[GpuSegment]):
        from .startree import GpuStarTreeOperator
        limit = int(query.options["numGroupsLimit"]) if "numGroupsLimit" in query.options and query.group_by \
            else self.num_groups_limit
        if null_handling_enabled(query):
            op = _null_handling_operator(query, segments, limit)
            if op is not None:
                return op
        st = GpuStarTreeOperator.plan(query, segments, limit) if not _has_nulls(query, segments) else None
        if st is not None:
            st.inner.device_trim = self.device_trim
            return st
        if query.is_selection:
            return GpuSelectionOperator(query, segments, limit)
        if any(ag.argument is not None and _is_case(ag.argument) for ag in query.aggregations):
            return GpuCaseAggregationOperator(query, segments, limit)
        if any(ag.filter is not None for ag in query.aggregations):
            if query.group_by:
                return GpuFilteredGroupByOperator(query, segments, limit, self.device_trim)
            return GpuFilteredAggregationOperator(query, segments, limit)
        op = GpuCombineOperator(query, segments, limit)
        op.device_trim = self.device_trim
        return op
