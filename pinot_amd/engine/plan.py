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
import ctypes
import math
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Union

import numpy as np

from .. import _lib
from ..query import predicate as predeval
from ..query.context import (UNBOUNDED, AggregationInfo, FilterContext, Function, Identifier, Literal,
                             QueryContext, columns_of)
from ..query.sql import parse
from ..spi import DEFAULT_NUM_GROUPS_LIMIT, DataType
from .results import AggregationResultsBlock, ExecutionStatistics, GroupByResultsBlock
from .segment import GpuSegment


class UnsupportedOnGpu(Exception):
    """Query shape outside the GPU subset (the Java side would call super.makeInstancePlan)."""


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


def _raw_predicate(column, dt: DataType, pred):
    """Value-based leaf on a raw column (RawValueBasedPredicateEvaluatorFactory + ScanBasedFilterOperator):
    literals converted to the column type first (FLOAT literals rounded to float32, as Float.parseFloat);
    integral ranges folded to closed integer intervals."""
    if dt == DataType.STRING:
        raise UnsupportedOnGpu(f"predicate on raw STRING column {column}")
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
    if len(vals) > 1024:
        raise UnsupportedOnGpu("raw IN list longer than 1024 values")
    if not vals:
        return _TRUE if exclusive else _FALSE
    arr = np.asarray(vals, dtype=np.float64 if real else np.int64)
    return _Leaf(_lib.LEAF_RAW_SET, column, exclusive=exclusive, ids=arr.view(np.int32).copy())


INVERTED_COST_RATIO = 0.5  # decode bytes allowed per forward-index byte (measured: tools/configs_bench.py C4)


def compile_predicate(seg: GpuSegment, pred) -> object:
    column = pred.column
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
            inv_ok = seg.inverted_bytes(column, ids) <= INVERTED_COST_RATIO * fwd
        if inv_ok:
            if ev.kind == "range":
                return _Leaf(_lib.LEAF_INVERTED, column, ids=ids)
            return _Leaf(_lib.LEAF_INVERTED, column, exclusive=ev.exclusive, ids=ids)
    if ev.kind == "range":
        return _Leaf(_lib.LEAF_DICT_RANGE, column, lo=ev.start, hi=ev.end)
    return _Leaf(_lib.LEAF_DICT_SET, column, exclusive=ev.exclusive, ids=np.asarray(ev.ids, dtype=np.int32))


def compile_filter(seg: GpuSegment, fc: Optional[FilterContext]):
    """FilterContext -> leaf/node tree for one segment, constants folded (FilterPlanNode.java:197-229)."""
    if fc is None:
        return _TRUE
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
        if isinstance(c, _Leaf) and c.kind in (_lib.LEAF_DICT_SET, _lib.LEAF_INVERTED, _lib.LEAF_RAW_SET):
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
        kids = [k for k in kids if not _is_const(k, _FALSE)]
        if not kids:
            return _FALSE
        if len(kids) == 1:
            return kids[0]
        return _Node(_lib.NODE_OR, kids)
    raise ValueError(fc.type)


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


def plan_aggregations(aggs: Sequence[AggregationInfo]):
    """Query aggregations -> GPU primitives (deduplicated) + per-function slot mapping."""
    prims = []  # (function, expr, col_a, col_b, log2m)
    mapping = []

    def slot(p):
        if p not in prims:
            prims.append(p)
        return prims.index(p)

    for ag in aggs:
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
            if expr[0] != _lib.EXPR_COLUMN:
                raise UnsupportedOnGpu("DISTINCTCOUNTHLL over an expression")
            mapping.append((f, slot((_lib.AGG_HLL,) + expr + (ag.log2m,))))
        else:
            raise UnsupportedOnGpu(f"aggregation {f} is not on the GPU path")
    return prims, mapping


# ------------------------------------------------------------------------------ operators
class GpuCombineOperator:
    """One operator over all segments of the query (the all-segment GPU variant of SURVEY.md §8b)."""

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int):
        self.query = query
        self.segments = list(segments)
        self.num_groups_limit = num_groups_limit
        for e in query.group_by:
            if not isinstance(e, Identifier):
                raise UnsupportedOnGpu(f"group-by expression {e}")
        self.prims, self.mapping = plan_aggregations(query.aggregations)
        self.trees = [compile_filter(s, query.filter) for s in self.segments]
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
        aggs = (_lib.Aggregation * max(len(self.prims), 1))()
        for i, (f, expr, ca, cb, log2m) in enumerate(self.prims):
            aggs[i].function = f
            aggs[i].expr = expr
            aggs[i].column_a = col_index[ca] if ca is not None else -1
            aggs[i].column_b = col_index[cb] if cb is not None else -1
            aggs[i].log2m = log2m
        keep.append(aggs)
        q.num_aggregations = len(self.prims)
        q.aggregations = aggs
        gb = (ctypes.c_int32 * max(len(self.query.group_by), 1))(*[col_index[e.name] for e in self.query.group_by])
        keep.append(gb)
        q.num_group_by = len(self.query.group_by)
        q.group_by_columns = gb
        q.num_groups_limit = self.num_groups_limit
        q.order_by_aggregation, q.order_by_desc, q.trim_size, okeys = self._trim_spec()
        if okeys:
            arr = (ctypes.c_int32 * len(okeys))(*okeys)
            keep.append(arr)
            q.num_order_by_keys = len(okeys)
            q.order_by_keys = arr
        return q

    def _trim_spec(self):
        """Server-level trim of GroupByUtils.createIndexedTableForCombineOperator (GroupByUtils.java:96-140):
        with ORDER BY the combine keeps trimSize = getTableCapacity(limit, minServerGroupTrimSize)
        = max(5 * limit, 5000) records (:55-58; default minServerGroupTrimSize 5000,
        InstancePlanMakerImplV2.java:92), ordered by the ORDER BY. The device trims when the ORDER BY is a
        single SUM/MIN/MAX/COUNT aggregation or only group-by columns; otherwise every group is returned (the broker's ORDER BY +
        LIMIT gives the same final rows)."""
        from .reduce import _agg_index
        q = self.query
        none = (-1, 0, 0, [])
        if not q.group_by or not q.order_by or not getattr(self, "device_trim", True):
            return none
        min_trim = int(q.options.get("minServerGroupTrimSize", 5000))
        if min_trim <= 0:  # trim disabled (GroupByUtils.java:108)
            return none
        trim = min(max(5 * int(q.limit), min_trim), 2 ** 31 - 1)
        gb = [str(e) for e in q.group_by]
        if all(str(ob.expression) in gb for ob in q.order_by) and len(q.order_by) <= 8 and len(gb) <= 8:
            keys = [(gb.index(str(ob.expression)) + 1) * (1 if ob.ascending else -1) for ob in q.order_by]
            return -1, 0, trim, keys
        if len(q.order_by) != 1:
            return none
        i = _agg_index(q, q.order_by[0].expression)
        if i is None:
            return none
        f, s = self.mapping[i]
        if f not in ("sum", "min", "max", "count") or q.aggregations[i].filter is not None:
            return none
        return int(s), int(not q.order_by[0].ascending), trim, []

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
        lib = _lib.load()
        if getattr(self, "_plan", None) is None:
            keep = []
            q = self._desc(keep)
            h = ctypes.c_uint64(0)
            _lib.check(lib.phip_plan_create(ctypes.byref(q), ctypes.byref(h)))
            self._plan = h.value
            self._lib = lib
        if prepare_only:
            return None
        res = ctypes.POINTER(_lib.Result)()
        _lib.check(lib.phip_plan_execute(self._plan, ctypes.byref(res)))
        return res

    def close(self):
        """Release the prepared plan (and with it the last references to unloaded segments)."""
        if getattr(self, "_plan", None):
            self._lib.phip_plan_destroy(self._plan)
            self._plan = None

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
        for ag in self.query.aggregations:
            if ag.function not in self._NON_SCAN:
                return False
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
        if self._non_scan_fit():
            return self._non_scan_block()
        return self._block_from_result(self.run_raw())

    # -- multi-GPU servers (include/pinot_hip.h "multi-GPU servers"; engine/distributed.py) -------------
    def execute_partial(self):
        """Runs the plan up to this GPU's dense partial group table (phip_plan_execute_partial). Returns the
        _lib.Partial (device pointers), or None when the plan cannot hand one out (hash-table key space,
        numGroupsLimit reached on this GPU) -- the caller then merges records instead."""
        if not self.query.group_by:
            return None
        lib = _lib.load()
        self.run_raw(prepare_only=True)
        part = _lib.Partial()
        rc = lib.phip_plan_execute_partial(self._plan, ctypes.byref(part))
        if rc == _lib.PHIP_ERR_UNSUPPORTED:
            return None
        _lib.check(rc)
        return part

    def finish(self, merged):
        """Result block of the (merged) partial table: compaction, server-level trim, statistics of `merged`."""
        lib = _lib.load()
        res = ctypes.POINTER(_lib.Result)()
        _lib.check(lib.phip_plan_finish(self._plan, ctypes.byref(merged), ctypes.byref(res)))
        return self._block_from_result(res)

    def _block_from_result(self, res):
        lib = _lib.load()
        try:
            r = res.contents
            stats = ExecutionStatistics(r.num_docs_scanned, r.num_entries_scanned_in_filter,
                                        r.num_entries_scanned_post_filter, r.num_total_docs,
                                        r.num_segments_processed, r.num_segments_matched)
            na = r.num_aggregations
            ng = r.num_groups
            m = 1 << max([p[4] for p in self.prims if p[0] == _lib.AGG_HLL] + [0])
            # (no groups: the library's arrays may be null)
            vals = np.ctypeslib.as_array(r.values, shape=(ng * na,)).reshape(ng, na).copy() if ng * na else np.zeros((ng, na))
            longs = (np.ctypeslib.as_array(r.long_values, shape=(ng * na,)).reshape(ng, na).copy() if ng * na
                     else np.zeros((ng, na), np.int64))
            hll = None
            if r.num_hll and ng:
                hll = np.ctypeslib.as_array(r.hll_registers, shape=(ng * r.num_hll * m,)).reshape(ng, r.num_hll, m).copy()
            hll_slot = {}
            for i, p in enumerate(self.prims):
                if p[0] == _lib.AGG_HLL:
                    hll_slot[i] = len(hll_slot)
            # long_exact[a]: the library kept an exact int64 sum (else it summed in double: int64 overflow bound)
            exact = [bool(r.long_exact[i]) for i in range(na)] if na else []

            def prim_value(g, i):
                f = self.prims[i][0]
                if f == _lib.AGG_COUNT:
                    return int(longs[g, i])
                if f == _lib.AGG_SUM:
                    return int(longs[g, i]) if exact[i] else float(vals[g, i])
                if f in (_lib.AGG_MIN, _lib.AGG_MAX):
                    return float(vals[g, i])
                return hll[g, hll_slot[i]].copy()

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
                dicts = []
                for k in range(nk):
                    dv = _lib.DictionaryView()
                    _lib.check(lib.phip_result_dictionary(res, k, ctypes.byref(dv)))
                    dicts.append(_dictionary_values(dv))
                groups = {}
                for g in range(ng):
                    key = tuple(dicts[k][keys[g, k]] for k in range(nk))
                    groups[key] = intermediates(g)
                blk = GroupByResultsBlock(self.query.aggregations, list(self.query.group_by), groups, stats,
                                          bool(r.num_groups_limit_reached))
                blk.num_groups_trimmed = bool(r.num_groups_trimmed)
            blk.device_ms = r.device_ms
            blk.scan_kernel_ms = r.scan_kernel_ms
            blk.filter_kernel_ms, blk.agg_kernel_ms = r.filter_kernel_ms, r.agg_kernel_ms
            blk.filter_bytes, blk.agg_bytes = int(r.filter_bytes), int(r.agg_bytes)
            return blk
        finally:
            lib.phip_result_free(res)


def _dictionary_values(dv):
    card = dv.cardinality
    t = DataType(dv.data_type)
    if t == DataType.STRING:
        w = dv.string_width
        raw = ctypes.string_at(dv.values, card * w)
        return [raw[i * w:(i + 1) * w].rstrip(b"\0").decode("utf-8") for i in range(card)]
    dt = {DataType.INT: np.int32, DataType.LONG: np.int64, DataType.FLOAT: np.float32, DataType.DOUBLE: np.float64}[t]
    arr = np.ctypeslib.as_array(ctypes.cast(dv.values, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(card,))
    return [x.item() for x in arr]


class GpuFilteredAggregationOperator:
    """FilteredAggregationOperator (pinot-core/.../operator/query/FilteredAggregationOperator.java:67-113)
    over all segments: the aggregations are grouped by their FILTER clause (unfiltered ones under the
    main filter), as AggregationFunctionUtils.buildFilteredAggregationInfos does, and every group runs as
    one GPU combine operator over main AND its filter. Results return in query order; numDocsScanned
    and the entries scanned are summed over the groups, like the reference operator's statistics."""

    def __init__(self, query: QueryContext, segments: Sequence[GpuSegment], num_groups_limit: int):
        if query.group_by:
            raise UnsupportedOnGpu("FILTER clause with GROUP BY (FilteredGroupByOperator)")
        self.query = query
        self.segments = list(segments)
        groups = {}
        for i, ag in enumerate(query.aggregations):
            groups.setdefault(ag.filter, []).append(i)
        self.parts = []
        for flt, idxs in groups.items():
            if flt is None:
                f = query.filter
            elif query.filter is None:
                f = flt
            else:
                f = FilterContext.AND(query.filter, flt)
            sub = QueryContext(query.table, [], [query.aggregations[i].unfiltered() for i in idxs], f, [],
                               limit=query.limit, options=dict(query.options))
            self.parts.append((idxs, GpuCombineOperator(sub, self.segments, num_groups_limit)))

    def next_block(self):
        results = [None] * len(self.query.aggregations)
        stats = ExecutionStatistics()
        scan_ms = device_ms = 0.0
        for idxs, op in self.parts:
            blk = op.next_block()
            for j, i in enumerate(idxs):
                results[i] = blk.results[j]
            s = blk.stats
            stats.num_docs_scanned += s.num_docs_scanned
            stats.num_entries_scanned_in_filter += s.num_entries_scanned_in_filter
            stats.num_entries_scanned_post_filter += s.num_entries_scanned_post_filter
            stats.num_total_docs = s.num_total_docs
            stats.num_segments_processed = s.num_segments_processed
            stats.num_segments_matched = max(stats.num_segments_matched, s.num_segments_matched)
            scan_ms += getattr(blk, "scan_kernel_ms", 0.0) or 0.0
            device_ms += getattr(blk, "device_ms", 0.0) or 0.0
        blk = AggregationResultsBlock(self.query.aggregations, results, stats)
        blk.scan_kernel_ms = scan_ms
        blk.device_ms = device_ms
        return blk

    def close(self):
        for _, op in self.parts:
            op.close()


class GpuInstancePlanMaker:
    """``pinot.server.query.executor.plan.maker.class`` plug-in."""

    def __init__(self, num_groups_limit: int = DEFAULT_NUM_GROUPS_LIMIT, device_trim: bool = True):
        """device_trim=False: return every group (a rank of a multi-GPU server, whose partial groups must
        meet in ``distributed.allreduce_block`` BEFORE the server-level trim, ``reduce.trim_groups``)."""
        self.num_groups_limit = num_groups_limit
        self.device_trim = device_trim

    def make_instance_plan(self, query: Union[str, QueryContext], segments: Sequence[GpuSegment]):
        if isinstance(query, str):
            query = parse(query)
        if any(ag.filter is not None for ag in query.aggregations):
            return GpuFilteredAggregationOperator(query, segments, self.num_groups_limit)
        op = GpuCombineOperator(query, segments, self.num_groups_limit)
        op.device_trim = self.device_trim
        return op
