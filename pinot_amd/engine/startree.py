"""Star-tree query path: fit check, tree traversal, and the GPU operator.

  StarTreeUtils.extractPredicateEvaluatorsMap  pinot-core/.../startree/StarTreeUtils.java:90-170
  StarTreeUtils.isFitForStarTree               :178-210
  StarTreeFilterOperator.traverseStarTree      pinot-core/.../startree/operator/StarTreeFilterOperator.java:212-364
  StarTreeFilterOperator.getFilterOperator     :154-196 (matched docs AND the remaining predicates)
  StarTreeAggregationExecutor / StarTreeGroupByExecutor  (aggregate the pre-aggregated ``function__column``)

The traversal runs on the host (the tree is small: one node per distinct dimension prefix above
maxLeafRecords); it yields the matched star-tree documents as doc ranges and the predicate columns the tree did
not resolve. The GPU then runs the ordinary filter + aggregation kernels over the star-tree documents (resident
beside their segment): a DOC_RANGES leaf AND the remaining predicates, aggregating SUM(sum__c) for SUM(c),
SUM(count__*) for COUNT(*), MIN(min__c) / MAX(max__c) -- one launch over all segments' star-trees.
"""
from collections import deque
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..query import predicate as predeval
from ..query.context import AggregationInfo, FilterContext, Function, Identifier, OrderByExpression, QueryContext
from ..segment.startree import ALL, STAR_HLL_LOG2M, avg_count_column, pair_column
from .results import AggregationResultsBlock, GroupByResultsBlock

USE_SCAN_TO_TRAVERSE_NODES_THRESHOLD = 10  # StarTreeFilterOperator.java:108


def _negated_predicate(fc):
    """NOT chains over one predicate -> (predicate, negated); None for anything else."""
    neg = False
    while fc.type == "NOT":
        neg = not neg
        fc = fc.children[0]
    if fc.type != "PREDICATE":
        return None
    return fc.predicate, neg


def _or_members(fc, out):
    """extractOrClausePredicates: OR of (NOT chains of) predicates, nested ORs flattened."""
    for c in fc.children:
        if c.type == "OR":
            if not _or_members(c, out):
                return False
            continue
        p = _negated_predicate(c)
        if p is None:
            return False
        out.append(p)
    return True


def _matching(seg, pred, negated):
    """Boolean mask over the column's dictionary ids (PredicateEvaluator on a dictionary-based column)."""
    d = seg.dictionary(pred.column)
    ev = predeval.evaluate(pred, d)
    mask = np.zeros(len(d), dtype=bool)
    ids = ev.matching_dict_ids(len(d))
    if len(ids):
        mask[np.asarray(ids, dtype=np.int64)] = True
    return ~mask if negated else mask


def predicate_map(seg, fc) -> Optional[Dict[str, List[tuple]]]:
    """extractPredicateEvaluatorsMap for one segment: column -> list of composite predicates (each a list of
    (predicate, negated) OR-ed together; the list is AND-ed), or None when the filter cannot use the star-tree
    (a predicate on a non-dictionary column, AND/OR nested under NOT, an OR spanning columns, an always-false
    leaf). Always-true leaves are dropped, as the reference does."""
    out: Dict[str, List[tuple]] = {}
    if fc is None:
        return out
    queue = deque([fc])
    while queue:
        n = queue.popleft()
        if n.type == "AND":
            queue.extend(n.children)
            continue
        if n.type == "CONSTANT":
            if not n.constant:
                return None
            continue
        if n.type == "OR":
            members = []
            if not _or_members(n, members):
                return None
            col, kept = None, []
            always_true = False
            for pred, neg in members:
                try:
                    m = seg.column_metadata(pred.column)
                except (KeyError, NotImplementedError):
                    return None
                if not m.has_dictionary:
                    return None
                mask = _matching(seg, pred, neg)
                if mask.all():
                    always_true = True
                    break
                if not mask.any():
                    continue
                if col is None:
                    col = pred.column
                elif col != pred.column:
                    return None
                kept.append((pred, neg))
            if always_true:
                continue
            if col is None:  # every member always false
                return None
            out.setdefault(col, []).append(kept)
            continue
        p = _negated_predicate(n)
        if p is None:
            return None
        pred, neg = p
        try:
            m = seg.column_metadata(pred.column)
        except (KeyError, NotImplementedError):
            return None
        if not m.has_dictionary:
            return None
        mask = _matching(seg, pred, neg)
        if not mask.any():
            return None
        if mask.all():
            continue
        out.setdefault(pred.column, []).append([(pred, neg)])
    return out


def _matching_dict_ids(seg, composites):
    """getMatchingDictIds: AND over the composite evaluators, each an OR of (negated) predicates."""
    acc = None
    for comp in composites:
        m = None
        for pred, neg in comp:
            x = _matching(seg, pred, neg)
            m = x if m is None else (m | x)
        acc = m if acc is None else (acc & m)
    return set(np.flatnonzero(acc).tolist())


class _Bulk:
    """All non-star children of one node, when each is a one-record leaf (see traverse)."""

    def __init__(self, parent):
        self.dimension_id = parent.child_dimension_id
        self.start, self.end = parent.start_doc, parent.end_doc  # the non-star children tile the node's range


def _bulk_leaves(node):
    """Cached per node: every non-star child is a leaf holding exactly one record (then the children's
    records are the contiguous range of the node's original records)."""
    flag = getattr(node, "_bulk", None)
    if flag is None:
        kids = [c for v, c in node.children.items() if v != ALL]
        flag = len(kids) > 64 and all(c.is_leaf and c.end_doc - c.start_doc == 1 for c in kids)
        if flag:
            lo = min(c.start_doc for c in kids)
            hi = max(c.end_doc for c in kids)
            flag = hi - lo == len(kids)
        node._bulk = flag
    return flag


def traverse(tree, seg, pmap, group_by_columns):
    """StarTreeFilterOperator.traverseStarTree (BFS). Returns (inclusive doc ranges as a flat int32 array,
    remaining predicate columns) or None when a predicate column has no matching dictionary id."""
    dims = tree.dimensions
    root = tree.root
    starts, ends = [], []
    found_leaf = root.is_leaf
    remaining_pred = set(pmap)
    remaining_gb = set(group_by_columns)
    global_remaining = set(remaining_pred) if found_leaf else None
    queue = deque([root])
    current_dim = -1
    matching = None
    while queue:
        node = queue.popleft()
        dim_id = node.dimension_id
        if dim_id > current_dim:
            name = dims[dim_id]
            remaining_pred.discard(name)
            remaining_gb.discard(name)
            if found_leaf and global_remaining is None:
                global_remaining = set(remaining_pred)
            matching = None
            current_dim = dim_id
        if isinstance(node, _Bulk):
            starts.append(node.start)
            ends.append(node.end)
            continue
        if not remaining_pred and not remaining_gb:
            starts.append(node.aggregated_doc)
            ends.append(node.aggregated_doc + 1)
            continue
        if node.is_leaf:
            starts.append(node.start_doc)
            ends.append(node.end_doc)
            continue
        child_dim = dims[dim_id + 1]
        star = None
        if (global_remaining is None or child_dim not in global_remaining) and child_dim not in remaining_gb:
            star = node.children.get(ALL)
        if child_dim in remaining_pred:
            if matching is None:
                matching = _matching_dict_ids(seg, pmap[child_dim])
                if not matching:
                    return None
            nchildren = len(node.children)
            if len(matching) * USE_SCAN_TO_TRAVERSE_NODES_THRESHOLD > nchildren:
                children = sorted(node.children.items())  # serialized order: by dimension value, ALL (-1) first
                if star is not None and len(matching) >= nchildren - 1:
                    hits = [c for v, c in children if v in matching]
                    if len(hits) == nchildren - 1:
                        queue.append(star)
                        found_leaf |= star.is_leaf
                    else:
                        queue.extend(hits)
                        found_leaf |= any(c.is_leaf for c in hits)
                else:
                    for v, c in children:
                        if v in matching:
                            queue.append(c)
                            found_leaf |= c.is_leaf
            else:
                for v in sorted(matching):
                    c = node.children.get(v)
                    if c is not None:
                        queue.append(c)
                        found_leaf |= c.is_leaf
        else:
            if star is not None:
                queue.append(star)
                found_leaf |= star.is_leaf
            elif _bulk_leaves(node):
                # every non-star child is a one-record leaf: they tile the node's record range, and each would
                # add its own record (as its range or as its aggregated doc) -- one range, not one node per value
                queue.append(_Bulk(node))
                found_leaf = True
            else:
                for v, c in sorted(node.children.items()):
                    if v != ALL:
                        queue.append(c)
                        found_leaf |= c.is_leaf
    # matched documents as merged inclusive ranges (the bitmap of the reference)
    if not starts:
        return np.zeros(0, dtype=np.int32), global_remaining or set()
    s = np.asarray(starts, dtype=np.int64)
    e = np.asarray(ends, dtype=np.int64)
    o = np.argsort(s, kind="stable")
    s, e = s[o], e[o]
    out = []
    cs, ce = int(s[0]), int(e[0])
    for a, b in zip(s[1:].tolist(), e[1:].tolist()):
        if a <= ce:
            ce = max(ce, b)
        else:
            out.extend((cs, ce - 1))
            cs, ce = a, b
    out.extend((cs, ce - 1))
    return np.asarray(out, dtype=np.int32), global_remaining or set()


def _remaining_filter(pmap, columns):
    """The remaining predicate columns' composites as one FilterContext (AND of per-column ORs)."""
    kids = []
    for col in sorted(columns):
        for comp in pmap[col]:
            ors = []
            for pred, neg in comp:
                f = FilterContext.PRED(pred)
                ors.append(FilterContext.NOT(f) if neg else f)
            kids.append(ors[0] if len(ors) == 1 else FilterContext.OR(*ors))
    if not kids:
        return None
    return kids[0] if len(kids) == 1 else FilterContext.AND(*kids)


_STAR_FUNCS = ("sum", "count", "min", "max", "avg", "distinctcounthll")


def _pair_of(ag):
    """AggregationFunctionUtils.getStoredFunctionColumnPair for the functions with a stored pair."""
    if ag.filter is not None or ag.function not in _STAR_FUNCS:
        return None
    if ag.function == "count":
        return ("count", "*")
    if not isinstance(ag.argument, Identifier):
        return None
    if ag.function == "distinctcounthll" and ag.log2m != STAR_HLL_LOG2M:  # the pair's HyperLogLog is log2m 8
        return None
    return (ag.function, ag.argument.name)


class GpuStarTreeOperator:
    """AggregationOperator / GroupByOperator over star-tree documents (AggregationPlanNode / GroupByPlanNode pick
    the star-tree when ``useStarTree`` is on and StarTreeUtils says it fits), for every segment at once. Use
    ``GpuStarTreeOperator.plan(...)``: it returns None when some segment has no fitting star-tree, and the caller
    builds the scan operators instead."""

    @classmethod
    def plan(cls, query: QueryContext, segments, num_groups_limit):
        if str(query.options.get("useStarTree", "true")).lower() == "false" or not segments:
            return None
        pairs = [_pair_of(a) for a in query.aggregations]
        if not pairs or any(p is None for p in pairs):
            return None
        if any(not isinstance(e, Identifier) for e in query.group_by):
            return None
        gb_cols = [e.name for e in query.group_by]
        chosen = []
        for seg in segments:
            pick = None
            pmap = predicate_map(seg, query.filter) if getattr(seg, "star_trees", None) else None
            if pmap is None:
                return None
            for tree, tseg in zip(seg.star_trees, seg.star_segments):
                have = set(tree.pairs)
                dims = set(tree.dimensions)
                if all(p in have for p in pairs) and set(gb_cols) <= dims and set(pmap) <= dims:
                    pick = (tree, tseg)
                    break
            if pick is None:
                return None
            chosen.append((seg, pick[0], pick[1], pmap))
        return cls(query, chosen, pairs, num_groups_limit)

    def __init__(self, query, chosen, pairs, num_groups_limit):
        from .plan import GpuCombineOperator
        self.query = query
        self.num_total_docs = sum(seg.num_docs for seg, _, _, _ in chosen)
        # per query function, the star-tree metric(s) it reads: SUM / MIN / MAX of their pair column, COUNT = SUM of
        # count__*, AVG = SUM of its (sum, count) columns (AvgPair merge)
        inner_aggs, self.slots = [], []
        for (f, c) in pairs:
            if f == "avg":
                self.slots.append((len(inner_aggs), len(inner_aggs) + 1))
                inner_aggs += [AggregationInfo("sum", Identifier(pair_column(f, c))),
                               AggregationInfo("sum", Identifier(avg_count_column(c)))]
                continue
            self.slots.append((len(inner_aggs),))
            if f == "distinctcounthll":  # max-merge of the documents' register rows
                inner_aggs.append(AggregationInfo(f, Identifier(pair_column(f, c)), STAR_HLL_LOG2M))
                continue
            inner_aggs.append(AggregationInfo("sum" if f == "count" else f, Identifier(pair_column(f, c))))
        mapping = {}
        for ag, sl in zip(query.aggregations, self.slots):
            if len(sl) == 1:
                a = inner_aggs[sl[0]]
                key = Function(ag.function, (ag.argument,) if ag.argument is not None else ())
                mapping[str(key)] = Function(a.function, (a.argument,))
        # ORDER BY an AVG has no single inner metric: the device trim is skipped and the operator trims its outer
        # groups on the host (reduce.trim_groups), exactly as the combine's IndexedTable would
        self.host_trim = any(f == "avg" for f, _ in pairs) and bool(query.order_by)
        order = []
        for ob in query.order_by:
            e = ob.expression
            if self.host_trim:
                break
            if str(e) in mapping:
                order.append(OrderByExpression(mapping[str(e)], ob.ascending))
            elif isinstance(e, Function) and e.name == "count":
                order.append(OrderByExpression(mapping.get("count()", e), ob.ascending))
            else:
                order.append(ob)
        self.inner_query = QueryContext(query.table, [], inner_aggs, None, list(query.group_by), order,
                                        limit=query.limit, options=dict(query.options))
        segs, per_seg = [], []
        self.docs_matched_ranges = []
        empty = False
        for seg, tree, tseg, pmap in chosen:
            res = traverse(tree, seg, pmap, [e.name for e in query.group_by])
            if res is None:
                ranges, rem = np.zeros(0, dtype=np.int32), set()
            else:
                ranges, rem = res
            segs.append(tseg)
            per_seg.append((_remaining_filter(pmap, rem), ranges))
            self.docs_matched_ranges.append(ranges)
        self.inner = GpuCombineOperator(self.inner_query, segs, num_groups_limit, segment_filters=per_seg)
        self.inner.device_trim = True
        self.functions = [f for f, _ in pairs]

    def _outer(self, vals):
        out = []
        for f, sl in zip(self.functions, self.slots):
            if f == "avg":
                out.append((float(vals[sl[0]]), int(vals[sl[1]])))
            elif f == "distinctcounthll":
                out.append(vals[sl[0]])
            else:
                v = vals[sl[0]]
                out.append(int(v) if f == "count" else float(v))
        return out

    def next_block(self):
        blk = self.inner.next_block()
        stats = blk.stats
        stats.num_total_docs = self.num_total_docs
        if not self.query.group_by:
            out = AggregationResultsBlock(self.query.aggregations, self._outer(blk.results), stats)
        else:
            groups = {k: self._outer(v) for k, v in blk.groups.items()}
            out = GroupByResultsBlock(self.query.aggregations, list(self.query.group_by), groups, stats,
                                      blk.num_groups_limit_reached)
            out.num_groups_trimmed = getattr(blk, "num_groups_trimmed", False)
            out.key_types = getattr(blk, "key_types", None)
            if self.host_trim and self.inner.device_trim:
                from .reduce import trim_groups
                out = trim_groups(self.query, out, getattr(self, "segment_trim", None))
        for a in ("device_ms", "scan_kernel_ms", "filter_kernel_ms", "agg_kernel_ms", "filter_bytes", "agg_bytes",
                  "segment_docs_matched"):
            setattr(out, a, getattr(blk, a, 0))
        out.star_tree = True
        return out

    def close(self):
        self.inner.close()


class HostSegmentView:
    """The host-side readers the traversal needs (dictionaries, column metadata) over an ImmutableSegment,
    without loading it on a device -- what the Java plan maker reads from the mapped segment."""

    def __init__(self, segment):
        from ..segment.dictionary import Dictionary
        self.segment = segment
        self.num_docs = segment.num_docs
        self.star_trees = list(segment.star_trees)
        self._dicts = {}
        self._Dictionary = Dictionary

    def column_metadata(self, column):
        return self.segment.columns[column].metadata

    def dictionary(self, column):
        d = self._dicts.get(column)
        if d is None:
            ci = self.segment.columns[column]
            m = ci.metadata
            d = self._Dictionary(ci.dictionary, m.data_type, m.cardinality, m.string_width)
            self._dicts[column] = d
        return d
