"""Cross-GPU merge of partial results blocks: the exchange step that replaces the CombineOperator merge.

In the reference, one server merges its per-segment blocks on the main thread
(AggregationResultsBlockMerger.mergeResultsBlocks, pinot-core/.../operator/combine/merger/
AggregationResultsBlockMerger.java:34-49; GroupByCombineOperator upserts value-keyed records,
…/operator/combine/GroupByCombineOperator.java:138-147). Here each GPU (one process per GPU) answers
the query over the segments it owns, and the partial blocks meet in collectives over
``torch.distributed`` ("nccl" = RCCL over xGMI on the GPU box, "gloo" in the CPU tests):

  aggregation  one all-reduce per merge operator over a packed vector: SUM for COUNT / exact int64
               sums (int64) and DOUBLE sums (float64), MIN / MAX (float64), MAX for HLL registers.
  group-by     keys are VALUES (dictionaries are per segment): the distinct key
               values of every group-by column are all-gathered into a node-global sorted dictionary,
               every rank scatters its groups into the dense mixed-radix table over those global ids
               (column 0 least significant, as DictionaryBasedGroupKeyGenerator), and the dense partials
               are all-reduced like the aggregation case. Above ``max_dense_groups`` the sparse records
               are all-gathered and merged instead.

Every rank returns the merged block (all-reduce semantics), so rank 0 can build the response.
"""
from typing import List, Optional

import numpy as np

from .results import AggregationResultsBlock, ExecutionStatistics, GroupByResultsBlock, merge_intermediate

_HLL_FUNCS = ("distinctcounthll", "distinctcountrawhll")


def _device(dist, group):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _reduce(dist, group, arr: np.ndarray, op):
    """All-reduce a numpy array in place through torch (int64 / float64 / int32)."""
    import torch
    if arr.size == 0:
        return arr
    t = torch.from_numpy(np.ascontiguousarray(arr)).to(_device(dist, group))
    dist.all_reduce(t, op=op, group=group)
    return t.cpu().numpy()


def _stats_vector(s: ExecutionStatistics) -> np.ndarray:
    return np.array([s.num_docs_scanned, s.num_entries_scanned_in_filter, s.num_entries_scanned_post_filter,
                     s.num_total_docs, s.num_segments_processed, s.num_segments_matched], dtype=np.int64)


def _stats_from(v) -> ExecutionStatistics:
    return ExecutionStatistics(*[int(x) for x in v])


class _Slots:
    """Layout of one row of intermediates across the four reduce operators."""

    def __init__(self, aggregations, sample_row, integral_sums):
        self.plan = []  # per function: list of (kind, index) where kind in int/fsum/min/max/hll
        self.n = {"int": 0, "fsum": 0, "min": 0, "max": 0}
        self.hll_m = 0
        self.nhll = 0
        for i, a in enumerate(aggregations):
            f = a.function
            if f == "count":
                self.plan.append([("int", self._take("int"))])
            elif f == "sum":
                self.plan.append([("int", self._take("int"))] if integral_sums[i] else [("fsum", self._take("fsum"))])
            elif f == "min":
                self.plan.append([("min", self._take("min"))])
            elif f == "max":
                self.plan.append([("max", self._take("max"))])
            elif f == "avg":
                s = ("int", self._take("int")) if integral_sums[i] else ("fsum", self._take("fsum"))
                self.plan.append([s, ("int", self._take("int"))])
            elif f == "minmaxrange":
                self.plan.append([("min", self._take("min")), ("max", self._take("max"))])
            elif f in _HLL_FUNCS:
                m = len(sample_row[i]) if sample_row is not None else 1 << a.log2m
                self.hll_m = m
                self.plan.append([("hll", self.nhll)])
                self.nhll += 1
            else:
                raise NotImplementedError(f)

    def _take(self, kind):
        self.n[kind] += 1
        return self.n[kind] - 1

    def empty(self, rows):
        return {"int": np.zeros((rows, self.n["int"]), np.int64),
                "fsum": np.zeros((rows, self.n["fsum"]), np.float64),
                "min": np.full((rows, self.n["min"]), np.inf),
                "max": np.full((rows, self.n["max"]), -np.inf),
                "hll": np.zeros((rows, self.nhll, max(self.hll_m, 1)), np.int32)}

    def put(self, bufs, r, row):
        for parts, v in zip(self.plan, row):
            vals = v if len(parts) > 1 else (v,)
            for (kind, j), x in zip(parts, vals):
                if kind == "hll":
                    bufs["hll"][r, j, :] = np.asarray(x, dtype=np.int32)
                elif kind == "int":
                    bufs["int"][r, j] = int(x)
                else:
                    bufs[kind][r, j] = float(x)

    def get(self, bufs, r):
        out = []
        for parts in self.plan:
            vals = []
            for kind, j in parts:
                if kind == "hll":
                    vals.append(bufs["hll"][r, j, :].astype(np.uint8))
                elif kind == "int":
                    vals.append(int(bufs["int"][r, j]))
                else:
                    vals.append(float(bufs[kind][r, j]))
            out.append(tuple(vals) if len(parts) > 1 else vals[0])
        return out


def _integral_sums(aggregations, rows):
    """A SUM is exact-int64 when its intermediate is a Python int on every rank (see results.py)."""
    out = []
    for i, a in enumerate(aggregations):
        if a.function == "sum":
            out.append(all(isinstance(r[i], (int, np.integer)) for r in rows) if rows else False)
        elif a.function == "avg":
            out.append(all(isinstance(r[i][0], (int, np.integer)) for r in rows) if rows else False)
        else:
            out.append(False)
    return out


def _all_true(dist, group, flags: List[bool]) -> List[bool]:
    import torch
    v = _reduce(dist, group, np.array([0 if f else 1 for f in flags] or [0], dtype=np.int64), dist.ReduceOp.SUM)
    return [int(x) == 0 for x in v[:len(flags)]]


def _reduce_bufs(dist, group, bufs):
    S, MIN, MAX = dist.ReduceOp.SUM, dist.ReduceOp.MIN, dist.ReduceOp.MAX
    return {"int": _reduce(dist, group, bufs["int"], S), "fsum": _reduce(dist, group, bufs["fsum"], S),
            "min": _reduce(dist, group, bufs["min"], MIN), "max": _reduce(dist, group, bufs["max"], MAX),
            "hll": _reduce(dist, group, bufs["hll"], MAX)}


def allreduce_block(block, dist=None, group=None, max_dense_groups: int = 1 << 22):
    """Merge this rank's partial block with every other rank's; returns the merged block on every rank."""
    if dist is None:
        import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return block
    stats = _stats_from(_reduce(dist, group, _stats_vector(block.stats), dist.ReduceOp.SUM))
    aggs = block.aggregations
    if isinstance(block, AggregationResultsBlock):
        integral = _all_true(dist, group, _integral_sums(aggs, [block.results]))
        slots = _Slots(aggs, block.results, integral)
        bufs = slots.empty(1)
        slots.put(bufs, 0, block.results)
        bufs = _reduce_bufs(dist, group, bufs)
        return AggregationResultsBlock(aggs, slots.get(bufs, 0), stats)

    # ---- group-by: node-global dictionaries over the key values --------------------------------
    keys = list(block.groups.keys())
    nk = len(block.group_by)
    world = dist.get_world_size(group)
    local_vals = [sorted({k[c] for k in keys}) for c in range(nk)]
    gathered = [None] * world
    dist.all_gather_object(gathered, local_vals, group=group)
    gdict = [sorted(set().union(*[g[c] for g in gathered])) for c in range(nk)]
    cards = [max(len(d), 1) for d in gdict]
    ndense = int(np.prod(cards, dtype=np.int64)) if nk else 1
    limit = _reduce(dist, group, np.array([int(block.num_groups_limit_reached)], np.int64), dist.ReduceOp.MAX)
    limit_reached = bool(limit[0])
    rows = list(block.groups.values())
    integral = _all_true(dist, group, _integral_sums(aggs, rows))
    if ndense > max_dense_groups:
        parts = [None] * world
        dist.all_gather_object(parts, block.groups, group=group)
        merged = {}
        for p in parts:
            for k, v in p.items():
                merged[k] = v if k not in merged else [merge_intermediate(a.function, x, y)
                                                       for a, x, y in zip(aggs, merged[k], v)]
        return GroupByResultsBlock(aggs, block.group_by, merged, stats, limit_reached)
    index = [{v: i for i, v in enumerate(d)} for d in gdict]
    strides = np.cumprod([1] + cards[:-1]).astype(np.int64)
    sample = rows[0] if rows else None
    # HLL width must agree on every rank even where this rank has no group
    slots = _Slots(aggs, sample, integral)
    for i, a in enumerate(aggs):
        if a.function in _HLL_FUNCS:
            slots.hll_m = 1 << a.log2m
    bufs = slots.empty(ndense)
    present = np.zeros(ndense, np.int64)
    for k, v in block.groups.items():
        d = int(sum(index[c][k[c]] * strides[c] for c in range(nk)))
        present[d] = 1
        slots.put(bufs, d, v)
    present = _reduce(dist, group, present, dist.ReduceOp.SUM)
    bufs = _reduce_bufs(dist, group, bufs)
    groups = {}
    for d in np.nonzero(present)[0]:
        key, rem = [], int(d)
        for c in range(nk):
            key.append(gdict[c][rem % cards[c]])
            rem //= cards[c]
        groups[tuple(key)] = slots.get(bufs, int(d))
    return GroupByResultsBlock(aggs, block.group_by, groups, stats, limit_reached)
