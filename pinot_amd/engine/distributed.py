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

from .results import (AggregationResultsBlock, ExecutionStatistics, GroupByResultsBlock, java_double_key,
                      merge_intermediate)

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


# ---- one SUM and one MAX per merge ----------------------------------------------------------------
# A row of intermediates is packed into a float64 SUM part and an int64 MAX part, so a merge is exactly two
# all-reduces whatever the functions (the reference merges per function: SumAggregationFunction.merge `+`,
# Min/Max `min`/`max`, HLL register max -- AggregationResultsBlockMerger.java:34-49):
#   SUM   int64 values (COUNT, exact integer SUMs) as two doubles (v >> 32, v & 0xffffffff): each half sums
#         exactly in a double over any realistic number of ranks (< 2^21), and the halves recombine to the exact
#         integer; double SUMs as themselves; execution statistics (< 2^53) as doubles.
#   MAX   MAX results as the order-preserving int64 image of the double (Double.compare order), MIN results as
#         its bitwise complement (the order reversed, so MAX of it is the MIN), HLL registers one per slot, and
#         per SUM slot a flag "this rank summed in double" (the int64 bound is per GPU): a SUM is exact only when
#         no rank overflowed to double.
def _f64_key(x: float) -> int:
    u = int(np.array([x], "<f8").view(np.uint64)[0])
    o = (~u & 0xFFFFFFFFFFFFFFFF) if u >> 63 else (u | (1 << 63))
    return o - (1 << 63)  # signed image, same order


def _f64_from_key(k: int) -> float:
    o = (int(k) + (1 << 63)) & 0xFFFFFFFFFFFFFFFF
    u = (o & ((1 << 63) - 1)) if o >> 63 else (~o & 0xFFFFFFFFFFFFFFFF)
    return float(np.array([u], np.uint64).view("<f8")[0])


class _Layout:
    """Where each function's intermediate lives in the SUM (float64) and MAX (int64) parts of a row."""

    def __init__(self, aggregations):
        self.plan = []
        self.nsum = 0
        self.nmax = 0
        for a in aggregations:
            f = a.function
            if f == "count":
                self.plan.append(("count", self._s(2)))
            elif f == "sum":
                self.plan.append(("sum", self._s(3), self._m(1)))
            elif f == "avg":
                self.plan.append(("avg", self._s(3), self._m(1), self._s(2)))
            elif f == "min":
                self.plan.append(("min", self._m(1)))
            elif f == "max":
                self.plan.append(("max", self._m(1)))
            elif f == "minmaxrange":
                self.plan.append(("range", self._m(1), self._m(1)))
            elif f in _HLL_FUNCS:
                m = 1 << a.log2m  # each function's own width (DISTINCTCOUNTHLL log2m may differ per function)
                self.plan.append(("hll", self._m(m), m))
            else:
                raise NotImplementedError(f)

    def _s(self, n):
        self.nsum += n
        return self.nsum - n

    def _m(self, n):
        self.nmax += n
        return self.nmax - n

    @staticmethod
    def _put_int(sv, i, v):
        v = int(v)
        sv[i] = float(v >> 32)
        sv[i + 1] = float(v & 0xFFFFFFFF)

    @staticmethod
    def _get_int(sv, i):
        return (int(sv[i]) << 32) + int(sv[i + 1])

    def _put_sum(self, sv, mv, i, j, v):
        if isinstance(v, (int, np.integer)) and -(1 << 63) <= int(v) < (1 << 63):
            self._put_int(sv, i, v)
        else:
            sv[i + 2] = float(v)
            mv[j] = 1

    def _get_sum(self, sv, mv, i, j):
        exact = self._get_int(sv, i)
        return float(exact) + float(sv[i + 2]) if mv[j] else exact

    def put(self, sv, mv, row):
        for p, v in zip(self.plan, row):
            k = p[0]
            if k == "count":
                self._put_int(sv, p[1], v)
            elif k == "sum":
                self._put_sum(sv, mv, p[1], p[2], v)
            elif k == "avg":
                self._put_sum(sv, mv, p[1], p[2], v[0])
                self._put_int(sv, p[3], v[1])
            elif k == "min":
                mv[p[1]] = ~_f64_key(float(v))
            elif k == "max":
                mv[p[1]] = _f64_key(float(v))
            elif k == "range":
                mv[p[1]] = ~_f64_key(float(v[0]))
                mv[p[2]] = _f64_key(float(v[1]))
            else:
                r = np.asarray(v, dtype=np.int64)
                if len(r) != p[2]:
                    raise ValueError(f"HLL intermediate of {len(r)} registers where log2m gives {p[2]}")
                mv[p[1]:p[1] + p[2]] = r

    def empty_max(self, rows):
        """MAX parts of rows no function touched: MIN = +inf, MAX = -inf (the functions' defaults)."""
        mv = np.zeros((rows, self.nmax), np.int64)
        for p in self.plan:
            if p[0] == "min":
                mv[:, p[1]] = ~_f64_key(float("inf"))
            elif p[0] == "max":
                mv[:, p[1]] = _f64_key(float("-inf"))
            elif p[0] == "range":
                mv[:, p[1]] = ~_f64_key(float("inf"))
                mv[:, p[2]] = _f64_key(float("-inf"))
        return mv

    def get(self, sv, mv):
        out = []
        for p in self.plan:
            k = p[0]
            if k == "count":
                out.append(self._get_int(sv, p[1]))
            elif k == "sum":
                out.append(self._get_sum(sv, mv, p[1], p[2]))
            elif k == "avg":
                out.append((self._get_sum(sv, mv, p[1], p[2]), self._get_int(sv, p[3])))
            elif k == "min":
                out.append(_f64_from_key(~int(mv[p[1]])))
            elif k == "max":
                out.append(_f64_from_key(int(mv[p[1]])))
            elif k == "range":
                out.append((_f64_from_key(~int(mv[p[1]])), _f64_from_key(int(mv[p[2]]))))
            else:
                out.append(np.asarray(mv[p[1]:p[1] + p[2]]).astype(np.uint8))
        return out


def _sum_max(dist, group, sv: np.ndarray, mv: np.ndarray):
    """The merge's two collectives: float64 SUM of `sv` and int64 MAX of `mv`, staged through one host buffer
    and one device buffer (a single copy each way)."""
    import torch
    dev = _device(dist, group)
    ns, nm = sv.size, mv.size
    host = torch.empty(ns + nm, dtype=torch.float64, pin_memory=dev.type == "cuda")
    hv = host.numpy()
    hv[:ns] = sv.ravel()
    hv[ns:].view(np.int64)[:] = mv.ravel()
    d = host.to(dev, non_blocking=True)
    if ns:
        dist.all_reduce(d[:ns], op=dist.ReduceOp.SUM, group=group)
    if nm:
        dist.all_reduce(d[ns:].view(torch.int64), op=dist.ReduceOp.MAX, group=group)
    out = d.cpu().numpy()
    return out[:ns].reshape(sv.shape), out[ns:].view(np.int64).reshape(mv.shape)


def _key_order(v):
    """A total order of one column's key values for the node-global dictionaries: None (null) last, NaN before it,
    -0.0 beside 0.0 (two keys: results.JavaDoubleKey)."""
    if not isinstance(v, float):
        return (v is None, False, 0 if v is None else v, False)
    x = float(v)  # (plain float comparisons, whatever the wrapper's equality)
    return (False, x != x, 0.0 if x != x else x, x == 0.0 and not np.signbit(x))


def allreduce_block(block, dist=None, group=None, max_dense_groups: int = 1 << 22):
    """Merge this rank's partial block with every other rank's; returns the merged block on every rank.

    Aggregation blocks: one float64 SUM + one int64 MAX all-reduce (_Layout). Group-by blocks: the key values
    are exchanged once (all_gather_object) into node-global dictionaries, every rank scatters its groups into
    the dense mixed-radix rows over those ids (column 0 least significant, as DictionaryBasedGroupKeyGenerator),
    and the rows merge with the same SUM + MAX pair; above `max_dense_groups` the records are all-gathered and
    merged by key instead."""
    if dist is None:
        import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return block
    aggs = block.aggregations
    if isinstance(block, AggregationResultsBlock):
        lay = _Layout(aggs)
        sv = np.zeros(6 + lay.nsum)
        mv = lay.empty_max(1)[0]
        sv[:6] = _stats_vector(block.stats)
        # a null intermediate (enableNullHandling: nothing non-null aggregated) contributes the function's identity,
        # and a presence flag per function (MAX over the ranks) says whether any rank had a value
        ident = lay.get(np.zeros(lay.nsum), lay.empty_max(1)[0])
        lay.put(sv[6:], mv, [ident[i] if v is None else v for i, v in enumerate(block.results)])
        present = np.array([v is not None for v in block.results], dtype=np.int64)
        sv, mv = _sum_max(dist, group, sv, np.concatenate([mv, present]))
        vals = lay.get(sv[6:], mv[:lay.nmax])
        vals = [v if mv[lay.nmax + i] else None for i, v in enumerate(vals)]
        return AggregationResultsBlock(aggs, vals, _stats_from(sv[:6]))

    # ---- group-by: node-global dictionaries over the key values --------------------------------
    keys = list(block.groups.keys())
    nk = len(block.group_by)
    world = dist.get_world_size(group)
    # An upper bound of the merged key space first (the sum over ranks of each column's distinct values): a large one
    # goes straight to the record merge, without all-gathering every distinct value as Python objects
    local_sets = [{k[c] for k in keys} for c in range(nk)]
    bound = _reduce(dist, group, np.array([len(x) for x in local_sets] + [0], dtype=np.int64), dist.ReduceOp.SUM)[:nk]
    if nk and float(np.prod(np.maximum(bound, 1).astype(np.float64))) > max_dense_groups:
        merged = _merge_records_columnar(block, dist, group)
        if merged is not None:
            return merged
    local_vals = [sorted(x, key=_key_order) for x in local_sets]
    gathered = [None] * world
    dist.all_gather_object(gathered, local_vals, group=group)
    gdict = [sorted(set().union(*[g[c] for g in gathered]), key=_key_order) for c in range(nk)]
    cards = [max(len(d), 1) for d in gdict]
    ndense = int(np.prod(cards, dtype=np.int64)) if nk else 1
    if ndense > max_dense_groups:
        parts = [None] * world
        dist.all_gather_object(parts, (block.groups, _stats_vector(block.stats), bool(block.num_groups_limit_reached)),
                               group=group)
        merged = {}
        for p, _, _ in parts:
            for k, v in p.items():
                merged[k] = v if k not in merged else [merge_intermediate(a.function, x, y)
                                                       for a, x, y in zip(aggs, merged[k], v)]
        stats = _stats_from(np.sum([p[1] for p in parts], axis=0))
        out = GroupByResultsBlock(aggs, block.group_by, merged, stats, any(p[2] for p in parts))
        out.key_types = getattr(block, "key_types", None)
        return out
    index = [{v: i for i, v in enumerate(d)} for d in gdict]
    strides = np.cumprod([1] + cards[:-1]).astype(np.int64)
    lay = _Layout(aggs)
    na = len(aggs)
    # SUM rows: [stats | presence count | row SUM parts]; MAX: [limit flag | row MAX parts | per-function presence]
    # (a null intermediate -- enableNullHandling, nothing non-null aggregated into that group -- contributes the
    # function's identity and presence 0; the merged group's function is null when no rank had a value)
    w = lay.nmax + na
    sv = np.zeros(6 + ndense * (1 + lay.nsum))
    mrows = np.zeros((ndense, w), np.int64)
    mrows[:, :lay.nmax] = lay.empty_max(ndense)
    sv[:6] = _stats_vector(block.stats)
    srows = sv[6:].reshape(ndense, 1 + lay.nsum)
    ident = lay.get(np.zeros(lay.nsum), lay.empty_max(1)[0])
    for k, v in block.groups.items():
        d = int(sum(index[c][k[c]] * strides[c] for c in range(nk)))
        srows[d, 0] = 1.0
        lay.put(srows[d, 1:], mrows[d, :lay.nmax], [ident[i] if x is None else x for i, x in enumerate(v)])
        mrows[d, lay.nmax:] = [x is not None for x in v]
    mv = np.concatenate([np.array([int(block.num_groups_limit_reached)], np.int64), mrows.ravel()])
    sv, mv = _sum_max(dist, group, sv, mv)
    srows = sv[6:].reshape(ndense, 1 + lay.nsum)
    mrows = mv[1:].reshape(ndense, w)
    groups = {}
    for d in np.nonzero(srows[:, 0])[0]:
        key, rem = [], int(d)
        for c in range(nk):
            key.append(gdict[c][rem % cards[c]])
            rem //= cards[c]
        vals = lay.get(srows[d, 1:], mrows[d, :lay.nmax])
        groups[tuple(key)] = [x if mrows[d, lay.nmax + i] else None for i, x in enumerate(vals)]
    out = GroupByResultsBlock(aggs, block.group_by, groups, _stats_from(sv[:6]), bool(mv[0]))
    out.key_types = getattr(block, "key_types", None)
    return out


_NUMERIC_KEYS = ("INT", "LONG", "FLOAT", "DOUBLE")


def _merge_records_columnar(block, dist, group):
    """The record merge of a large key space as columns over the communicator (GroupByCombineOperator's upsert by
    key, GroupByCombineOperator.java:138-147, across GPUs): every rank packs its groups into an int64 key matrix
    (per group-by column the value -- a FLOAT / DOUBLE as its bits -- and a null-key flag), an int64 value matrix
    (COUNTs and exact SUMs as integers, double results as their bits, a presence flag per function for null
    intermediates) and a u8 HLL register matrix; three all_gathers (RCCL on the GPUs) bring every rank's rows, and
    the rows merge by key in rank order (np.unique + np.add / minimum / maximum.at: the same answer on every rank,
    independent of arrival order). None when a group-by column is not numeric (STRING keys keep the object merge);
    every rank decides the same way."""
    aggs = block.aggregations
    nk = len(block.group_by)
    kt = getattr(block, "key_types", None)
    ok = kt is not None and len(kt) == nk and all(t in _NUMERIC_KEYS for t in kt)
    keys = list(block.groups.keys())
    vals = list(block.groups.values())
    n = len(keys)
    # per SUM / AVG: does any rank hold a double (the exact integer column then carries doubles for everyone)
    any_f = [1 if ag.function in ("sum", "avg") and any(
        v[a] is not None and not isinstance(v[a][0] if ag.function == "avg" else v[a], (int, np.integer))
        for v in vals) else 0 for a, ag in enumerate(aggs)]
    flags = _reduce(dist, group, np.array([0 if ok else 1] + any_f, dtype=np.int64), dist.ReduceOp.MAX)
    if flags[0]:
        return None
    any_f = [int(x) for x in flags[1:]]
    floats = [t in ("FLOAT", "DOUBLE") for t in kt]
    K = np.zeros((n, 2 * nk), dtype=np.int64)
    for c in range(nk):
        col = [k[c] for k in keys]
        K[:, nk + c] = [v is None for v in col]
        if floats[c]:
            x = np.array([0.0 if v is None else float(v) for v in col], dtype=np.float64)
            b = x.view(np.int64).copy()  # keyed by the bits, as the reference (doubleToLongBits): -0.0 and 0.0
            b[np.isnan(x)] = 0x7FF8000000000000  # two groups, every NaN one (results.JavaDoubleKey)
            K[:, c] = b
        else:
            K[:, c] = [0 if v is None else int(v) for v in col]
    # value columns: (kind, agg, part) with kind I (int64) / F (double bits) / P (presence)
    cols = []
    for a, ag in enumerate(aggs):
        f = ag.function
        if f == "count":
            cols.append(("I", a, None))
        elif f == "sum":
            cols.append(("F" if any_f[a] else "I", a, None))
        elif f in ("min", "max"):
            cols.append(("F", a, None))
        elif f in ("avg", "minmaxrange"):
            cols.append(("F", a, 0))
            cols.append(("I" if f == "avg" else "F", a, 1))
        cols.append(("P", a, None))
    V = np.zeros((n, len(cols)), dtype=np.int64)
    for j, (kind, a, part) in enumerate(cols):
        f = aggs[a].function
        if f in _HLL_FUNCS:
            if kind == "P":
                V[:, j] = 1
            continue
        col = [v[a] for v in vals]
        if kind == "P":
            V[:, j] = [x is not None for x in col]
            continue
        ident = {"min": float("inf"), "max": float("-inf")}.get(f, 0)
        if part is not None:
            ident = (float("inf"), float("-inf"))[part] if f == "minmaxrange" else 0
            col = [ident if x is None else x[part] for x in col]
        else:
            col = [ident if x is None else x for x in col]
        if kind == "F":
            V[:, j] = np.array(col, dtype=np.float64).view(np.int64)
        else:
            V[:, j] = np.array([int(x) for x in col], dtype=np.int64)
    # HLL registers: each function's 2^log2m (the query's, the same on every rank) side by side
    hoff, width = {}, 0
    for a, ag in enumerate(aggs):
        if ag.function in _HLL_FUNCS:
            hoff[a] = (width, 1 << ag.log2m)
            width += 1 << ag.log2m
    H = np.zeros((n, max(width, 1)), dtype=np.uint8)
    for a, (o, m) in hoff.items():
        for i, v in enumerate(vals):
            H[i, o:o + m] = np.asarray(v[a], dtype=np.uint8)[:m]
    Ka = _all_gather_rows(dist, group, K.reshape(-1)).reshape(-1, 2 * nk) if nk else np.zeros((0, 0), np.int64)
    Va = _all_gather_rows(dist, group, V.reshape(-1)).reshape(-1, len(cols))
    Ha = _all_gather_rows(dist, group, H)
    st = _reduce(dist, group, np.concatenate([_stats_vector(block.stats), [0]]), dist.ReduceOp.SUM)[:6]
    lim = _reduce(dist, group, np.array([int(block.num_groups_limit_reached)], np.int64), dist.ReduceOp.MAX)[0]
    uniq, inv = np.unique(Ka, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    G = len(uniq)
    merged_cols = []
    for j, (kind, a, part) in enumerate(cols):
        f = aggs[a].function
        if kind == "P":
            acc = np.zeros(G, dtype=np.int64)
            np.maximum.at(acc, inv, Va[:, j])
        elif kind == "I":
            acc = np.zeros(G, dtype=np.int64)
            np.add.at(acc, inv, Va[:, j])
        else:
            x = Va[:, j].view(np.float64)
            op = "min" if (f == "min" or (f == "minmaxrange" and part == 0)) else \
                ("max" if (f == "max" or (f == "minmaxrange" and part == 1)) else "sum")
            acc = np.full(G, {"min": np.inf, "max": -np.inf, "sum": 0.0}[op])
            {"min": np.minimum, "max": np.maximum, "sum": np.add}[op].at(acc, inv, x)
        merged_cols.append(acc)
    Hm = np.zeros((G, Ha.shape[1]), dtype=np.uint8)
    np.maximum.at(Hm, inv, Ha)
    groups = {}
    col_of = {}
    for j, (kind, a, part) in enumerate(cols):
        col_of[(kind == "P", a, part)] = j
    for g in range(G):
        key = []
        for c in range(nk):
            if uniq[g, nk + c]:
                key.append(None)
            elif floats[c]:
                key.append(java_double_key(float(np.int64(uniq[g, c]).view(np.float64))))
            else:
                key.append(int(uniq[g, c]))
        row = []
        for a, ag in enumerate(aggs):
            f = ag.function
            present = merged_cols[col_of[(True, a, None)]][g]
            if f in _HLL_FUNCS:
                o, m = hoff[a]
                row.append(Hm[g, o:o + m].copy())
                continue
            if not present:
                row.append(None)
                continue
            if f in ("avg", "minmaxrange"):
                x0 = merged_cols[col_of[(False, a, 0)]][g]
                x1 = merged_cols[col_of[(False, a, 1)]][g]
                row.append((float(x0), int(x1)) if f == "avg" else (float(x0), float(x1)))
            else:
                x = merged_cols[col_of[(False, a, None)]][g]
                row.append(int(x) if cols[col_of[(False, a, None)]][0] == "I" else float(x))
        groups[tuple(key)] = row
    out = GroupByResultsBlock(aggs, block.group_by, groups, _stats_from(st), bool(lim))
    out.key_types = kt
    return out


# ------------------------------------------------------------------------------------------------------
# Device-resident merge (include/pinot_hip.h "multi-GPU servers"): node-global dictionaries registered once
# at load, dense partial group tables all-reduced in place on the GPUs.
# ------------------------------------------------------------------------------------------------------
_SIGN64 = -(1 << 63)


def _column_info(seg, column):
    s = getattr(seg, "segment", seg)  # GpuSegment or ImmutableSegment
    return s.columns[column]


def _order_keys(values: np.ndarray, dt) -> np.ndarray:
    """int64 keys whose signed order is the reference's dictionary order (FLOAT / DOUBLE as Float.compare /
    Double.compare: -0.0 < 0.0, NaN last)."""
    from ..spi import DataType
    if dt in (DataType.INT, DataType.LONG):
        return values.astype(np.int64)
    if dt == DataType.FLOAT:
        u = values.astype("<f4").view(np.uint32).astype(np.int64)
        return np.where(u & 0x80000000, ~u & 0xFFFFFFFF, u | 0x80000000)
    u = values.astype("<f8").view(np.uint64)
    o = np.where(u >> np.uint64(63), ~u, u | np.uint64(1 << 63))
    return (o ^ np.uint64(1 << 63)).view(np.int64)


def _values_of_keys(keys: np.ndarray, dt) -> np.ndarray:
    from ..spi import DataType
    if dt == DataType.INT:
        return keys.astype("<i4")
    if dt == DataType.LONG:
        return keys.astype("<i8")
    if dt == DataType.FLOAT:
        u = np.where(keys & 0x80000000, keys & 0x7FFFFFFF, ~keys & 0xFFFFFFFF).astype(np.uint32)
        return u.view("<f4")
    o = keys.view(np.uint64) ^ np.uint64(1 << 63)
    u = np.where(o >> np.uint64(63), o & np.uint64((1 << 63) - 1), ~o)
    return u.view("<f8")


def _all_gather_rows(dist, group, arr: np.ndarray) -> np.ndarray:
    """Concatenation over ranks of a 1-D int64 or 2-D uint8 array whose length differs per rank."""
    import torch
    dev = _device(dist, group)
    world = dist.get_world_size(group)
    n = torch.tensor([arr.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    cap = max(max(sizes), 1)
    pad = np.zeros((cap,) + arr.shape[1:], arr.dtype)
    pad[:arr.shape[0]] = arr
    t = torch.from_numpy(pad).to(dev)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return np.concatenate([o.cpu().numpy()[:k] for o, k in zip(outs, sizes)])


def global_dictionary(segments, column, dist=None, group=None):
    """Node-global dictionary of `column`: the sorted distinct union of its dictionary values over every
    rank's segments. Returns (data type, values) -- a LE numpy array, or for STRING an
    (n, width) uint8 array of '\\0'-padded values. Exchanged once, at load: one all-gather of the local union."""
    from ..spi import DataType
    infos = [_column_info(s, column) for s in segments]
    dts = {int(ci.metadata.data_type) for ci in infos}
    if len(dts) > 1:
        raise ValueError(f"column {column} has different types across segments")
    multi = dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1
    dt = DataType(dts.pop()) if dts else None
    if multi:  # agree on the type (a rank may own no segment)
        v = _reduce(dist, group, np.array([int(dt) if dt is not None else -1], np.int64), dist.ReduceOp.MAX)
        dt = DataType(int(v[0]))
    if dt is None:
        raise ValueError(f"no segment holds column {column}")
    for ci in infos:
        if not ci.metadata.has_dictionary:
            raise ValueError(f"column {column} has no dictionary in some segment")
    if dt == DataType.STRING:
        width = max([ci.metadata.string_width for ci in infos] + [1])
        if multi:
            width = int(_reduce(dist, group, np.array([width], np.int64), dist.ReduceOp.MAX)[0])
        rows = []
        for ci in infos:
            w, card = ci.metadata.string_width, ci.metadata.cardinality
            r = np.zeros((card, width), np.uint8)
            r[:, :w] = np.frombuffer(ci.dictionary, np.uint8)[:card * w].reshape(card, w)
            rows.append(r)
        local = np.unique(np.concatenate(rows) if rows else np.zeros((0, width), np.uint8), axis=0)
        allv = _all_gather_rows(dist, group, local) if multi else local
        return dt, np.unique(allv, axis=0) if len(allv) else allv.reshape(0, width)
    code = {DataType.INT: "i4", DataType.LONG: "i8", DataType.FLOAT: "f4", DataType.DOUBLE: "f8"}[dt]
    keys = [_order_keys(np.frombuffer(ci.dictionary, ">" + code)[:ci.metadata.cardinality], dt) for ci in infos]
    local = np.unique(np.concatenate(keys)) if keys else np.zeros(0, np.int64)
    allk = np.unique(_all_gather_rows(dist, group, local)) if multi else local
    return dt, _values_of_keys(allk, dt)


def register_global_dictionaries(segments, columns, dist=None, group=None, device: int = -1):
    """phip_global_dictionary for each group-by column the server will key across GPUs (call once after the
    segments are loaded, on every rank). Plans created afterwards key those columns by the global ids."""
    import ctypes
    from .. import _lib
    from ..spi import DataType
    lib = _lib.load()
    out = {}
    for col in columns:
        dt, vals = global_dictionary(segments, col, dist, group)
        vals = np.ascontiguousarray(vals)
        width = vals.shape[1] if dt == DataType.STRING else 0
        card = vals.shape[0]
        _lib.check(lib.phip_global_dictionary(device, col.encode(), int(dt), card, width,
                                              vals.ctypes.data_as(ctypes.c_void_p) if card else None))
        out[col] = (dt, vals)
    return out


def unregister_global_dictionaries(columns, device: int = -1):
    """Drop the node-global dictionaries of `columns` (plans created afterwards use query-global ones)."""
    from .. import _lib
    lib = _lib.load()
    for col in columns:
        _lib.check(lib.phip_global_dictionary(device, col.encode(), 0, -1, 0, None))


class _DeviceArray:
    """__cuda_array_interface__ view of device memory the library owns (torch.as_tensor wraps it, no copy)."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"data": (int(ptr), False), "shape": tuple(shape), "typestr": typestr,
                                         "version": 2}


def partial_tensors(part):
    """(table [num_rows, G] int64, hll [num_hll * G * m] int32 or None) aliasing the partial's device buffers."""
    import torch
    dev = torch.device("cuda", part.device)
    table = torch.as_tensor(_DeviceArray(part.table, (part.num_rows, part.num_groups), "<i8"), device=dev)
    hll = None
    if part.num_hll:
        n = part.num_hll * part.num_groups * (1 << part.log2m)
        hll = torch.as_tensor(_DeviceArray(part.hll, (n,), "<i4"), device=dev)
    return table, hll


def _rows_op(dist, group, table, rows, op):
    if not rows:
        return
    lo, hi = min(rows), max(rows)
    if hi - lo + 1 == len(rows):  # contiguous: reduce the view in place
        dist.all_reduce(table[lo:hi + 1], op=op, group=group)
        return
    idx = list(rows)
    sub = table[idx].contiguous()
    dist.all_reduce(sub, op=op, group=group)
    table[idx] = sub


def allreduce_partial_table(table, hll, kinds, stats, dist, group=None, any_f64=None):
    """Merge this rank's dense partial table with every other rank's, in place (torch tensors on the
    communicator's device: RCCL over xGMI on the GPU server, gloo in CPU tests). `kinds` are the rows'
    phip_partial row kinds. One collective per reduce operator and type:
      int64 SUM    COUNT / SUM_I64 rows and the six execution statistics, staged together;
      float64 SUM  SUM_F64 rows;
      int64 MAX    MAX rows as the signed image of their order-preserving u64 (sign bit flipped) and MIN rows as
                   the complement of that image (order reversed, so the MAX of it is the MIN);
      uint8 MAX    HLL registers (held as u32 by the library, exchanged as bytes).
    A row that is an exact int64 sum here but a double sum on another rank (the overflow bound is per GPU) is
    converted to doubles first: `any_f64[r]` says whether any rank holds row r in double (distributed_block
    exchanges it with its shape check; None = exchange it here). Returns (merged kinds, merged stats)."""
    import torch
    from .. import _lib
    S, MAX = dist.ReduceOp.SUM, dist.ReduceOp.MAX
    kinds = list(kinds)
    dev = table.device
    if any_f64 is None:
        f64 = torch.tensor([1 if k == _lib.ROW_SUM_F64 else 0 for k in kinds], dtype=torch.int64, device=dev)
        dist.all_reduce(f64, op=MAX, group=group)
        any_f64 = [int(x) for x in f64.cpu().tolist()]
    for r, k in enumerate(kinds):
        if k == _lib.ROW_SUM_I64 and any_f64[r]:
            table[r].copy_(table[r].to(torch.float64).view(torch.int64))
            kinds[r] = _lib.ROW_SUM_F64
    ints = [r for r, k in enumerate(kinds) if k in (_lib.ROW_COUNT, _lib.ROW_SUM_I64, _lib.ROW_HLL)]
    dbls = [r for r, k in enumerate(kinds) if k == _lib.ROW_SUM_F64]
    mins = [r for r, k in enumerate(kinds) if k == _lib.ROW_MIN]
    maxs = [r for r, k in enumerate(kinds) if k == _lib.ROW_MAX]
    ng = table.shape[1]
    st = torch.tensor(list(stats), dtype=torch.int64, device=dev)
    stage = torch.cat([table[ints].reshape(-1), st]) if ints else st
    dist.all_reduce(stage, op=S, group=group)
    if ints:
        table[ints] = stage[:len(ints) * ng].view(len(ints), ng)
    if dbls:
        _rows_op(dist, group, table.view(torch.float64), dbls, S)
    if mins or maxs:
        rows = mins + maxs
        sub = table[rows].bitwise_xor(_SIGN64)
        nm = len(mins)
        if nm:
            sub[:nm] = sub[:nm].bitwise_not()
        dist.all_reduce(sub, op=MAX, group=group)
        if nm:
            sub[:nm] = sub[:nm].bitwise_not()
        table[rows] = sub.bitwise_xor(_SIGN64)
    if hll is not None:
        h8 = hll.to(torch.uint8)  # registers are <= 64: one byte each on the wire instead of four
        dist.all_reduce(h8, op=MAX, group=group)
        hll.copy_(h8)
    return kinds, [int(x) for x in stage[-6:].cpu().tolist()]


def _finish_agg_via_host(op, part, dist, group, any_f64):
    """The aggregation partial merged over a CPU communicator (gloo tests on one GPU): table + statistics + registers
    staged through host tensors, then copied back before phip_plan_finish."""
    import torch
    dev = torch.device("cuda", part.device)
    nr = part.num_rows
    buf = torch.as_tensor(_DeviceArray(part.table, (nr + 6,), "<i8"), device=dev)
    hb = buf.cpu()
    kinds = [part.row_kinds[r] for r in range(nr)]
    t2 = hb[:nr].view(nr, 1).clone()
    kinds2, stats = allreduce_partial_table(t2, None, kinds, hb[nr:].tolist(), dist, group, any_f64)
    hb[:nr] = t2.view(-1)
    hb[nr:] = torch.tensor(stats, dtype=torch.int64)
    buf.copy_(hb)
    if part.num_hll:
        h = torch.as_tensor(_DeviceArray(part.hll, (part.num_hll << part.log2m,), "|u1"), device=dev)
        hh = h.cpu()
        dist.all_reduce(hh, op=dist.ReduceOp.MAX, group=group)
        h.copy_(hh)
    torch.cuda.current_stream(dev).synchronize()
    for r, k in enumerate(kinds2):
        part.row_kinds[r] = k
    return op.finish(part)


def allreduce_aggregation_partial(part, dist, group=None, any_f64=None):
    """Merge an aggregation-only plan's one-group partial (phip_plan_execute_partial) across ranks in place, on the
    device: when every row sums as int64 (COUNT, exact SUMs -- SSB Q1.x) the rows and the statistics after them are
    one contiguous int64 SUM all-reduce, plus one uint8 MAX for HLL registers; other mixes go through
    allreduce_partial_table (one collective per reduce operator) with the statistics staged from the host."""
    import torch
    from .. import _lib
    dev = torch.device("cuda", part.device)
    nr = part.num_rows
    kinds = [part.row_kinds[r] for r in range(nr)]
    if any_f64 is None:
        any_f64 = [0] * nr
    hll = None
    if part.num_hll:
        hll = torch.as_tensor(_DeviceArray(part.hll, (part.num_hll << part.log2m,), "|u1"), device=dev)
    if all(k in (_lib.ROW_COUNT, _lib.ROW_SUM_I64, _lib.ROW_HLL) for k in kinds) and not any(any_f64[:nr]):
        buf = torch.as_tensor(_DeviceArray(part.table, (nr + 6,), "<i8"), device=dev)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        if hll is not None:
            dist.all_reduce(hll, op=dist.ReduceOp.MAX, group=group)
        torch.cuda.current_stream(dev).synchronize()
        return
    table = torch.as_tensor(_DeviceArray(part.table, (nr, 1), "<i8"), device=dev)
    kinds2, stats = allreduce_partial_table(table, None, kinds, list(part.stats), dist, group, any_f64)
    if hll is not None:
        dist.all_reduce(hll, op=dist.ReduceOp.MAX, group=group)
    torch.cuda.current_stream(dev).synchronize()
    for r, k in enumerate(kinds2):
        part.row_kinds[r] = k
    for i, x in enumerate(stats):
        part.stats[i] = x
    part.stats_dev = None  # (phip_plan_finish takes the host statistics)


MAX_EXACT_RANKS = 16  # runtime.cpp: exact int64 SUMs are bounded by 2^58 per GPU, 16 x 2^58 = 2^62


def distributed_block(op, dist=None, group=None, fallback_op=None):
    """This rank's share of a query merged with every other rank's; every rank returns the merged block.

    Group-by over registered global dictionaries takes the device path: each rank's dense partial table
    (phip_plan_execute_partial) is all-reduced in place on the GPUs, then phip_plan_finish compacts and trims
    it (the server-level trim runs once, after the merge). When any rank cannot hand out a dense table (hash
    key space, numGroupsLimit reached), every rank falls back to the record merge (allreduce_block) over
    `fallback_op` (an operator of the same query made with device_trim=False). Aggregation-only queries
    merge their result slots with one SUM and one MAX all-reduce (allreduce_block). A rank whose execution
    raises tells the others through the shape check, so every rank raises instead of waiting in a collective."""
    import torch
    from .. import _lib
    if dist is None:
        import torch.distributed as dist
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    if not multi:
        return op.next_block()
    if not hasattr(op, "execute_partial"):
        return allreduce_block(op.next_block(), dist, group)
    err = None
    part = None
    try:
        _lib.load(with_torch=True)  # (torch's HIP runtime: the library must share it, _lib.load)
        part = op.execute_partial()
    except Exception as e:  # noqa: BLE001 -- re-raised below, after the other ranks learned of it
        part, err = None, e
    dev = _device(dist, group)
    shape = [0, 0, 0] if part is None or not part.global_keys else [1, part.num_groups, part.num_rows]
    nrow = _lib.PARTIAL_MAX_ROWS
    # an exact int64 partial is bounded by 2^58 per GPU (the library's plan-time bound), so the int64 SUM of up to
    # MAX_EXACT_RANKS of them cannot wrap; past that every SUM row merges in double (the reference's own type)
    wide = dist.get_world_size(group) > MAX_EXACT_RANKS
    f64 = [1 if shape[0] and r < part.num_rows and (part.row_kinds[r] == _lib.ROW_SUM_F64 or
                                                    (wide and part.row_kinds[r] == _lib.ROW_SUM_I64)) else 0
           for r in range(nrow)]
    v = torch.tensor([1 if err is not None else 0, 1 - shape[0], shape[1], shape[2], -shape[1], -shape[2]] + f64,
                     dtype=torch.int64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX, group=group)
    v = [int(x) for x in v.cpu().tolist()]
    if v[0]:
        if part is not None:  # the plan must not stay blocked behind a table nobody will finish
            op.abandon_partial()
        if err is not None:
            raise err
        raise RuntimeError("the query failed on another rank (distributed_block)")
    if v[1] == 0 and v[2] == -v[4] and v[3] == -v[5]:
        try:
            any_f64 = v[6:6 + part.num_rows]
            if not getattr(op.query, "group_by", None):  # aggregation-only: the one-group table, merged in place
                if _device(dist, group).type != "cuda":  # (gloo over host memory: stage through the host)
                    return _finish_agg_via_host(op, part, dist, group, any_f64)
                allreduce_aggregation_partial(part, dist, group, any_f64)
                return op.finish(part)
            table, hll = partial_tensors(part)
            kinds = [part.row_kinds[r] for r in range(part.num_rows)]
            if table.device != dev:  # (gloo over host memory: stage through the host, CPU-communicator tests)
                t2, h2 = table.to(dev), (hll.to(dev) if hll is not None else None)
                kinds, stats = allreduce_partial_table(t2, h2, kinds, list(part.stats), dist, group, any_f64)
                table.copy_(t2)
                if hll is not None:
                    hll.copy_(h2)
            else:
                kinds, stats = allreduce_partial_table(table, hll, kinds, list(part.stats), dist, group, any_f64)
            torch.cuda.current_stream(table.device).synchronize()
            for r, k in enumerate(kinds):
                part.row_kinds[r] = k
            for i, x in enumerate(stats):
                part.stats[i] = x
            return op.finish(part)
        except BaseException:
            try:  # a failed merge or finish leaves the table pending: hand it back so the plan runs again
                op.abandon_partial()
            except Exception:  # noqa: BLE001 -- the original error is the one to report
                pass
            raise
    if part is not None:  # this rank's table was handed out but the ranks merge records: give it back
        op.abandon_partial()
    err = None
    try:
        blk = (fallback_op or op).next_block()
    except Exception as e:  # noqa: BLE001 -- every rank learns of it before raising (no rank left in a collective)
        blk, err = None, e
    f = torch.tensor([1 if err is not None else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(f, op=dist.ReduceOp.MAX, group=group)
    if int(f.item()):
        if err is not None:
            raise err
        raise RuntimeError("the query failed on another rank (distributed_block record merge)")
    return allreduce_block(blk, dist, group)
