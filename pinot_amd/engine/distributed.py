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


def allreduce_partial_table(table, hll, kinds, stats, dist, group=None):
    """Merge this rank's dense partial table with every other rank's, in place (torch tensors on the
    communicator's device: RCCL over xGMI on the GPU server, gloo in CPU tests). `kinds` are the rows'
    phip_partial row kinds (COUNT / SUM_I64 -> int64 SUM, SUM_F64 -> float64 SUM, MIN / MAX on the
    order-preserving u64 image -> signed MIN / MAX after flipping the sign bit, HLL registers -> int32 MAX).
    A row that is an exact int64 sum here but a double sum on another rank (the overflow bound is per
    GPU) is converted to doubles first. Returns (merged kinds, merged stats)."""
    import torch
    from .. import _lib
    S, MIN, MAX = dist.ReduceOp.SUM, dist.ReduceOp.MIN, dist.ReduceOp.MAX
    kinds = list(kinds)
    dev = table.device
    f64 = torch.tensor([1 if k == _lib.ROW_SUM_F64 else 0 for k in kinds], dtype=torch.int64, device=dev)
    dist.all_reduce(f64, op=MAX, group=group)
    for r, k in enumerate(kinds):
        if k == _lib.ROW_SUM_I64 and int(f64[r]):
            table[r].copy_(table[r].to(torch.float64).view(torch.int64))
            kinds[r] = _lib.ROW_SUM_F64
    ints = [r for r, k in enumerate(kinds) if k in (_lib.ROW_COUNT, _lib.ROW_SUM_I64, _lib.ROW_HLL)]
    dbls = [r for r, k in enumerate(kinds) if k == _lib.ROW_SUM_F64]
    mins = [r for r, k in enumerate(kinds) if k == _lib.ROW_MIN]
    maxs = [r for r, k in enumerate(kinds) if k == _lib.ROW_MAX]
    _rows_op(dist, group, table, ints, S)
    if dbls:
        tf = table.view(torch.float64)
        _rows_op(dist, group, tf, dbls, S)
    for rows, op in ((mins, MIN), (maxs, MAX)):
        if rows:
            for r in rows:
                table[r].bitwise_xor_(_SIGN64)
            _rows_op(dist, group, table, rows, op)
            for r in rows:
                table[r].bitwise_xor_(_SIGN64)
    if hll is not None:
        dist.all_reduce(hll, op=MAX, group=group)
    st = torch.tensor(list(stats), dtype=torch.int64, device=dev)
    dist.all_reduce(st, op=S, group=group)
    return kinds, [int(x) for x in st.cpu().tolist()]


def distributed_block(op, dist=None, group=None, fallback_op=None):
    """This rank's share of a query merged with every other rank's; every rank returns the merged block.

    Group-by over registered global dictionaries takes the device path: each rank's dense partial table
    (phip_plan_execute_partial) is all-reduced in place on the GPUs, then phip_plan_finish compacts and trims
    it (the server-level trim runs once, after the merge). When any rank cannot hand out a dense table (hash
    key space, numGroupsLimit reached), every rank falls back to the record merge (allreduce_block) over
    `fallback_op` (an operator of the same query made with device_trim=False). Aggregation-only queries
    all-reduce the few result slots (allreduce_block)."""
    import torch
    if dist is None:
        import torch.distributed as dist
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    if not multi:
        return op.next_block()
    if not getattr(op.query, "group_by", None) or not hasattr(op, "execute_partial"):
        return allreduce_block(op.next_block(), dist, group)
    part = op.execute_partial()
    dev = _device(dist, group)
    shape = [0, 0, 0] if part is None or not part.global_keys else [1, part.num_groups, part.num_rows]
    v = torch.tensor([1 - shape[0], shape[1], shape[2], -shape[1], -shape[2]], dtype=torch.int64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX, group=group)
    v = [int(x) for x in v.cpu().tolist()]
    if v[0] == 0 and v[1] == -v[3] and v[2] == -v[4]:
        table, hll = partial_tensors(part)
        kinds = [part.row_kinds[r] for r in range(part.num_rows)]
        if table.device != dev:  # (gloo over host memory: stage through the host, CPU-communicator tests)
            t2, h2 = table.to(dev), (hll.to(dev) if hll is not None else None)
            kinds, stats = allreduce_partial_table(t2, h2, kinds, list(part.stats), dist, group)
            table.copy_(t2)
            if hll is not None:
                hll.copy_(h2)
        else:
            kinds, stats = allreduce_partial_table(table, hll, kinds, list(part.stats), dist, group)
        torch.cuda.current_stream(table.device).synchronize()
        for r, k in enumerate(kinds):
            part.row_kinds[r] = k
        for i, x in enumerate(stats):
            part.stats[i] = x
        return op.finish(part)
    blk = (fallback_op or op).next_block()
    return allreduce_block(blk, dist, group)
