"""bench.py's cpu_baseline leg -- TEST / BENCH INFRASTRUCTURE ONLY (see oracle/__init__.py).

Drives oracle/cpu_scan.c, the OpenMP C restatement of Pinot's CPU server path for conjunctive dict-id
filters + SUM(column expression) (the SSB Q1.x shape), over the same segments the GPU holds. Predicates
become dict-id ranges through each segment's own dictionary (RangePredicateEvaluatorFactory /
EqualsPredicateEvaluatorFactory semantics, a binary search per segment -- host-side planning, outside the
timed region, as the plan build is for the GPU). Label: "restatement, not Pinot".
"""
import ctypes
import os
import time

import numpy as np

from . import build as _build

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libcpuscan.so")
_MAX_LEAVES = 8


class _Leaf(ctypes.Structure):
    _fields_ = [("fwd", ctypes.c_void_p), ("bits", ctypes.c_int32), ("sorted", ctypes.c_int32),
                ("lo", ctypes.c_int32), ("hi", ctypes.c_int32)]


class _Seg(ctypes.Structure):
    _fields_ = [("num_docs", ctypes.c_int32), ("nleaves", ctypes.c_int32), ("leaves", _Leaf * _MAX_LEAVES),
                ("fwd_a", ctypes.c_void_p), ("dict_a", ctypes.c_void_p), ("fwd_b", ctypes.c_void_p),
                ("dict_b", ctypes.c_void_p), ("bits_a", ctypes.c_int32), ("bits_b", ctypes.c_int32),
                ("expr", ctypes.c_int32), ("pad", ctypes.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            _build()
        L = ctypes.CDLL(_SO)
        L.cb_run.argtypes = [ctypes.POINTER(_Seg), ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
        L.cb_run.restype = ctypes.c_double
        L.cb_max_threads.restype = ctypes.c_int32
        _lib = L
    return _lib


def _dict_range(d, pred):
    """Matching dict ids [lo, hi) of an EQ / RANGE predicate over a sorted INT dictionary."""
    if pred.type == "EQ":
        v = int(pred.values[0])
        lo = int(np.searchsorted(d, v, "left"))
        return lo, lo + 1 if lo < len(d) and d[lo] == v else lo
    if pred.type != "RANGE":
        raise NotImplementedError(pred.type)
    lo, hi = 0, len(d)
    if pred.lower != "*":
        lo = int(np.searchsorted(d, float(pred.lower), "left" if pred.lower_inclusive else "right"))
    if pred.upper != "*":
        hi = int(np.searchsorted(d, float(pred.upper), "right" if pred.upper_inclusive else "left"))
    return lo, max(lo, hi)


def _padded(b):
    return np.frombuffer(b + b"\0" * 16, dtype=np.uint8)


def _expr(e):
    from pinot_amd.query.context import Function, Identifier
    while isinstance(e, Function) and e.name == "cast":
        e = e.args[0]
    if isinstance(e, Identifier):
        return 0, e.name, None
    ops = {"plus": 1, "minus": 2, "times": 3}
    if isinstance(e, Function) and e.name in ops:
        a, b = _expr(e.args[0]), _expr(e.args[1])
        if a[0] == 0 and b[0] == 0:
            return ops[e.name], a[1], b[1]
    raise NotImplementedError(str(e))


class Prepared:
    """One query over a list of ImmutableSegments, ready to run (buffers kept alive here)."""

    def __init__(self, qc, segments):
        if len(qc.aggregations) != 1 or qc.aggregations[0].function != "sum" or qc.group_by:
            raise NotImplementedError("cpu baseline: one SUM, no GROUP BY")
        expr, ca, cb = _expr(qc.aggregations[0].argument)
        preds = []
        f = qc.filter
        if f is not None:
            kids = f.children if f.type == "AND" else [f]
            for k in kids:
                if k.type != "PREDICATE":
                    raise NotImplementedError("cpu baseline: AND of predicates")
                preds.append(k.predicate)
        if len(preds) > _MAX_LEAVES:
            raise NotImplementedError("too many leaves")
        self.keep = []
        self.segs = (_Seg * len(segments))()
        for i, seg in enumerate(segments):
            s = self.segs[i]
            s.num_docs = seg.num_docs
            s.nleaves = len(preds)
            for j, p in enumerate(preds):
                ci = seg.columns[p.column]
                d = np.frombuffer(ci.dictionary, dtype=">i4").astype(np.int64)
                lo, hi = _dict_range(d, p)
                fwd = _padded(ci.forward)
                self.keep.append(fwd)
                s.leaves[j] = _Leaf(fwd.ctypes.data, ci.metadata.bits_per_element, int(ci.metadata.is_sorted), lo, hi)
            for col, fa, da, ba in ((ca, "fwd_a", "dict_a", "bits_a"), (cb, "fwd_b", "dict_b", "bits_b")):
                if col is None:
                    continue
                ci = seg.columns[col]
                if ci.metadata.is_sorted or not ci.metadata.has_dictionary or int(ci.metadata.data_type) != 0:
                    raise NotImplementedError("cpu baseline: projected columns are unsorted dictionary INTs")
                fwd, dic = _padded(ci.forward), _padded(ci.dictionary)
                self.keep += [fwd, dic]
                setattr(s, fa, fwd.ctypes.data)
                setattr(s, da, dic.ctypes.data)
                setattr(s, ba, ci.metadata.bits_per_element)
            s.expr = expr

    def run(self, threads):
        m = ctypes.c_int64(0)
        total = lib().cb_run(self.segs, len(self.segs), threads, ctypes.byref(m))
        return total, m.value


def usable_cpus():
    """(cpus this process may run on, how that was found): the affinity mask (os.sched_getaffinity), capped by
    the cgroup CPU quota when one is set (a GPU box's share of a larger host: nproc shows the host's CPUs, the
    quota how many of them the process gets). SURVEY.md §8(d): the CPU baseline runs one worker per such CPU,
    as maxExecutionThreads = cores would (QueryMultiThreadingUtils.java:46-65)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        quota = None
    n = min(aff, quota) if quota else aff
    return n, f"sched_getaffinity {aff}, cgroup cpu.max quota {quota if quota else 'none'}, nproc {os.cpu_count()}"


def time_queries(qcs, segments, threads=None, min_seconds=2.0, max_reps=100000):
    """Runs every query over all segments with `threads` workers (default: usable_cpus()), repeated until
    min_seconds have passed; returns (rows scanned per second, threads, reps, results). Rows = sum of
    numTotalDocs per query run."""
    threads = threads or usable_cpus()[0]
    preps = [Prepared(q, segments) for q in qcs]
    rows_per_rep = sum(s.num_docs for s in segments) * len(preps)
    results = [p.run(threads) for p in preps]  # warm-up (page-in)
    t0 = time.perf_counter()
    reps = 0
    while True:
        for p in preps:
            p.run(threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_seconds or reps >= max_reps:
            break
    return rows_per_rep * reps / el, threads, reps, el, results


# ------------------------------------------------------------------------------------------------ group-by
_CG_MAX_LEAVES = 8
_CG_MAX_KEYS = 6


class _Col(ctypes.Structure):
    _fields_ = [("fwd", ctypes.c_void_p), ("bits", ctypes.c_int32), ("sorted", ctypes.c_int32),
                ("card", ctypes.c_int32), ("pad", ctypes.c_int32)]


class _GSeg(ctypes.Structure):
    _fields_ = [("num_docs", ctypes.c_int32), ("nleaves", ctypes.c_int32), ("nkeys", ctypes.c_int32),
                ("nvals", ctypes.c_int32), ("leaf_col", _Col * _CG_MAX_LEAVES),
                ("leaf_match", ctypes.c_void_p * _CG_MAX_LEAVES), ("key_col", _Col * _CG_MAX_KEYS),
                ("key_remap", ctypes.c_void_p * _CG_MAX_KEYS), ("val_col", _Col * 2), ("val_dict", ctypes.c_void_p * 2),
                ("hll_col", _Col), ("hll_dict", ctypes.c_void_p)]


class _GQuery(ctypes.Structure):
    _fields_ = [("nkeys", ctypes.c_int32), ("expr", ctypes.c_int32), ("log2m", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("radix", ctypes.c_int64 * _CG_MAX_KEYS), ("num_keys", ctypes.c_int64)]


def _group_lib():
    L = lib()
    if not getattr(L, "_cg_ready", False):
        L.cg_run.argtypes = [ctypes.POINTER(_GQuery), ctypes.POINTER(_GSeg), ctypes.c_int32, ctypes.c_int32,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.cg_run.restype = ctypes.c_int32
        L._cg_ready = True
    return L


def _leaf_predicates(f):
    """The filter as an AND of per-column leaves: each child a predicate or an OR of predicates on one column
    (the SSB Q2.x-Q4.x shapes). Returns [(column, [predicates])]."""
    if f is None:
        return []
    kids = f.children if f.type == "AND" else (f,)
    out = []
    for k in kids:
        if k.type == "PREDICATE":
            out.append((k.predicate.column, [k.predicate]))
        elif k.type == "OR" and all(c.type == "PREDICATE" for c in k.children) and \
                len({c.predicate.column for c in k.children}) == 1:
            out.append((k.children[0].predicate.column, [c.predicate for c in k.children]))
        else:
            raise NotImplementedError("cpu group-by baseline: AND of per-column leaves")
    if len(out) > _CG_MAX_LEAVES:
        raise NotImplementedError("too many leaves")
    return out


def _col(ci):
    m = ci.metadata
    return _Col(0, m.bits_per_element, int(m.is_sorted), m.cardinality, 0)


class PreparedGroupBy:
    """One SSB-shaped group-by (C3: Q2.x-Q4.x; C5) over a list of ImmutableSegments, for oracle/cpu_scan.c's
    cg_run: leaves = per-dict-id match tables evaluated on the dictionary VALUES (oracle.executor's predicate
    semantics), group keys remapped to query-global dict ids (the union of the segments' dictionaries, sorted),
    at most one SUM of a dictionary INT expression and one DISTINCTCOUNTHLL of a dictionary INT column."""

    def __init__(self, qc, segments):
        from pinot_amd.query.context import Identifier

        from .executor import OracleSegment, _pred_on_values
        if not qc.group_by or not all(isinstance(e, Identifier) for e in qc.group_by):
            raise NotImplementedError("cpu group-by baseline: GROUP BY columns")
        if len(qc.group_by) > _CG_MAX_KEYS:
            raise NotImplementedError("too many group-by columns")
        self.qc = qc
        self.key_cols = [e.name for e in qc.group_by]
        self.sum_agg = self.hll_agg = None
        expr, ca, cb = -1, None, None
        self.log2m = 0
        hll_col = None
        for i, a in enumerate(qc.aggregations):
            if a.function == "sum" and self.sum_agg is None:
                self.sum_agg = i
                expr, ca, cb = _expr(a.argument)
            elif a.function == "distinctcounthll" and self.hll_agg is None and isinstance(a.argument, Identifier):
                self.hll_agg, self.log2m, hll_col = i, a.log2m, a.argument.name
            elif a.function == "count" and a.argument is None:
                pass
            else:
                raise NotImplementedError(f"cpu group-by baseline: {a.function}")
        leaves = _leaf_predicates(qc.filter)
        osegs = [OracleSegment(s) for s in segments]
        # query-global dictionaries of the key columns: the union of every segment's values, sorted
        self.global_dicts = []
        for c in self.key_cols:
            self.global_dicts.append(np.unique(np.concatenate([o.dictionary(c) for o in osegs])))
        cards = [len(g) for g in self.global_dicts]
        radix, r = [], 1
        for card in cards:
            radix.append(r)
            r *= card
        self.num_keys = r
        self.query = _GQuery(len(self.key_cols), expr, self.log2m, 0, (ctypes.c_int64 * _CG_MAX_KEYS)(*radix), r)
        self.keep = []
        self.segs = (_GSeg * len(segments))()

        def keep(a):
            self.keep.append(a)
            return a.ctypes.data

        for i, (seg, o) in enumerate(zip(segments, osegs)):
            s = self.segs[i]
            s.num_docs = seg.num_docs
            s.nleaves = len(leaves)
            for j, (c, preds) in enumerate(leaves):
                ci = seg.columns[c]
                d = o.dictionary(c)
                hit = np.zeros(len(d), dtype=bool)
                for p in preds:
                    hit |= _pred_on_values(p, d, ci.metadata)
                col = _col(ci)
                col.fwd = keep(_padded(ci.forward))
                s.leaf_col[j] = col
                s.leaf_match[j] = keep(np.ascontiguousarray(hit.astype(np.uint8)))
            s.nkeys = len(self.key_cols)
            for j, c in enumerate(self.key_cols):
                ci = seg.columns[c]
                col = _col(ci)
                col.fwd = keep(_padded(ci.forward))
                s.key_col[j] = col
                remap = np.searchsorted(self.global_dicts[j], o.dictionary(c)).astype(np.int32)
                s.key_remap[j] = keep(np.ascontiguousarray(remap))
            vals = [c for c in (ca, cb) if c is not None]
            s.nvals = len(vals)
            for j, c in enumerate(vals + ([hll_col] if hll_col else [])):
                ci = seg.columns[c]
                if not ci.metadata.has_dictionary or int(ci.metadata.data_type) != 0:
                    raise NotImplementedError("cpu group-by baseline: value columns are dictionary INTs")
                col = _col(ci)
                col.fwd = keep(_padded(ci.forward))
                dic = keep(_padded(ci.dictionary))
                if j < len(vals):
                    s.val_col[j] = col
                    s.val_dict[j] = dic
                else:
                    s.hll_col = col
                    s.hll_dict = dic
        m = (1 << self.log2m) if self.log2m else 0
        if m and self.num_keys * m * 32 > (4 << 30):
            raise NotImplementedError("cpu group-by baseline: HLL registers of a key space this large")

    def run(self, threads):
        """(sums, counts, registers or None, matched docs) over the dense key space."""
        m = (1 << self.log2m) if self.log2m else 0
        sums = np.empty(self.num_keys, dtype=np.int64)
        counts = np.empty(self.num_keys, dtype=np.int64)
        regs = np.empty(self.num_keys * m if m else 1, dtype=np.uint8)
        matched = ctypes.c_int64(0)
        rc = _group_lib().cg_run(ctypes.byref(self.query), self.segs, len(self.segs), threads, sums.ctypes.data,
                                 counts.ctypes.data, regs.ctypes.data, ctypes.byref(matched))
        if rc != 0:
            raise RuntimeError("cg_run failed")
        return sums, counts, (regs.reshape(self.num_keys, m) if m else None), matched.value

    def groups(self, out):
        """{key value tuple: (exact SUM or None, count, registers or None)} of the groups with matched docs, keys in
        GROUP BY order (the results blocks' key tuples)."""
        sums, counts, regs, _ = out
        nz = np.nonzero(counts)[0]
        res = {}
        ids = []
        rem = nz.copy()
        for g in self.global_dicts:
            ids.append(rem % len(g))
            rem //= len(g)
        cols = [g[i] for g, i in zip(self.global_dicts, ids)]
        for n, k in enumerate(nz):
            key = tuple(c[n].item() if hasattr(c[n], "item") else c[n] for c in cols)
            res[key] = (int(sums[k]) if self.sum_agg is not None else None, int(counts[k]),
                        regs[k] if regs is not None else None)
        return res


def time_group_by(qcs, segments, threads=None, min_seconds=2.0, max_reps=100000):
    """Every group-by query over all segments, repeated until min_seconds have passed; returns (rows scanned per
    second, threads, reps, seconds). Rows = numTotalDocs per query run."""
    threads = threads or usable_cpus()[0]
    preps = [PreparedGroupBy(q, segments) for q in qcs]
    rows_per_rep = sum(s.num_docs for s in segments) * len(preps)
    for p in preps:
        p.run(threads)
    t0 = time.perf_counter()
    reps = 0
    while True:
        for p in preps:
            p.run(threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_seconds or reps >= max_reps:
            break
    return rows_per_rep * reps / el, threads, reps, el
