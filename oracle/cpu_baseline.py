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
