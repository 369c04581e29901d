"""Drives the node-plan paths of libpinot_hip (node.cpp: one query over segments on several devices) against the HIP
stand-in under ASan: HOSTSIM_DEVICES stand-in devices, segments spread over them, the dense exchange (the peer merge:
the stand-in has no RCCL), the record merge (aggregation-only, hash-table key spaces) and the sub-plans' descriptors.
The stand-in's aggregation kernels mark key 0 of every dense table with one doc, so the merged table holds that group
(the stand-in's merge kernels run on the host; its gather writes a fixed pattern, so values are not checked here --
tests/test_gpu_node.py checks them against the oracle on the GPU)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pinot_amd import _lib  # noqa: E402

_lib.LIB_PATH = sys.argv[1]
from pinot_amd.engine.plan import GpuCombineOperator, GpuInstancePlanMaker  # noqa: E402
from pinot_amd.engine.segment import GpuSegment  # noqa: E402
from pinot_amd.query.sql import parse  # noqa: E402
from pinot_amd.segment.creator import SegmentCreator  # noqa: E402
from pinot_amd.spi import DataType  # noqa: E402

ndev = int(os.environ["HOSTSIM_DEVICES"])
lib = _lib.load()
_lib.check(lib.phip_init((ctypes.c_int32 * ndev)(*range(ndev)), ndev))
rng = np.random.default_rng(5)
segs = []
for k in range(2 * ndev):
    n = 3000 + 17 * k
    c = SegmentCreator(f"n{k}", no_dictionary_columns=["r"])
    c.add_column("g", DataType.STRING, np.array([f"k{x}" for x in rng.integers(k, 9 + k, n)]))
    c.add_column("h", DataType.INT, rng.integers(0, 5 + k, n))
    c.add_column("m", DataType.LONG, rng.integers(-10 ** 6, 10 ** 6, n))
    c.add_column("r", DataType.LONG, rng.integers(0, 50, n))
    segs.append(GpuSegment(c.build(), device=k % ndev))
pm = GpuInstancePlanMaker()
os.environ["PHIP_NODE_EXCHANGE"] = "peer"
dense = GpuCombineOperator(parse("SELECT h, g, COUNT(*), SUM(m), MAX(m) FROM t GROUP BY h, g LIMIT 1000"), segs, 100000)
blk = dense.next_block()
parts, kind = dense.exchange()
assert parts == ndev and kind == _lib.EXCHANGE_PEER, (parts, kind)
assert len(blk.groups) == 1, blk.groups  # key 0, marked in every part's table
assert len(blk.segment_docs_matched) == len(segs), blk.segment_docs_matched
assert blk.stats.num_segments_processed == len(segs), blk.stats
dense.close()
# hash-table key space (forced): the parts' tables are inserted into the root's by key (node_merge.hip hash_merge_*)
os.environ["PHIP_GB_HASH"] = "1"
hashed = GpuCombineOperator(parse("SELECT h, g, COUNT(*), SUM(m), MAX(m) FROM t GROUP BY h, g LIMIT 1000"), segs, 100000)
hashed.next_block()
parts, kind = hashed.exchange()
assert parts == ndev and kind == _lib.EXCHANGE_HASH, (parts, kind)
hashed.close()
del os.environ["PHIP_GB_HASH"]
for q in ("SELECT COUNT(*), SUM(m), MIN(m), DISTINCTCOUNTHLL(h) FROM t WHERE h < 3",  # one group: the host merge
          "SELECT r, COUNT(*), SUM(m) FROM t GROUP BY r LIMIT 1000",  # raw key: each device its own ids -> records
          "SELECT g, h, SUM(m) FROM t GROUP BY g, h ORDER BY SUM(m) DESC LIMIT 3"):  # trim: the record sub-plans
    op = GpuCombineOperator(parse(q), segs, 100000)
    op.next_block()
    parts, kind = op.exchange()
    assert parts == ndev and kind in (_lib.EXCHANGE_RECORDS, _lib.EXCHANGE_PEER), (q, parts, kind)
    if "GROUP BY r" in q or "GROUP BY" not in q:
        assert kind == _lib.EXCHANGE_RECORDS, (q, kind)
    op.close()
# partial-table calls on a node plan are refused (it merges internally)
op = GpuCombineOperator(parse("SELECT h, COUNT(*) FROM t GROUP BY h LIMIT 100"), segs, 100000)
op.run_raw(prepare_only=True)
part = _lib.Partial()
assert lib.phip_plan_execute_partial(op._plan, ctypes.byref(part)) == _lib.PHIP_ERR_INVALID
op.close()
# selection over several devices: UNSUPPORTED (the Java plan maker keeps its operator)
try:
    pm.make_instance_plan(parse("SELECT h, m FROM t LIMIT 10"), segs).next_block()
    raise SystemExit("selection over several devices accepted")
except _lib.PhipError as e:
    assert getattr(e, "code", _lib.PHIP_ERR_UNSUPPORTED) == _lib.PHIP_ERR_UNSUPPORTED, e
except Exception as e:  # (the plan maker may raise its UnsupportedOnGpu for the refusal)
    assert "Unsupported" in type(e).__name__, e
for s in segs:
    s.destroy()
print("HOSTSIM NODE OK")
