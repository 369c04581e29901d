"""Timeline probe of one group-by query (C1 GROUP_BY_LOW_CARD): run under rocprofv3 --kernel-trace to see the
device work between the aggregation kernel and the result copy."""
import ctypes
import sys
import time

sys.path.insert(0, ".")
from pinot_amd import _lib  # noqa: E402
from pinot_amd.engine.plan import GpuInstancePlanMaker  # noqa: E402
from pinot_amd.engine.segment import GpuSegment  # noqa: E402
from pinot_amd.query.sql import parse  # noqa: E402
from tools import bq  # noqa: E402

_lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
segs = [GpuSegment(r) for r in bq.make_segments(10_000_000, 1)]
op = GpuInstancePlanMaker().make_instance_plan(parse(bq.QUERIES[sys.argv[1] if len(sys.argv) > 1 else "GROUP_BY_LOW_CARD"]), segs)
for i in range(8):
    t0 = time.perf_counter()
    r = op.run_raw()
    t1 = time.perf_counter()
    c = r.contents
    print(f"wall {1e3 * (t1 - t0):.3f} ms device {c.device_ms:.3f} filter {c.filter_kernel_ms:.3f} agg {c.agg_kernel_ms:.3f} groups {c.num_groups}")
    _lib.load().phip_result_free(r)
