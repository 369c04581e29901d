import ctypes, sys, time
sys.path.insert(0, '.')
from pinot_amd import _lib
from pinot_amd.engine.plan import GpuInstancePlanMaker
from pinot_amd.engine.segment import GpuSegment
from pinot_amd.query.sql import parse
from tools import bq
_lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
raws = bq.make_segments(10_000_000, 1)
segs = [GpuSegment(r) for r in raws]
qc = parse(bq.QUERIES["STARTREE_FILTER_QUERY"])
op = GpuInstancePlanMaker(num_groups_limit=10 ** 9).make_instance_plan(qc, segs)
for i in range(5):
    r = op.run_raw(); c = r.contents; print(c.device_ms, c.filter_kernel_ms, c.agg_kernel_ms, c.num_groups); _lib.load().phip_result_free(r)
