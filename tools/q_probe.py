"""Runs one BenchmarkQueries query (tools/bq.py) repeatedly on cuda:0, for a rocprofv3 kernel trace:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 tools/q_probe.py STARTREE_SUM_QUERY 20

Segments carry the reference table's star-tree (the STARTREE_* queries take it); the prepared plan is executed
through phip_plan_execute, so only the plan's own launches show up after the warm-up."""
import ctypes
import sys

sys.path.insert(0, ".")
from pinot_amd import _lib  # noqa: E402
from pinot_amd.engine.plan import GpuInstancePlanMaker  # noqa: E402
from pinot_amd.engine.segment import GpuSegment  # noqa: E402
from pinot_amd.query.sql import parse  # noqa: E402
from tools import bq  # noqa: E402


def main():
    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    segs = [GpuSegment(r) for r in bq.make_segments(10_000_000, 1, star_tree=True)]
    op = GpuInstancePlanMaker().make_instance_plan(parse(bq.QUERIES[name]), segs)
    run = op.inner if hasattr(op, "inner") and hasattr(op.inner, "run_raw") else op
    for i in range(reps):
        r = run.run_raw()
        c = r.contents
        print(f"{name} rep {i}: device {c.device_ms:.3f} ms, filter {c.filter_kernel_ms:.3f}, "
              f"agg {c.agg_kernel_ms:.3f}, groups {c.num_groups}", flush=True)
        _lib.load().phip_result_free(r)


if __name__ == "__main__":
    main()
