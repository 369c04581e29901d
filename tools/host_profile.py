"""Where the host time of an aggregation-only execution goes (measurement tool): the sorted headline's Q1.2 / Q1.3
executed N times under cProfile after a warm-up, the top functions by cumulative and own time."""
import cProfile
import ctypes
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    os.environ.setdefault("PHIP_KERNEL_TIMING", "0")
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    qs = ["Q1.2", "Q1.3"]
    cols = ssb.columns_for(qs)
    segs = []
    for i in range(0, 100, 10):
        for r in ssb.make_segments(100, cols, seed=42, segments=range(i, i + 10), layout="sorted"):
            segs.append(GpuSegment(r))
    ops = [GpuInstancePlanMaker().make_instance_plan(parse(ssb.SSB_QUERIES[q]), segs) for q in qs]
    for _ in range(50):
        for op in ops:
            op.next_block()
    n = 400
    t0 = time.perf_counter()
    for _ in range(n):
        for op in ops:
            op.next_block()
    wall = (time.perf_counter() - t0) / (n * len(ops)) * 1e6
    print(f"mean wall per execution: {wall:.1f} us", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        for op in ops:
            op.next_block()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
