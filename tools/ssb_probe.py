"""Runs SSB queries repeatedly on cuda:0 over SF100 segments (one layout), for rocprofv3 kernel traces and PMC passes:

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES ... -- python3 tools/ssb_probe.py --queries Q1.1 --layout sorted --reps 20

The plans are prepared once; only their executions run after the segments load."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", default="Q1.1")
    ap.add_argument("--layout", default="sorted")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sf", type=int, default=100)
    args = ap.parse_args()
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    queries = args.queries.split(",")
    cols = ssb.columns_for(queries)
    nseg = (args.sf * ssb.ROWS_PER_SF) // ssb.SEGMENT_ROWS
    gsegs = []
    for i in range(0, nseg, 10):
        for r in ssb.make_segments(args.sf, cols, seed=42, segments=range(i, min(nseg, i + 10)), layout=args.layout):
            gsegs.append(GpuSegment(r))
            for ci in r.columns.values():
                if not ci.metadata.is_sorted:
                    ci.forward = b""
    ops = {q: GpuInstancePlanMaker().make_instance_plan(parse(ssb.SSB_QUERIES[q]), gsegs) for q in queries}
    for q in queries:
        ms = []
        for _ in range(args.reps):
            blk = ops[q].next_block()
            ms.append((blk.filter_kernel_ms, blk.agg_kernel_ms))
        f = sum(m[0] for m in ms) / len(ms)
        a = sum(m[1] for m in ms) / len(ms)
        print(f"{q}: filter {f:.4f} ms, agg {a:.4f} ms (HIP events, mean of {len(ms)})", flush=True)
    for op in ops.values():
        op.close()
    for g in gsegs:
        g.destroy()


if __name__ == "__main__":
    main()
