"""Filter-kernel variants on the unsorted SSB SF100 layout (measurement tool): per variant the median filter-kernel
time of Q1.x's filter as a SUM query (tile masks written for the aggregation kernel) and as COUNT(*) (no masks),
with the library's measurement switches set per plan (PHIP_FILTER_PROBE = stream only, PHIP_FILTER_BPC = workgroups
per CU, PHIP_MASK_NT = non-temporal mask stores).

    python tools/filter_explore.py [--segs 100] [--reps 20]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=100)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="base;PHIP_FILTER_PROBE=1;PHIP_FILTER_BPC=4;PHIP_FILTER_BPC=3;"
                                          "PHIP_MASK_NT=1;PHIP_FILTER_PROBE=1,PHIP_FILTER_BPC=4")
    args = ap.parse_args()
    import torch  # noqa: F401  (same import order as bench.py)
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    lib = _lib.load()
    _lib.check(lib.phip_init((ctypes.c_int32 * 1)(0), 1))
    qs = ["Q1.1", "Q1.2", "Q1.3"]
    cols = ssb.columns_for(qs)
    segs = []
    for i in range(0, args.segs, 10):
        for r in ssb.make_segments(100, cols, segments=list(range(i, min(i + 10, args.segs))), layout="unsorted"):
            segs.append(GpuSegment(r))
    sqls = {}
    for q in qs:
        sqls[q + " sum"] = ssb.SSB_QUERIES[q]
        sqls[q + " count"] = "select count(*) from lineorder where " + ssb.SSB_QUERIES[q].split(" where ", 1)[1]
    for var in args.variants.split(";"):
        env = {} if var == "base" else dict(kv.split("=") for kv in var.split(","))
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        out = []
        for name, sql in sqls.items():
            op = GpuInstancePlanMaker().make_instance_plan(parse(sql), segs)
            ts = []
            for _ in range(args.reps + 3):
                res = op.run_raw()
                ts.append(res.contents.filter_kernel_ms)
                lib.phip_result_free(res)
            op.close()
            out.append(f"{name} {np.median(ts[3:]):.4f}")
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        print(f"{var:40s} " + "  ".join(out), flush=True)
    for s in segs:
        s.destroy()


if __name__ == "__main__":
    main()
