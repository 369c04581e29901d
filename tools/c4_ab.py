"""A/B of library settings on config C4 inside ONE process (the C4 segments are built and loaded once; the
settings are environment variables the library reads when a plan is prepared). Per setting and selectivity:
p50 latency and mean filter-kernel time (HIP events).

  python tools/c4_ab.py "PHIP_CONTIG=0" "PHIP_CONTIG=1" "PHIP_CONTIG=1 PHIP_FILTER_BPC=2" ...
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import ctypes

    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import c4
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    sels = [float(x) for x in os.environ.get("C4_SELS", "0.0001,0.01,0.5").split(",")]
    aggs = os.environ.get("C4_AGGS", "COUNT(*)").split(";")
    distinct = [c4.make_segment(i) for i in range(4)]
    gsegs = [GpuSegment(r) for _ in range(25) for r in distinct]
    print(f"loaded {len(gsegs)} segments", flush=True)
    base = dict(os.environ)
    for cfg in sys.argv[1:]:
        os.environ.clear()
        os.environ.update(base)
        for kv in cfg.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        for agg in aggs:
            for sel in sels:
                op = GpuInstancePlanMaker().make_instance_plan(parse(c4.query(sel, agg)), gsegs)
                for _ in range(3):
                    op.next_block()
                lat, fk = [], []
                for _ in range(10):
                    t0 = time.perf_counter()
                    b = op.next_block()
                    lat.append((time.perf_counter() - t0) * 1e3)
                    fk.append(b.filter_kernel_ms)
                op.close()
                print(f"{cfg:45s} {agg:9s} sel={sel:<7} p50 {np.median(lat):.3f} ms  filter {np.mean(fk):.3f} ms "
                      f"docs {b.stats.num_docs_scanned}", flush=True)
    for g in gsegs:
        g.destroy()


if __name__ == "__main__":
    main()
