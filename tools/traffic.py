"""HBM traffic per launch of the query kernels from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py.

MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half of a wide coalesced stream's bytes on gfx950
(128-B requests tallied at 64 B), so for a streaming kernel it is doubled; other access shapes are uncalibrated,
so both figures are kept (raw and x2) and bench.py uses x2 only for the streaming filter kernel. WRITE_SIZE (KB)
is taken as is; the two counters need separate passes (TCC slots). Per kernel family (filter_kernel,
fused_filter_agg, agg_kernel): bytes per launch = sum over dispatches / dispatches. One pair of passes per layout.

  python tools/traffic.py --layout sorted <fetch_dir> <write_dir> [--layout unsorted <fetch_dir> <write_dir>]
         --queries Q1.1,Q1.2,Q1.3 --sf 100 -o profiles/r02_traffic.json
"""
import argparse
import csv
import glob
import json
import os

import re


def family(kernel_name):
    """filter_kernel (plain filter launch), fused_filter_agg (filter_kernel<C, NA> with NA > 0: it aggregated its
    own tiles) or agg_kernel; None for the small kernels."""
    m = re.search(r"phip::filter_kernel<(\w+), (\d+)>", kernel_name)
    if m:
        return "fused_filter_agg" if int(m.group(2)) > 0 else "filter_kernel"
    if "phip::agg_kernel<" in kernel_name:
        return "agg_kernel"
    return None


def per_kernel(d, counter):
    tot, n = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                k = family(row["Kernel_Name"])
                if k is None:
                    continue
                tot[k] = tot.get(k, 0.0) + float(row["Counter_Value"]) * 1024
                n[k] = n.get(k, 0) + 1
    return tot, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", nargs=3, action="append", metavar=("NAME", "FETCH_DIR", "WRITE_DIR"), required=True)
    ap.add_argument("--calib", nargs=2, metavar=("FETCH_DIR", "BENCH_LOG"),
                    help="FETCH_SIZE pass over a stream-only probe run of bench.py (PHIP_FILTER_PROBE=1 PHIP_FUSE=0) and "
                         "that run's JSON line: stream_factor = the filter kernel's streamed bytes / its FETCH_SIZE")
    ap.add_argument("--queries", required=True)
    ap.add_argument("--sf", type=int, default=100)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    out = {"queries": a.queries.split(","), "sf": a.sf, "per_launch": {}, "dispatches": {},
           "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes (separate runs) over bench.py --layout "
                     "<name>; HBM bytes per launch per kernel family: raw = FETCH + WRITE, x2 = 2 x FETCH + "
                     "WRITE (the gfx950 correction for wide coalesced streams)"}
    for name, fdir, wdir in a.layout:
        ft, fn = per_kernel(fdir, "FETCH_SIZE")
        wt, wn = per_kernel(wdir, "WRITE_SIZE")
        pl = {}
        for k in ft:
            if not fn.get(k):
                continue
            f = ft[k] / fn[k]
            w = wt.get(k, 0.0) / wn[k] if wn.get(k) else 0.0
            pl[k] = {"fetch_raw": int(f), "write": int(w), "raw": int(f + w), "x2": int(2 * f + w)}
        out["per_launch"][name] = pl
        out["dispatches"][name] = {"fetch": fn, "write": wn}
    if a.calib:
        ft, fn = per_kernel(a.calib[0], "FETCH_SIZE")
        line = [l for l in open(a.calib[1]) if l.startswith("{")][-1]
        j = json.loads(line)
        ks = (j.get("roofline") or {}).get("kernels", {})
        if "filter_kernel" not in ks or not fn.get("filter_kernel"):
            raise SystemExit("calibration run has no plain filter_kernel launches")
        stream = ks["filter_kernel"]["stream_bytes_per_launch"]
        fetch = ft["filter_kernel"] / fn["filter_kernel"]
        out["stream_factor"] = round(stream / fetch, 4)
        out["calibration"] = {"run": "bench.py PHIP_FILTER_PROBE=1 PHIP_FUSE=0 (stream-only filter launches: the "
                                     "staged tiles' bytes are known exactly)",
                              "stream_bytes_per_launch": int(stream), "fetch_size_per_launch": int(fetch),
                              "layout": j.get("config", {}).get("layout")}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
