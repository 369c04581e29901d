"""HBM traffic per launch of the query kernels from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py.

MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half of a wide coalesced stream's bytes on gfx950
(128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE (KB) is taken as is; the two counters need
separate passes (TCC slots). Per kernel (filter_kernel, agg_kernel): bytes per launch = 2 x sum(FETCH_SIZE) /
fetch-pass dispatches + sum(WRITE_SIZE) / write-pass dispatches. One pair of passes per bench layout.

  python tools/traffic.py --layout sorted <fetch_dir> <write_dir> [--layout unsorted <fetch_dir> <write_dir>]
         --queries Q1.1,Q1.2,Q1.3 --sf 100 -o profiles/r02_traffic.json
"""
import argparse
import csv
import glob
import json
import os

KERNELS = ("filter_kernel", "agg_kernel")


def per_kernel(d, counter):
    tot, n = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                for k in KERNELS:
                    if f"phip::{k}<" in row["Kernel_Name"]:
                        tot[k] = tot.get(k, 0.0) + float(row["Counter_Value"]) * 1024
                        n[k] = n.get(k, 0) + 1
    return tot, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", nargs=3, action="append", metavar=("NAME", "FETCH_DIR", "WRITE_DIR"), required=True)
    ap.add_argument("--queries", required=True)
    ap.add_argument("--sf", type=int, default=100)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    out = {"queries": a.queries.split(","), "sf": a.sf, "per_launch": {}, "dispatches": {},
           "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE passes (separate runs) over "
                     "bench.py --layout <name>; HBM bytes per launch per kernel"}
    for name, fdir, wdir in a.layout:
        ft, fn = per_kernel(fdir, "FETCH_SIZE")
        wt, wn = per_kernel(wdir, "WRITE_SIZE")
        out["per_launch"][name] = {k: int(2 * ft[k] / fn[k] + (wt.get(k, 0.0) / wn[k] if wn.get(k) else 0.0))
                                   for k in ft if fn.get(k)}
        out["dispatches"][name] = {"fetch": fn, "write": wn}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
