"""HBM traffic per bench step from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py.

MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half of a wide coalesced stream's bytes on gfx950
(128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE (KB) is taken as is. Only the query
kernels (filter_kernel / agg_kernel and their small reductions) are counted; segment-load kernels are not.

  python tools/traffic.py <fetch_dir> <write_dir> --steps K --warmup W --queries Q1.1,Q1.2,Q1.3 --sf 100 -o out.json
"""
import argparse
import csv
import glob
import json
import os

QUERY_KERNELS = ("filter_kernel", "agg_kernel", "finalize_partials", "slab_reduce", "group_", "roaring_or",
                 "masks_to_words", "fill_u64", "exclusive_scan")


def total_kb(d, counter):
    tot, n = 0.0, 0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                if not any(k in row["Kernel_Name"] for k in QUERY_KERNELS):
                    continue
                tot += float(row["Counter_Value"])
                n += 1
    return tot, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--queries", required=True)
    ap.add_argument("--sf", type=int, default=100)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    fkb, fn = total_kb(a.fetch_dir, "FETCH_SIZE")
    wkb, wn = total_kb(a.write_dir, "WRITE_SIZE")
    runs = a.steps + a.warmup  # every step runs each query once; warm-up steps are profiled too
    per_step = (2 * fkb + wkb) * 1024 / runs
    out = {"queries": a.queries.split(","), "sf": a.sf, "hbm_bytes_per_step": int(per_step),
           "fetch_bytes_per_step": int(2 * fkb * 1024 / runs), "write_bytes_per_step": int(wkb * 1024 / runs),
           "dispatch_rows": [fn, wn], "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE passes over "
                                                 "bench.py; query kernels only; (warmup+steps) runs"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
