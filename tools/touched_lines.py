"""The byte floor of bench.py's gathers at the memory system's access granularity: for every query of the headline
step and every segment, the 64-B lines of the projected columns' fixed-bit forward indexes that hold at least one
matched doc's id, plus the dictionary lines the matched ids select. A gather moves whole lines, so these bytes must
cross HBM / L2 whatever the kernel -- the `touched` floor bench.py prints next to the algorithmic bytes (which
price a matched doc at b/8 bytes). Matched docs come from the library's own filter (phip_filter_bitmap per
segment); outside any timed region.

    python tools/touched_lines.py --layout sorted --layout unsorted -o profiles/r04_touched.json
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LINE_BITS = 512  # 64-B lines


def lines_of(docs, bits):
    """Distinct 64-B lines holding bits [d*b, d*b + b) of the matched docs d (a value may straddle two lines)."""
    if len(docs) == 0:
        return 0
    first = (docs.astype(np.int64) * bits) >> 9
    last = (docs.astype(np.int64) * bits + bits - 1) >> 9
    return int(len(np.union1d(first, last)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", action="append", default=None)
    ap.add_argument("--queries", default="Q1.1,Q1.2,Q1.3")
    ap.add_argument("--segs", type=int, default=100)
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--materialize-min", type=int, default=1 << 20,
                    help="dictionary bytes from which a value-only column reads doc-order values (-1: never)")
    args = ap.parse_args()
    from pinot_amd import _lib
    from pinot_amd.engine.plan import GpuCombineOperator, plan_aggregations
    from pinot_amd.engine.segment import GpuSegment
    from pinot_amd.query.sql import parse
    from tools import ssb
    _lib.check(_lib.load().phip_init((ctypes.c_int32 * 1)(0), 1))
    queries = args.queries.split(",")
    cols = ssb.columns_for(queries)
    out = {"queries": queries, "sf": 100, "line_bytes": 64, "per_query": {}, "materialize_min": args.materialize_min,
           "method": "per segment: distinct 64-B lines of each projected column's fixed-bit words holding a matched "
                     "doc's id bits, + distinct 64-B dictionary lines of the matched ids (phip_filter_bitmap docs); "
                     "a value-only column with a dictionary of >= materialize_min bytes: the fewer of those and the "
                     "lines of its doc-order values"}
    for layout in args.layout or ["sorted"]:
        res = {q: {"id_line_bytes": 0, "dict_line_bytes": 0, "matched": 0} for q in queries}
        for i in range(0, args.segs, 10):
            for raw in ssb.make_segments(100, cols, seed=42, segments=list(range(i, min(i + 10, args.segs))),
                                         layout=layout):
                g = GpuSegment(raw)
                for q in queries:
                    qc = parse(ssb.SSB_QUERIES[q])
                    op = GpuCombineOperator(qc, [g], 100_000)
                    words = op.filter_bitmap()
                    op.close()
                    docs = np.nonzero(np.unpackbits(words.view(np.uint8), bitorder="little")[:raw.num_docs])[0]
                    res[q]["matched"] += int(len(docs))
                    prims, _ = plan_aggregations(qc.aggregations)
                    seen = set()
                    for p in prims:
                        for c in (p[2], p[3]):
                            if c is None or c in seen:
                                continue
                            seen.add(c)
                            m = raw.columns[c].metadata
                            if not m.has_dictionary:
                                res[q]["id_line_bytes"] += 8 * len(docs)
                                continue
                            w = 4 if int(m.data_type) in (0, 2) else 8
                            b = m.bits_per_element
                            ids = np.frombuffer(raw.columns[c].forward, dtype=np.uint8)
                            # the matched docs' dict ids (MSB-first fixed-bit stream)
                            bitpos = docs.astype(np.int64) * b
                            vals = np.zeros(len(docs), dtype=np.int64)
                            padded = np.concatenate([ids, np.zeros(8, np.uint8)])
                            for k in range(b):
                                pos = bitpos + k
                                bit = (padded[pos >> 3] >> (7 - (pos & 7))) & 1
                                vals = (vals << 1) | bit
                            via_ids = 64 * lines_of(docs, b) + 64 * int(len(np.unique((vals * w) >> 6)))
                            where = ssb.SSB_QUERIES[q].upper().split("WHERE", 1)[-1].split("GROUP BY")[0]
                            if (args.materialize_min >= 0 and m.cardinality * w >= args.materialize_min
                                    and c.upper() not in where):
                                # a value-only column with a large dictionary also has doc-order values (runtime.cpp
                                # ensure_vals), INT / LONG ones bit-packed at their range's width (packed_value_bits):
                                # the floor is the cheaper of the two routes
                                vb = 8 * w
                                if int(m.data_type) in (0, 1):
                                    dv = np.frombuffer(raw.columns[c].dictionary, dtype=">i4" if w == 4 else ">i8")
                                    rb = max(1, int(dv[-1]) - int(dv[0])).bit_length()
                                    vb = rb if rb <= 32 and rb < 8 * w else vb
                                via_vals = 64 * lines_of(docs, vb)
                                res[q]["value_line_bytes"] = res[q].get("value_line_bytes", 0) + via_vals
                                res[q]["ids_dict_line_bytes"] = res[q].get("ids_dict_line_bytes", 0) + via_ids
                                res[q]["id_line_bytes"] += min(via_vals, via_ids)
                                continue
                            res[q]["id_line_bytes"] += 64 * lines_of(docs, b)
                            res[q]["dict_line_bytes"] += via_ids - 64 * lines_of(docs, b)
                g.destroy()
        for q in queries:
            res[q]["touched_bytes"] = res[q]["id_line_bytes"] + res[q]["dict_line_bytes"]
        out["per_query"][layout] = res
        print(json.dumps({layout: res}), flush=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
