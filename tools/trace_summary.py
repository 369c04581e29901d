"""Per-query kernel averages from a rocprofv3 --kernel-trace CSV, and the roofline fraction recomputed from them.

The bench's `roofline.frac` = mean algorithmic bytes per launch / mean launch time (HIP events on the library's
stream). This script recomputes it from the profiler's own dispatch timestamps, so the tracked profile reproduces
the number without trusting the bench's events:

  # headline: bench.py --no-concurrent run; each execution of Q1.1, Q1.2, Q1.3 launches exactly one kernel of the
  # family, so the family's dispatches cycle through the queries in order
  python tools/trace_summary.py cycle run_kernel_trace.csv --queries Q1.1,Q1.2,Q1.3 --family fused_filter_agg \
      --bench bench_line.json --layout sorted -o profiles/r06_trace_sorted.json

  # group-by queries: tools/gb_ab.py --gap 0.25 run (the GPU idles before each query's executions); the trace is
  # cut at idle gaps and the i-th cluster of query kernels belongs to the i-th query gb_ab printed
  python tools/trace_summary.py gaps run_kernel_trace.csv --gb-ab gb_ab.log -o profiles/r06_trace_gb.json

Families: filter_kernel (plain filter launch), fused_filter_agg (filter_kernel<C, NA != 0>: a filter launch that
aggregated its own tiles), agg_kernel (separate aggregation launch); tools/traffic.py names them the same way.
"""
import argparse
import csv
import json
import re

HBM_PEAK_GBS = 8000.0


def family(name):
    m = re.search(r"phip::filter_kernel<(\w+), (-?\d+)>", name)
    if m:
        return "fused_filter_agg" if int(m.group(2)) != 0 else "filter_kernel"
    if "phip::agg_kernel<" in name:
        return "agg_kernel"
    return None


def read_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def _stats(durs_ns):
    if not durs_ns:
        return None
    return {"dispatches": len(durs_ns), "mean_us": round(sum(durs_ns) / len(durs_ns) / 1e3, 3),
            "min_us": round(min(durs_ns) / 1e3, 3), "max_us": round(max(durs_ns) / 1e3, 3)}


def cycle(a):
    rows = [r for r in read_trace(a.trace) if family(r[2]) == a.family]
    qs = a.queries.split(",")
    if len(rows) % len(qs):
        raise SystemExit(f"{len(rows)} {a.family} dispatches do not cycle through {len(qs)} queries")
    per = {q: [] for q in qs}
    for i, (s, e, _) in enumerate(rows):
        per[qs[i % len(qs)]].append(e - s)
    out = {"trace": a.trace, "family": a.family, "method": "dispatch i belongs to query i mod len(queries)",
           "per_query": {q: _stats(v) for q, v in per.items()}}
    alld = [d for v in per.values() for d in v]
    out["all"] = _stats(alld)
    if a.bench:
        line = [l for l in open(a.bench) if l.lstrip().startswith("{")][-1]
        j = json.loads(line)
        # (a run with --layout unsorted reports the unsorted layout at the top level)
        rf = j["unsorted_layout"]["roofline"] if a.layout == "unsorted" and "unsorted_layout" in j else j["roofline"]
        k = rf["kernels"][a.family]
        mean_s = sum(alld) / len(alld) * 1e-9
        ach = k["alg_bytes_per_launch"] / mean_s / 1e9
        out["recomputed"] = {"alg_bytes_per_launch": k["alg_bytes_per_launch"],
                             "trace_mean_launch_ms": round(mean_s * 1e3, 5), "achieved_GBps": round(ach, 1),
                             "frac": round(ach / HBM_PEAK_GBS, 4),
                             "bench_ms_per_launch": k["ms_per_launch"], "bench_frac": k["frac"],
                             "frac_ratio_trace_over_bench": round(ach / HBM_PEAK_GBS / k["frac"], 4) if k["frac"] else None}
    return out


def gaps(a):
    rows = read_trace(a.trace)
    logs = [json.loads(l) for l in open(a.gb_ab) if l.lstrip().startswith("{") and '"query"' in l]
    # clusters of query kernels separated by >= gap_ms of idle GPU
    clusters, cur, last_end = [], [], None
    for s, e, n in rows:
        if last_end is not None and s - last_end >= a.gap_ms * 1e6:
            clusters.append(cur)
            cur = []
        cur.append((s, e, n))
        last_end = max(e, last_end or e)
    clusters.append(cur)
    clusters = [c for c in clusters if any(family(n) for _, _, n in c)]
    if len(clusters) != len(logs):
        raise SystemExit(f"{len(clusters)} clusters of query kernels vs {len(logs)} gb_ab lines")
    out = {"trace": a.trace, "method": f"clusters split at >= {a.gap_ms} ms of idle GPU, in gb_ab.py's order",
           "per_query": {}}
    for c, j in zip(clusters, logs):
        fam = {}
        for s, e, n in c:
            f = family(n)
            if f:
                fam.setdefault(f, []).append(e - s)
        d = {f: _stats(v) for f, v in fam.items()}
        for f, v in fam.items():
            b = j.get("agg_bytes") if f == "agg_kernel" else j.get("filter_bytes")
            if b:
                ach = b / (sum(v) / len(v) * 1e-9) / 1e9
                d[f]["alg_bytes"] = b
                d[f]["frac"] = round(ach / HBM_PEAK_GBS, 4)
        d["hip_events_ms"] = {"filter": j.get("filter_ms"), "agg": j.get("agg_ms")}
        d["set"] = j.get("set")
        out["per_query"][j["query"] + (f" [{j['set']}]" if j.get("set") else "")] = d
    return out


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="mode", required=True)
    c = sub.add_parser("cycle")
    c.add_argument("trace")
    c.add_argument("--queries", required=True)
    c.add_argument("--family", default="fused_filter_agg")
    c.add_argument("--bench")
    c.add_argument("--layout", default=None, choices=[None, "sorted", "unsorted"])
    c.add_argument("-o", "--out")
    g = sub.add_parser("gaps")
    g.add_argument("trace")
    g.add_argument("--gb-ab", required=True)
    g.add_argument("--gap-ms", type=float, default=100.0)
    g.add_argument("-o", "--out")
    a = ap.parse_args()
    out = cycle(a) if a.mode == "cycle" else gaps(a)
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
