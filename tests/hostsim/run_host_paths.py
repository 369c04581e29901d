"""Drives every host-side path of libpinot_hip (runtime.cpp) against the HIP stand-in under ASan."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pinot_amd import _lib  # noqa: E402

_lib.LIB_PATH = sys.argv[1]
from pinot_amd.engine.plan import GpuInstancePlanMaker  # noqa: E402
from pinot_amd.engine.reduce import broker_response  # noqa: E402
from pinot_amd.engine.segment import GpuSegment  # noqa: E402
from pinot_amd.query.sql import parse  # noqa: E402
from pinot_amd.segment.creator import SegmentCreator  # noqa: E402
from pinot_amd.spi import DataType  # noqa: E402
from tests import fixtures  # noqa: E402

pm = GpuInstancePlanMaker()
segs = {n: GpuSegment(fixtures.segment_for(n)) for n in ("test_data_sv", "fast_filtered_count")}
for case in fixtures.expected()["queries"]:
    s = segs[case["data"]]
    broker_response(pm, case["query"], [s, s])
    qc = parse(case["query"])
    pm.make_instance_plan(qc, [s]).filter_bitmap()
for c in fixtures.expected()["docsets"]:
    g = GpuSegment(fixtures.docset_segment(c["sets"], c["num_docs"]))
    for p in ("s", "t"):
        q = parse("SELECT COUNT(*) FROM t WHERE " + fixtures.docset_filter(c["op"], len(c["sets"]), p))
        pm.make_instance_plan(q, [g]).filter_bitmap()
    g.destroy()
rng = np.random.default_rng(0)
raws = []
for k in range(3):
    n = 5000 + k
    c = SegmentCreator(f"s{k}", no_dictionary_columns=["r"], inverted_index_columns=["h"])
    c.add_column("g", DataType.STRING, np.array([f"k{x}" for x in rng.integers(k, 40 + k, n)]))
    c.add_column("h", DataType.INT, rng.integers(0, 7 + k, n))
    c.add_column("m", DataType.LONG, rng.integers(-10 ** 12, 10 ** 12, n))
    c.add_column("d", DataType.DOUBLE, rng.random(n))
    c.add_column("r", DataType.LONG, rng.integers(0, 100, n))
    raws.append(c.build())
gs = [GpuSegment(r) for r in raws]
for q in ("SELECT g, h, COUNT(*), SUM(m), SUM(d), MIN(d), MAX(m), DISTINCTCOUNTHLL(m) FROM t WHERE h <> 3 "
          "GROUP BY g, h LIMIT 100000",
          "SELECT SUM(r), AVG(d), DISTINCTCOUNTHLL(g) FROM t WHERE h IN (1, 2) OR m > 0",
          "SELECT COUNT(*) FROM t WHERE NOT (h = 1 AND (g = 'k3' OR d < 0.5))"):
    pm.make_instance_plan(parse(q), gs).next_block()
# the compacted group-by outputs come back in one copy (runtime.cpp contiguous_out): the stub's gather pattern must
# reach the result arrays unchanged (values i + 0.25, exact sums 1000 + i, registers 3 i + 1)
import ctypes  # noqa: E402
from pinot_amd.engine.plan import GpuCombineOperator as _GCO  # noqa: E402
for q in ("SELECT h, COUNT(*), SUM(m), MAX(d) FROM t GROUP BY h LIMIT 100000",
          "SELECT h, COUNT(*), SUM(m), DISTINCTCOUNTHLL(r) FROM t GROUP BY h LIMIT 100000"):
    op = _GCO(parse(q), gs, 100000)
    res = op.run_raw()
    r = res.contents
    ng, na = r.num_groups, r.num_aggregations
    assert ng >= 1 and na == 3, (ng, na)
    for i in range(ng * na):
        assert r.values[i] == 0.25 + i and r.long_values[i] == 1000 + i, (q, i, r.values[i], r.long_values[i])
    if r.num_hll:
        for i in range(ng * r.num_hll * 256):
            assert r.hll_registers[i] == (i * 3 + 1) & 0xFF, (q, i)
    _lib.load().phip_result_free(res)
    op.close()
# filtered aggregations: several filter programs in one plan (per-entry staging, interleaved inverted words,
# per-program statistics), and the descriptor checks of num_filter_programs / aggregation.program
pm.make_instance_plan(parse("SELECT COUNT(*), SUM(m) FILTER(WHERE h IN (1, 2)), MIN(d) FILTER(WHERE h = 4 AND "
                            "g <> 'k7'), DISTINCTCOUNTHLL(g) FILTER(WHERE m > 0) FROM t WHERE h <> 3"), gs).next_block()
from pinot_amd.engine.plan import GpuCombineOperator  # noqa: E402
from pinot_amd.query.context import FilterContext  # noqa: E402
base = parse("SELECT COUNT(*), SUM(m) FROM t")
flt = parse("SELECT COUNT(*) FROM t WHERE h = 1").filter
for progs, aprog in (([flt] * 9, [0, 8]), ([flt, None], [0, 2])):
    op = GpuCombineOperator(base, gs, 100_000, programs=(progs, aprog))
    try:
        op.next_block()
        raise SystemExit(f"descriptor accepted: {len(progs)} programs, {aprog}")
    except _lib.PhipError:
        pass
    op.close()
# FILTER + GROUP BY: the infos as programs of one group-by plan (own COUNT rows), with and without device trim
fgb = ("SELECT g, COUNT(*) FILTER(WHERE h = 1), SUM(m) FILTER(WHERE d < 0.5) s, MAX(d) FROM t WHERE h <> 3 "
       "GROUP BY g ORDER BY s DESC LIMIT 3")
pm.make_instance_plan(parse(fgb), gs).next_block()
GpuInstancePlanMaker(device_trim=False).make_instance_plan(parse(fgb), gs).next_block()
os.environ["PHIP_GB_HASH"] = "1"  # the hash-table group-by's host path (allocation, key decode)
pm.make_instance_plan(parse("SELECT g, h, COUNT(*), SUM(m), DISTINCTCOUNTHLL(m) FROM t GROUP BY g, h"), gs).next_block()
pm.make_instance_plan(parse(fgb), gs).next_block()
del os.environ["PHIP_GB_HASH"]
# raw STRING columns: var-byte chunk parsing at load (every codec; the stub decodes nothing), RAW_STRING leaves
# (the library's sorted, deduplicated set copy; range bounds), CASE statistics programs
rs = []
for k, codec in enumerate(("PASS_THROUGH", "SNAPPY", "ZSTANDARD", "GZIP")):
    c = SegmentCreator(f"rs{k}", no_dictionary_columns=["s"], raw_compression={"s": codec}, docs_per_chunk=97)
    c.add_column("s", DataType.STRING, np.array([["", "a", "ab", "\U0001F600", "\uffff", "b" * 30][x]
                                                for x in rng.integers(0, 6, 3001 + k)]))
    c.add_column("h", DataType.INT, rng.integers(0, 5, 3001 + k))
    rs.append(GpuSegment(c.build()))
in_list = ", ".join(f"'v{i}'" for i in range(3000)) + ", 'a', 'a', ''"
for q in (f"SELECT COUNT(*), SUM(h) FROM t WHERE s IN ({in_list})",
          "SELECT COUNT(*) FROM t WHERE s NOT IN ('a', 'ab') AND h > 1",
          "SELECT COUNT(*) FROM t WHERE s BETWEEN 'a' AND '\uffff' OR s < ''",
          "SELECT COUNT(*) FROM t WHERE s > 'a'",
          "SELECT SUM(CASE WHEN s = 'a' THEN h ELSE 0 END), COUNT(*) FROM t WHERE h <> 2"):
    pm.make_instance_plan(parse(q), rs).next_block()
from pinot_amd.engine.plan import _Leaf  # noqa: E402
op = GpuCombineOperator(parse("SELECT COUNT(*) FROM t WHERE s = 'a'"), rs[:1], 100_000)
op.trees = [_Leaf(_lib.LEAF_RAW_STRING_SET, "s", ids=np.array([2, 0, 5, 3], dtype=np.int32))]  # offsets past the end
try:
    op.next_block()
    raise SystemExit("malformed RAW_STRING_SET accepted")
except _lib.PhipError:
    pass
op.close()
# round 5: raw STRING keys / HLL / selection (device hashing and the host merge of representatives), tuple keys
# (forced on a small key space), the HLL-ordered trim, packed doc-order values
for q in ("SELECT s, h, COUNT(*) FROM t GROUP BY s, h LIMIT 1000",
          "SELECT h, DISTINCTCOUNTHLL(s), DISTINCTCOUNTHLL(s, 10) FROM t GROUP BY h LIMIT 100",
          "SELECT s, h FROM t WHERE h > 1 LIMIT 50"):
    pm.make_instance_plan(parse(q), rs).next_block()
os.environ["PHIP_TUPLE_KEYS"] = "1"
pm.make_instance_plan(parse("SELECT g, h, COUNT(*), SUM(m) FROM t GROUP BY g, h ORDER BY SUM(m) DESC LIMIT 5"),
                      gs).next_block()
pm.make_instance_plan(parse("SELECT g, h, r, COUNT(*) FROM t GROUP BY g, h, r ORDER BY g, h LIMIT 5"), gs).next_block()
del os.environ["PHIP_TUPLE_KEYS"]
hq = parse("SELECT g, DISTINCTCOUNTHLL(m), COUNT(*) FROM t GROUP BY g ORDER BY DISTINCTCOUNTHLL(m) DESC, g LIMIT 2")
hq.options["minServerGroupTrimSize"] = "3"
pm.make_instance_plan(hq, gs).next_block()
os.environ["PHIP_MATERIALIZE_MIN_DICT"] = "0"
pm.make_instance_plan(parse("SELECT SUM(m), MAX(h), SUM(r) FROM t WHERE d < 0.5"), gs).next_block()
del os.environ["PHIP_MATERIALIZE_MIN_DICT"]
for g in rs:
    g.destroy()
for g in gs:
    g.destroy()
for s in segs.values():
    s.destroy()
print("HOSTSIM OK")
