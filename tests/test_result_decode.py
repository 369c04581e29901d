"""The aggregation-only fast decode of phip_result (plan.GpuCombineOperator._aggregation_block over one
_lib.RESULT_IMAGE read) against the values the library laid out, on a host-built result (no GPU): exact int64 sums
and counts, double sums / MIN / MAX, AVG and MINMAXRANGE pairs, statistics and kernel fields; HLL and group-by
results fall back to the general path (None)."""
import ctypes
from types import SimpleNamespace

from pinot_amd import _lib
from pinot_amd.engine.plan import GpuCombineOperator, plan_aggregations
from pinot_amd.query.sql import parse


def _result(vals, longs, exact, nhll=0, ngroups=1):
    r = _lib.Result()
    n = len(vals)
    keep = [(ctypes.c_double * n)(*vals), (ctypes.c_int64 * n)(*longs), (ctypes.c_int32 * n)(*exact)]
    r.num_docs_scanned, r.num_entries_scanned_in_filter, r.num_entries_scanned_post_filter = 11, 22, 33
    r.num_total_docs, r.num_segments_processed, r.num_segments_matched = 44, 5, 4
    r.num_aggregations, r.num_groups, r.num_hll = n, ngroups, nhll
    r.values = ctypes.cast(keep[0], ctypes.POINTER(ctypes.c_double))
    r.long_values = ctypes.cast(keep[1], ctypes.POINTER(ctypes.c_int64))
    r.long_exact = ctypes.cast(keep[2], ctypes.POINTER(ctypes.c_int32))
    r.filter_kernel_ms, r.agg_kernel_ms, r.device_ms, r.scan_kernel_ms = 0.25, 0.5, 0.75, 0.125
    r.filter_bytes, r.agg_bytes, r.stream_bytes, r.fused = 1000, 2000, 900, 1
    return r, keep


def test_aggregation_fast_decode():
    qc = parse("SELECT COUNT(*), SUM(a), SUM(b), MIN(b), AVG(a), MINMAXRANGE(b) FROM t")
    prims, mapping = plan_aggregations(qc.aggregations)
    # prims: COUNT, SUM(a), SUM(b), MIN(b), MAX(b) (AVG / MINMAXRANGE share the SUM / COUNT / MIN slots)
    kinds = [p[0] for p in prims]
    vals = [0.0] * len(prims)
    longs = [0] * len(prims)
    exact = [0] * len(prims)
    for i, (k, col) in enumerate((p[0], p[2]) for p in prims):
        if k == _lib.AGG_COUNT:
            longs[i] = 1234
        elif k == _lib.AGG_SUM and col == "a":
            longs[i], exact[i], vals[i] = 2 ** 60 + 7, 1, float(2 ** 60 + 7)
        elif k == _lib.AGG_SUM:
            vals[i] = 12.5
        elif k == _lib.AGG_MIN:
            vals[i] = -3.0
        else:
            vals[i] = 9.0
    r, keep = _result(vals, longs, exact)
    op = SimpleNamespace(prims=prims, mapping=mapping, query=qc)
    blk = GpuCombineOperator._aggregation_block(op, ctypes.pointer(r))
    assert blk.results == [1234, 2 ** 60 + 7, 12.5, -3.0, (2 ** 60 + 7, 1234), (-3.0, 9.0)]
    assert isinstance(blk.results[1], int) and isinstance(blk.results[2], float)
    s = blk.stats
    assert (s.num_docs_scanned, s.num_entries_scanned_in_filter, s.num_entries_scanned_post_filter, s.num_total_docs,
            s.num_segments_processed, s.num_segments_matched) == (11, 22, 33, 44, 5, 4)
    assert (blk.filter_kernel_ms, blk.agg_kernel_ms, blk.device_ms, blk.scan_kernel_ms) == (0.25, 0.5, 0.75, 0.125)
    assert (blk.filter_bytes, blk.agg_bytes, blk.stream_bytes, blk.fused) == (1000, 2000, 900, True)
    assert _lib.AGG_HLL not in kinds


def test_fast_decode_leaves_hll_and_groups_to_the_general_path():
    qc = parse("SELECT COUNT(*) FROM t")
    prims, mapping = plan_aggregations(qc.aggregations)
    op = SimpleNamespace(prims=prims, mapping=mapping, query=qc)
    r, keep = _result([0.0], [5], [0], nhll=1)
    assert GpuCombineOperator._aggregation_block(op, ctypes.pointer(r)) is None
    r, keep = _result([0.0], [5], [0], ngroups=3)
    assert GpuCombineOperator._aggregation_block(op, ctypes.pointer(r)) is None


def test_dictionary_lookup_strings_and_numbers():
    """Group keys' values from a result dictionary (plan._dictionary_lookup): NUL-padded fixed-width strings come
    back without the padding (interior bytes kept), numbers as Python scalars, repeated and empty id lists."""
    from pinot_amd.engine.plan import _dictionary_lookup
    from pinot_amd.spi import DataType
    words = ["", "a", "MFGR#1221", "héllo", "x y"]
    w = max(len(s.encode()) for s in words)
    blob = (ctypes.c_uint8 * (len(words) * w))(*b"".join(s.encode().ljust(w, b"\0") for s in words))
    dv = _lib.DictionaryView(int(DataType.STRING), len(words), w, 0, ctypes.addressof(blob))
    ids = [4, 0, 2, 2, 3, 1]
    assert _dictionary_lookup(dv, ids) == [words[i] for i in ids]
    assert _dictionary_lookup(dv, []) == []
    nums = (ctypes.c_int64 * 4)(-5, 2 ** 40, 0, 7)
    dv = _lib.DictionaryView(int(DataType.LONG), 4, 0, 0, ctypes.addressof(nums))
    got = _dictionary_lookup(dv, [1, 3, 0])
    assert got == [2 ** 40, 7, -5] and all(type(v) is int for v in got)
    dbl = (ctypes.c_double * 2)(1.5, -0.25)
    dv = _lib.DictionaryView(int(DataType.DOUBLE), 2, 0, 0, ctypes.addressof(dbl))
    assert _dictionary_lookup(dv, [1, 0]) == [-0.25, 1.5]


def test_columnar_block_real_keys_by_bits():
    """The {key: intermediates} view of a columnar group-by block keeps raw DOUBLE keys -0.0 and 0.0 as two groups
    (the device keys reals by their bits, as the reference's Double2IntOpenHashMap does) and NaN as one; a plain
    dict over Python floats would merge -0.0 into 0.0 and overwrite that group's values."""
    import numpy as np

    from pinot_amd.engine.results import GroupByResultsBlock, JavaDoubleKey
    qc = parse("SELECT z, COUNT(*) FROM t GROUP BY z")
    blk = GroupByResultsBlock(qc.aggregations, list(qc.group_by), None)
    blk.key_types = ["DOUBLE"]
    keys = np.array([0.0, -0.0, 1.5, np.nan], dtype=np.float64)
    blk.set_columns([keys], [np.array([3, 5, 7, 11], np.int64)], [("count", 0)])
    g = blk.groups
    assert len(g) == 4
    assert g[(0.0,)] == [3] and g[(JavaDoubleKey(-0.0),)] == [5] and g[(1.5,)] == [7]
    assert g[(JavaDoubleKey(float("nan")),)] == [11]
    # object key columns (null keys beside reals) wrap the same way
    blk2 = GroupByResultsBlock(qc.aggregations, list(qc.group_by), None)
    blk2.key_types = ["DOUBLE"]
    blk2.set_columns([np.array([-0.0, None, 0.0], dtype=object)], [np.array([1, 2, 3], np.int64)], [("count", 0)])
    assert len(blk2.groups) == 3 and blk2.groups[(JavaDoubleKey(-0.0),)] == [1] and blk2.groups[(None,)] == [2]


def test_oracle_real_keys_by_bits():
    """The oracle keys raw DOUBLE group values by their bits too: -0.0 and 0.0 two groups with their own counts."""
    import numpy as np

    from oracle import executor
    from pinot_amd.segment.creator import SegmentCreator
    from pinot_amd.spi import DataType
    c = SegmentCreator("z", no_dictionary_columns=["z"])
    c.add_column("z", DataType.DOUBLE, np.array([-0.0, 0.0, 0.0, -0.0, -0.0, 2.5]))
    blk, _ = executor.execute(parse("SELECT z, COUNT(*) FROM t GROUP BY z"), [c.build()])
    got = {(float(k[0]), bool(np.signbit(k[0]))): v[0] for k, v in blk.groups.items()}
    assert got == {(0.0, True): 3, (0.0, False): 2, (2.5, False): 1}
