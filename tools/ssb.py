"""Python front end of tools/ssbgen.c: synthetic SSB flattened-lineorder segments + the SSB queries.

Query text follows pinot-integration-tests/src/test/resources/ssb/ssb_query_set.yaml:22-98 with the
star joins flattened away (dimension attributes are lineorder columns), which is the
"SSB flattened" configuration BASELINE.json names.
"""
import ctypes
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from pinot_amd.segment.creator import ColumnIndexes, ColumnMetadata, ImmutableSegment
from pinot_amd.spi import DataType

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libssbgen.so")
ROWS_PER_SF = 6_000_000
SEGMENT_ROWS = 6_000_000

SSB_QUERIES = {
    "Q1.1": "select sum(CAST(LO_EXTENDEDPRICE AS DOUBLE) * LO_DISCOUNT) as revenue from lineorder "
            "where D_YEAR = 1993 and LO_DISCOUNT between 1 and 3 and LO_QUANTITY < 25",
    "Q1.2": "select sum(CAST(LO_EXTENDEDPRICE AS DOUBLE) * LO_DISCOUNT) as revenue from lineorder "
            "where D_YEARMONTHNUM = 199401 and LO_DISCOUNT between 4 and 6 and LO_QUANTITY between 26 and 35",
    "Q1.3": "select sum(CAST(LO_EXTENDEDPRICE AS DOUBLE) * LO_DISCOUNT) as revenue from lineorder "
            "where D_WEEKNUMINYEAR = 6 and D_YEAR = 1994 and LO_DISCOUNT between 5 and 7 "
            "and LO_QUANTITY between 26 and 35",
    "Q2.1": "select sum(CAST(LO_REVENUE AS DOUBLE)), D_YEAR, P_BRAND1 from lineorder "
            "where P_CATEGORY = 'MFGR#12' and S_REGION = 'AMERICA' group by D_YEAR, P_BRAND1 "
            "order by D_YEAR, P_BRAND1 limit 100000",
    "Q2.2": "select sum(CAST(LO_REVENUE AS DOUBLE)), D_YEAR, P_BRAND1 from lineorder "
            "where P_BRAND1 between 'MFGR#2221' and 'MFGR#2228' and S_REGION = 'ASIA' "
            "group by D_YEAR, P_BRAND1 order by D_YEAR, P_BRAND1 limit 100000",
    "Q2.3": "select sum(CAST(LO_REVENUE AS DOUBLE)), D_YEAR, P_BRAND1 from lineorder "
            "where P_BRAND1 = 'MFGR#2221' and S_REGION = 'EUROPE' group by D_YEAR, P_BRAND1 "
            "order by D_YEAR, P_BRAND1 limit 100000",
    "Q3.1": "select C_NATION, S_NATION, D_YEAR, sum(LO_REVENUE) as revenue from lineorder "
            "where C_REGION = 'ASIA' and S_REGION = 'ASIA' and D_YEAR >= 1992 and D_YEAR <= 1997 "
            "group by C_NATION, S_NATION, D_YEAR order by D_YEAR asc, revenue desc limit 100000",
    "Q3.2": "select C_CITY, S_CITY, D_YEAR, sum(LO_REVENUE) as revenue from lineorder "
            "where C_NATION = 'UNITED STATES' and S_NATION = 'UNITED STATES' and D_YEAR >= 1992 "
            "and D_YEAR <= 1997 group by C_CITY, S_CITY, D_YEAR order by D_YEAR asc, revenue desc limit 100000",
    "Q3.3": "select C_CITY, S_CITY, D_YEAR, sum(LO_REVENUE) as revenue from lineorder "
            "where (C_CITY='UNITED KI1' or C_CITY='UNITED KI5') and (S_CITY='UNITED KI1' or S_CITY='UNITED KI5') "
            "and D_YEAR >= 1992 and D_YEAR <= 1997 group by C_CITY, S_CITY, D_YEAR "
            "order by D_YEAR asc, revenue desc limit 100000",
    "Q3.4": "select C_CITY, S_CITY, D_YEAR, sum(LO_REVENUE) as revenue from lineorder "
            "where (C_CITY='UNITED KI1' or C_CITY='UNITED KI5') and (S_CITY='UNITED KI1' or S_CITY='UNITED KI5') "
            "and D_YEARMONTH = 'Jul1995' group by C_CITY, S_CITY, D_YEAR order by D_YEAR asc, revenue desc "
            "limit 100000",
    "Q4.1": "select D_YEAR, C_NATION, sum(LO_REVENUE - LO_SUPPLYCOST) as profit from lineorder "
            "where C_REGION = 'AMERICA' and S_REGION = 'AMERICA' and (P_MFGR = 'MFGR#1' or P_MFGR = 'MFGR#2') "
            "group by D_YEAR, C_NATION order by D_YEAR, C_NATION limit 100000",
    "Q4.2": "select D_YEAR, S_NATION, P_CATEGORY, sum(LO_REVENUE - LO_SUPPLYCOST) as profit from lineorder "
            "where C_REGION = 'AMERICA' and S_REGION = 'AMERICA' and (D_YEAR = 1997 or D_YEAR = 1998) "
            "and (P_MFGR = 'MFGR#1' or P_MFGR = 'MFGR#2') group by D_YEAR, S_NATION, P_CATEGORY "
            "order by D_YEAR, S_NATION, P_CATEGORY limit 100000",
    "Q4.3": "select D_YEAR, S_CITY, P_BRAND1, sum(LO_REVENUE - LO_SUPPLYCOST) as profit from lineorder "
            "where C_REGION = 'AMERICA' and S_NATION = 'UNITED STATES' and (D_YEAR = 1997 or D_YEAR = 1998) "
            "and P_CATEGORY = 'MFGR#14' group by D_YEAR, S_CITY, P_BRAND1 order by D_YEAR, S_CITY, P_BRAND1 "
            "limit 100000",
    # config C5: DISTINCTCOUNTHLL + GROUP BY
    "C5": "select D_YEAR, C_NATION, DISTINCTCOUNTHLL(LO_CUSTKEY), sum(LO_REVENUE - LO_SUPPLYCOST) from lineorder "
          "where C_REGION = 'AMERICA' and S_REGION = 'AMERICA' group by D_YEAR, C_NATION "
          "order by D_YEAR, C_NATION limit 100000",
}


def build():
    src = os.path.join(_HERE, "ssbgen.c")
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-o", _SO, src, "-lm"])


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_SO)
        L.ssbgen_num_columns.restype = ctypes.c_int32
        L.ssbgen_column_name.argtypes = [ctypes.c_int32]
        L.ssbgen_column_name.restype = ctypes.c_char_p
        L.ssbgen_column_type.argtypes = [ctypes.c_int32]
        L.ssbgen_column_type.restype = ctypes.c_int32
        L.ssbgen_column.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                    ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
        L.ssbgen_column.restype = ctypes.c_int32
        _lib = L
    return _lib


def column_ids():
    L = lib()
    return {L.ssbgen_column_name(i).decode(): i for i in range(L.ssbgen_num_columns())}


def columns_for(queries):
    from pinot_amd.query.context import columns_of
    from pinot_amd.query.sql import parse
    cols = []
    for q in queries:
        qc = parse(SSB_QUERIES[q])
        need = list(qc.filter.columns()) if qc.filter else []
        for a in qc.aggregations:
            if a.argument is not None:
                need += columns_of(a.argument)
        for e in qc.group_by:
            need += columns_of(e)
        for c in need:
            if c not in cols:
                cols.append(c)
    return cols


LAYOUTS = {"unsorted": 0, "sorted": 1}  # sorted: rows ordered by LO_ORDERDATE


def _gen_column(seed, first_row, nrows, sf, cid, name, layout="unsorted"):
    L = lib()
    fwd = np.empty((nrows * 31 + 7) // 8 + 16, dtype=np.uint8)
    dict_cap = 11_000_000 * 4
    dbuf = np.empty(dict_cap, dtype=np.uint8)
    card, bits, width, srt = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    flen, dlen = ctypes.c_int64(), ctypes.c_int64()
    rc = L.ssbgen_column(seed, first_row, nrows, sf, cid, LAYOUTS[layout], fwd.ctypes.data, len(fwd),
                         dbuf.ctypes.data, dict_cap, ctypes.byref(card), ctypes.byref(bits), ctypes.byref(flen),
                         ctypes.byref(dlen), ctypes.byref(width), ctypes.byref(srt))
    if rc != 0:
        raise RuntimeError(f"ssbgen_column({name}) failed: {rc}")
    dt = DataType.STRING if L.ssbgen_column_type(cid) == 4 else DataType.INT
    meta = ColumnMetadata(name, dt, nrows, card.value, bits.value, bool(srt.value), True, False, width.value)
    return name, ColumnIndexes(meta, fwd[:flen.value].tobytes(), dbuf[:dlen.value].tobytes(), None)


def make_segments(sf, columns, seed=42, segment_rows=SEGMENT_ROWS, segments=None, workers=None, layout="unsorted"):
    """Segments [0, nseg) of an SF-`sf` flattened lineorder; `segments` selects a subset (indexes);
    layout "sorted" orders the rows by LO_ORDERDATE (date columns then carry sorted forward indexes)."""
    total = sf * ROWS_PER_SF
    nseg = (total + segment_rows - 1) // segment_rows
    which = list(range(nseg)) if segments is None else list(segments)
    ids = column_ids()
    tasks = []
    for s in which:
        first = s * segment_rows
        n = min(segment_rows, total - first)
        for c in columns:
            tasks.append((s, first, n, c))
    workers = workers or min(16, os.cpu_count() or 4)
    with ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(lambda t: (t[0], _gen_column(seed, t[1], t[2], sf, ids[t[3]], t[3], layout)), tasks))
    out = {}
    for s in which:
        first = s * segment_rows
        out[s] = ImmutableSegment(f"lineorder_{s}", min(segment_rows, total - first))
    for s, (name, ci) in res:
        out[s].columns[name] = ci
    return [out[s] for s in which]
