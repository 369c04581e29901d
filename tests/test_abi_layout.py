"""CPU test: the ctypes mirror of the C ABI (pinot_amd/_lib.py) has the byte layout of include/pinot_hip.h.

A gcc-compiled probe prints sizeof / offsetof for every field of every ABI struct; the ctypes
Structures must agree field by field (the same layout a Java FFM StructLayout binds).
"""
import ctypes
import os
import shutil
import subprocess

import pytest

from pinot_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAIRS = [("phip_column_desc", _lib.ColumnDesc), ("phip_segment_desc", _lib.SegmentDesc),
         ("phip_raw_range", _lib.RawRange), ("phip_filter_node", _lib.FilterNode),
         ("phip_aggregation", _lib.Aggregation), ("phip_query_desc", _lib.QueryDesc),
         ("phip_select_expr", _lib.SelectExpr),
         ("phip_order_term", _lib.OrderTerm),
         ("phip_result", _lib.Result), ("phip_dictionary_view", _lib.DictionaryView),
         ("phip_partial", _lib.Partial)]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_ctypes_layout_matches_header(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "include/pinot_hip.h"', "int main(void) {"]
    for cname, py in PAIRS:
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", ROOT, "-o", str(exe), str(src)])
    got = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        c, f, v = line.split()
        got[(c, f)] = int(v)
    for cname, py in PAIRS:
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def _declared_symbols():
    import re
    with open(os.path.join(ROOT, "include", "pinot_hip.h")) as f:
        text = f.read()
    return set(re.findall(r"PHIP_API\s+[\w\s\*]+?\b(phip_\w+)\s*\(", text))


def test_library_exports_every_declared_symbol():
    """The built libpinot_hip.so loads on a GPU-less host and exports every entry point the header declares
    (dlsym only -- no compute call without a GPU); the ctypes mirror binds exactly that set."""
    declared = _declared_symbols()
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libpinot_hip.so not built (python -c 'import __graft_entry__ as g; g.build()')")
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in sorted(declared) if not hasattr(so, s)]
    assert not missing, missing
