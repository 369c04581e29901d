"""Pinot's own star-tree bytes (tests/golden/pinot_startree, copied by make_pinot_startree.py from the reference's
pinot-segment-local/src/test/resources/data/startree/segment, used by StarTreeIndexSeparatorTest.java:43) read
by the product's reader (pinot_amd/segment/startree.read_pinot_star_trees), and pinned against the raw rows the
segment was built from (the reference's airlineStats 2014-01-15 Avro: 313 rows, DaysSinceEpoch 16085).

Every one of the 1004 star-tree documents is checked: its count__* and max__ArrDelay equal COUNT(*) and
MAX(ArrDelay) of the raw rows that match its non-star dimension values (a star dimension matches every row),
and the tree's invariants hold (root aggregate = 313 = segment.total.docs; a star child's aggregate = the
aggregate of its non-star siblings; a node's aggregated document = the aggregate of its documents)."""
import os

import numpy as np
import pytest

from oracle.executor import OracleSegment
from pinot_amd.segment import startree as st
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pinot_startree")
DIMS = ["AirlineID", "Origin", "Dest"]


def raw_rows():
    d = np.load(os.path.join(HERE, "airline_2014_01_15.npz"))
    return {k: d[k] for k in d.files}


def parent_segment():
    """The 313-row segment rebuilt from the raw rows: Pinot's dictionaries are the sorted distinct values, so
    these dict ids are the ones the star-tree forward indexes hold."""
    r = raw_rows()
    c = SegmentCreator("airlineStats_OFFLINE_16085_16085_0")
    c.add_column("AirlineID", DataType.INT, r["AirlineID"])
    c.add_column("Origin", DataType.STRING, r["Origin"])
    c.add_column("Dest", DataType.STRING, r["Dest"])
    c.add_column("ArrDelay", DataType.INT, r["ArrDelay"])
    return c.build()


def pinot_tree(seg):
    with open(os.path.join(HERE, "star_tree_index"), "rb") as f:
        idx = f.read()
    with open(os.path.join(HERE, "star_tree_index_map")) as f:
        imap = f.read()
    with open(os.path.join(HERE, "metadata.properties")) as f:
        meta = f.read()
    trees = st.read_pinot_star_trees(idx, imap, meta, seg.columns, name=seg.name + ".startree")
    assert len(trees) == 1
    return trees[0]


@pytest.fixture(scope="module")
def tree_and_segment():
    seg = parent_segment()
    return pinot_tree(seg), seg


def _walk(node, starred, out):
    """(node, dims starred on its path) for every node."""
    out.append((node, frozenset(starred)))
    if node.children:
        for v, c in node.children.items():
            _walk(c, starred | ({c.dimension_id} if v == st.ALL else set()), out)
    return out


def test_metadata_matches_segment():
    props = st.parse_properties(open(os.path.join(HERE, "metadata.properties")).read())
    assert props["segment.total.docs"] == ["313"]
    for d, card, bits in (("AirlineID", 14, 4), ("Origin", 97, 7), ("Dest", 104, 7)):
        assert int(props[f"column.{d}.cardinality"][0]) == card
        assert int(props[f"column.{d}.bitsPerElement"][0]) == bits
    seg = parent_segment()
    for d in DIMS:
        m = seg.columns[d].metadata
        assert m.cardinality == int(props[f"column.{d}.cardinality"][0])
        assert m.bits_per_element == int(props[f"column.{d}.bitsPerElement"][0])


def test_tree_structure(tree_and_segment):
    tree, _ = tree_and_segment
    assert tree.dimensions == DIMS
    assert tree.docs.num_docs == 1004
    assert tree.pairs == [("count", "*"), ("max", "ArrDelay")]
    assert tree.config.max_leaf_records == 10
    nodes = _walk(tree.root, set(), [])
    assert len(nodes) == tree.num_nodes
    for n, _ in nodes:
        if n.children:
            vals = [v for v in n.children if v != st.ALL]
            assert vals == sorted(vals) and len(set(vals)) == len(vals)
            assert all(c.dimension_id == n.child_dimension_id for c in n.children.values())
            assert n.children[vals[0]].dimension_id == n.dimension_id + 1
        else:
            assert 0 <= n.start_doc < n.end_doc <= 1004
            # maxLeafRecords: a leaf is not split further when it holds at most 10 records or is at the last level
            assert n.end_doc - n.start_doc <= 10 or n.dimension_id == len(DIMS) - 1


def test_aggregates_and_star_invariants(tree_and_segment):
    tree, _ = tree_and_segment
    o = OracleSegment(tree.docs)
    cnt = np.asarray(o.values("count__*"), dtype=np.int64)
    mx = np.asarray(o.values("max__ArrDelay"), dtype=np.float64)
    assert cnt[tree.root.aggregated_doc] == 313  # = segment.total.docs
    for n, _ in _walk(tree.root, set(), []):
        a = n.aggregated_doc
        if n is not tree.root:
            # the aggregated document of a node aggregates the node's documents
            assert cnt[a] == cnt[n.start_doc:n.end_doc].sum(), (n.dimension_id, n.dimension_value)
            assert mx[a] == mx[n.start_doc:n.end_doc].max()
        if n.children and st.ALL in n.children:
            star = n.children[st.ALL]
            kids = [c for v, c in n.children.items() if v != st.ALL]
            assert cnt[star.aggregated_doc] == sum(cnt[c.aggregated_doc] for c in kids)
            assert mx[star.aggregated_doc] == max(mx[c.aggregated_doc] for c in kids)
            # createAggregatedDocs: a node with a star child takes the star child's aggregated document
            assert n.aggregated_doc == star.aggregated_doc


def test_every_document_against_the_raw_rows(tree_and_segment):
    """Each star-tree document = COUNT(*) / MAX(ArrDelay) of the raw rows matching its non-star dimensions."""
    tree, seg = tree_and_segment
    o = OracleSegment(tree.docs)
    ids = {d: np.asarray(o.dict_ids(d)) for d in DIMS}
    cnt = np.asarray(o.values("count__*"), dtype=np.int64)
    mx = np.asarray(o.values("max__ArrDelay"), dtype=np.float64)
    po = OracleSegment(seg)
    raw_ids = {d: np.asarray(po.dict_ids(d)) for d in DIMS}
    arr = np.asarray(po.values("ArrDelay"), dtype=np.float64)
    starred = {}  # doc -> dims starred
    for n, s in _walk(tree.root, set(), []):
        if not n.children:
            for d in range(n.start_doc, n.end_doc):
                assert starred.setdefault(d, s) == s
        a = n.aggregated_doc
        agg_star = s | set(range(n.dimension_id + 1, len(DIMS)))
        if a >= 0 and not (n.start_doc <= a < n.end_doc and not n.children):
            starred.setdefault(a, frozenset(agg_star))
    assert sorted(starred) == list(range(1004)), "every document is a leaf record or an aggregated document"
    for doc, s in starred.items():
        m = np.ones(len(arr), dtype=bool)
        for j, d in enumerate(DIMS):
            if j not in s:
                m &= raw_ids[d] == ids[d][doc]
            else:
                assert ids[d][doc] == st.STAR_IN_FORWARD_INDEX
        assert cnt[doc] == int(m.sum()) > 0, doc
        assert mx[doc] == arr[m].max(), doc


# Queries the tree fits (split-order dimensions; count__* / max__ArrDelay), answered from Pinot's star-tree
# documents by the host traversal (engine/startree.traverse) + the oracle, against the oracle over the 313 raw rows
# -- BaseStarTreeV2Test's criterion on Pinot-written bytes.
QUERIES = [
    "SELECT COUNT(*), MAX(ArrDelay) FROM t",
    "SELECT AirlineID, COUNT(*), MAX(ArrDelay) FROM t GROUP BY AirlineID ORDER BY AirlineID LIMIT 100",
    "SELECT Origin, COUNT(*) FROM t WHERE AirlineID = 19805 GROUP BY Origin ORDER BY Origin LIMIT 100",
    "SELECT Dest, MAX(ArrDelay), COUNT(*) FROM t WHERE Origin IN ('LAX', 'ORD', 'SFO') GROUP BY Dest "
    "ORDER BY Dest LIMIT 200",
    "SELECT COUNT(*), MAX(ArrDelay) FROM t WHERE Dest = 'JFK' AND AirlineID <> 19805",
    "SELECT AirlineID, Dest, COUNT(*), MAX(ArrDelay) FROM t WHERE Origin BETWEEN 'A' AND 'M' "
    "GROUP BY AirlineID, Dest ORDER BY AirlineID, Dest LIMIT 500",
    "SELECT Origin, Dest, COUNT(*) FROM t GROUP BY Origin, Dest ORDER BY COUNT(*) DESC, Origin, Dest LIMIT 10",
    "SELECT COUNT(*) FROM t WHERE NOT Origin = 'LAX' AND (Dest = 'JFK' OR Dest = 'ORD')",
]


def star_segment():
    seg = parent_segment()
    seg.star_trees = [pinot_tree(seg)]
    return seg


@pytest.mark.parametrize("sql", QUERIES)
def test_host_traversal_equals_scan(sql):
    from oracle import executor
    from pinot_amd.query.sql import parse
    from tests.test_startree import _star_answer
    seg = star_segment()
    qc = parse(sql)
    got, ndocs = _star_answer(qc, seg)
    want, _ = executor.execute(qc, [seg])
    assert ndocs > 0
    if not qc.group_by:
        assert [float(x) for x in got] == [float(x) for x in want.results]
    else:
        assert set(got) == set(want.groups)
        for k, v in want.groups.items():
            assert [float(x) for x in got[k]] == [float(x) for x in v], k
