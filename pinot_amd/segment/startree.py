"""Star-tree index: builder and the host-side tree.

Restates the reference's single-tree builder
(pinot-segment-local/.../startree/v2/builder/BaseSingleTreeBuilder.java:300-460, OnHeapSingleTreeBuilder.java:60-159):

* segment records (dimension dict ids in ``dimensionsSplitOrder``, metric values) are sorted by the dimensions
  and records with equal dimensions aggregated (``sortAndAggregateSegmentRecords``);
* ``constructStarTree``: a node whose range holds more than ``maxLeafRecords`` records is split on the next
  dimension into one child per value (the records are sorted, so every child is a contiguous range) plus, when it
  has more than one child and the dimension is not in ``skipStarNodeCreationForDimensions``, a star child whose
  records -- appended at the end -- are the node's records with that dimension replaced by STAR, re-sorted by the
  remaining dimensions and aggregated (``generateRecordsForStarNode``);
* ``createAggregatedDocs``: every node gets an aggregated document (one appended record with every deeper
  dimension STAR; a one-record leaf reuses its record; a node with a star child reuses the star child's).

STAR is stored as dictionary id 0 in the star-tree forward index (StarTreeV2Constants.STAR_IN_FORWARD_INDEX = 0),
and ALL (-1) names the star child. Metric columns are named like AggregationFunctionColumnPair.toColumnName
(``sum__col``, ``count__*``, ``min__col``, ``max__col``, ``avg__col``) and hold the aggregated values the
ValueAggregators produce (SUM / MIN / MAX as DOUBLE, COUNT as LONG). AvgValueAggregator's AvgPair (sum, count) is held
as two numeric columns, ``avg__col`` (the DOUBLE sum) and ``avg__col$count`` (the LONG count), so the GPU sums both
like any metric instead of decoding serialized pairs. DistinctCountHLLValueAggregator's HyperLogLog (log2m 8, the
default) is held as its registers: ``distinctcounthll__col`` stores 256 u8 registers per star-tree document (the
register-wise max of its raw documents' (register, rho) offers), which the GPU max-merges per matched document
(PHIP_FWD_HLL_REGISTERS) instead of deserializing clearspring HyperLogLog bytes. The star-tree documents form an ordinary
ImmutableSegment (dimension columns share the parent segment's dictionaries), so the GPU loads and scans them with
the same kernels as any segment.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..spi import DataType

STAR_IN_FORWARD_INDEX = 0  # StarTreeV2Constants.java:39
ALL = -1                   # StarTreeNode.ALL
DEFAULT_MAX_LEAF_RECORDS = 10_000  # StarTreeV2BuilderConfig.DEFAULT_MAX_LEAF_RECORDS

_PAIR_FUNCS = ("sum", "count", "min", "max", "avg", "distinctcounthll")
STAR_HLL_LOG2M = 8  # DistinctCountHLLValueAggregator: HyperLogLog(log2m = 8) unless configured


@dataclass(frozen=True)
class StarTreeIndexConfig:
    """StarTreeIndexConfig (pinot-spi/.../config/table/StarTreeIndexConfig.java): split order, star-node
    skips, function-column pairs (``"SUM__col"``, ``"COUNT__*"``, ...; case-insensitive function) and
    maxLeafRecords."""
    dimensions_split_order: Sequence[str]
    function_column_pairs: Sequence[str]
    skip_star_node_creation: Sequence[str] = ()
    max_leaf_records: int = DEFAULT_MAX_LEAF_RECORDS

    def pairs(self):
        out = []
        for p in self.function_column_pairs:
            f, _, c = p.partition("__")
            f = f.lower()
            if f not in _PAIR_FUNCS:
                raise ValueError(f"star-tree function {f} is outside the GPU subset (SUM/COUNT/MIN/MAX/AVG/"
                                 f"DISTINCTCOUNTHLL)")
            if f == "count":
                c = "*"
            if (f, c) not in out:
                out.append((f, c))
        return out


@dataclass
class TreeNode:
    dimension_id: int = -1
    dimension_value: int = ALL
    start_doc: int = 0
    end_doc: int = 0
    aggregated_doc: int = -1
    child_dimension_id: int = -1
    children: Optional[Dict[int, "TreeNode"]] = None  # dimension value (ALL for the star child) -> node

    @property
    def is_leaf(self):
        return self.children is None


def pair_column(f, c):
    """AggregationFunctionColumnPair.toColumnName."""
    return f"{f}__{c}"


def avg_count_column(c):
    """The count half of an AVG pair's (sum, count) (AvgPair.getCount)."""
    return f"avg__{c}$count"


def metric_slots(pairs):
    """Per function-column pair, its stored metrics as (column name, aggregation kind): AVG expands to its sum and
    its count (AvgValueAggregator.applyRawValue: sum += value, count += 1)."""
    out = []
    for f, c in pairs:
        if f == "avg":
            out += [(pair_column(f, c), "sum", c), (avg_count_column(c), "count", c)]
        elif f == "distinctcounthll":
            out.append((pair_column(f, c), "hll", c))
        else:
            out.append((pair_column(f, c), f, c))
    return out


@dataclass
class StarTree:
    config: StarTreeIndexConfig
    dimensions: List[str]
    root: TreeNode
    num_nodes: int
    docs: object              # ImmutableSegment of the star-tree documents
    pairs: List[tuple] = field(default_factory=list)

    def pair_columns(self):
        return [pair_column(f, c) for f, c in self.pairs]


class _Records:
    """Growable record store (dimension ids + aggregated metric values)."""

    def __init__(self, k, metric_dtypes, cap=1024):
        self.k = k
        self.n = 0
        self.dims = np.zeros((cap, k), dtype=np.int32)
        # metric_dtypes: a dtype, or (dtype, row width) for register rows
        self.mets = [np.zeros((cap, dt[1]), dtype=dt[0]) if isinstance(dt, tuple) else np.zeros(cap, dtype=dt)
                     for dt in metric_dtypes]

    def append(self, dims, mets):
        m = len(dims)
        if self.n + m > len(self.dims):
            cap = max(2 * len(self.dims), self.n + m)
            nd = np.zeros((cap, self.k), dtype=np.int32)
            nd[:self.n] = self.dims[:self.n]
            self.dims = nd
            for i, a in enumerate(self.mets):
                na = np.zeros((cap,) + a.shape[1:], dtype=a.dtype)
                na[:self.n] = a[:self.n]
                self.mets[i] = na
        self.dims[self.n:self.n + m] = dims
        for a, v in zip(self.mets, mets):
            a[self.n:self.n + m] = v
        self.n += m


def _aggregate_runs(dims, mets, funcs):
    """Sorted records -> one record per run of equal dimensions, metrics merged in record order
    (ValueAggregator.applyAggregatedValue: SUM/COUNT add, MIN/MAX compare, HLL register-wise max; raw HLL records
    arrive as packed (register << 8 | rho) offers and leave as register rows)."""
    n = len(dims)
    if n == 0:
        return dims, mets
    change = np.ones(n, dtype=bool)
    change[1:] = np.any(dims[1:] != dims[:-1], axis=1)
    starts = np.flatnonzero(change)
    out = []
    for f, v in zip(funcs, mets):
        if f in ("sum", "count"):
            out.append(np.add.reduceat(v, starts))
        elif f == "min":
            out.append(np.minimum.reduceat(v, starts))
        elif f == "hll" and v.ndim == 1:  # raw offers -> one register row per run
            run = np.cumsum(change) - 1
            rows = np.zeros((len(starts), 1 << STAR_HLL_LOG2M), dtype=np.uint8)
            np.maximum.at(rows, (run, (v >> 8).astype(np.int64)), (v & 0xFF).astype(np.uint8))
            out.append(rows)
        else:
            out.append(np.maximum.reduceat(v, starts, axis=0))
    return dims[starts], out


class _Builder:
    def __init__(self, config, dims_ids, metric_values, metric_types=None):
        metric_types = metric_types or {}
        self.cfg = config
        self.dimensions = list(config.dimensions_split_order)
        self.k = len(self.dimensions)
        self.pairs = config.pairs()
        self.slots = metric_slots(self.pairs)
        self.funcs = [k for _, k, _ in self.slots]
        self.skip = {self.dimensions.index(d) for d in config.skip_star_node_creation}
        self.max_leaf = int(config.max_leaf_records)
        n = len(dims_ids[0]) if dims_ids else 0
        D = np.stack([np.asarray(a, dtype=np.int32) for a in dims_ids], axis=1) if self.k else np.zeros((n, 0), np.int32)
        M = []
        for _, k, c in self.slots:
            if k == "count":
                M.append(np.ones(n, dtype=np.int64))     # CountValueAggregator / AvgPair count: 1 per raw record
            elif k == "hll":  # DistinctCountHLLValueAggregator.getInitialAggregatedValue: offer the raw value
                from ..engine.hll import hash_values, register_rho
                from ..spi import DataType as _DT
                vals = metric_values[c]
                dt = _DT.STRING if (len(vals) and isinstance(vals[0], str)) else (
                    _DT.LONG if np.asarray(vals).dtype.kind in "iu" else _DT.DOUBLE)
                j, rho = register_rho(hash_values(vals, metric_types.get(c, dt)), STAR_HLL_LOG2M)
                M.append((j << 8 | rho).astype(np.int32))
            else:
                M.append(np.asarray(metric_values[c], dtype=np.float64))  # Sum/Min/Max/Avg sum: doubleValue()
        # sortAndAggregateSegmentRecords: sort by the dimensions in split order, merge equal ones
        order = np.lexsort(D.T[::-1]) if self.k else np.arange(n)
        dims, mets = _aggregate_runs(D[order], [m[order] for m in M], self.funcs)
        self.rec = _Records(self.k, [(m.dtype, m.shape[1]) if m.ndim == 2 else m.dtype for m in mets],
                            cap=max(2 * len(dims), 16))
        self.rec.append(dims, mets)
        self.num_nodes = 1
        self.root = TreeNode(start_doc=0, end_doc=self.rec.n)

    def build(self):
        if self.rec.n:
            self._construct(self.root, 0, self.rec.n)
            self._aggregated_docs(self.root)
        return self.root

    def _construct(self, node, start, end):
        child_dim = node.dimension_id + 1
        if child_dim == self.k:
            return
        node.child_dimension_id = child_dim
        vals = self.rec.dims[start:end, child_dim]
        change = np.flatnonzero(vals[1:] != vals[:-1]) + 1
        bounds = np.concatenate(([0], change, [end - start]))
        children = {}
        for a, b in zip(bounds[:-1], bounds[1:]):
            self.num_nodes += 1
            children[int(vals[a])] = TreeNode(child_dim, int(vals[a]), start + int(a), start + int(b))
        node.children = children
        # one-record leaves tiling the node's range (the traversal then takes them as one range)
        node._bulk = len(children) > 64 and bool(np.all(np.diff(bounds) == 1))
        if child_dim not in self.skip and len(children) > 1:
            children[ALL] = self._star_node(start, end, child_dim)
        for child in list(children.values()):
            if child.end_doc - child.start_doc > self.max_leaf:
                self._construct(child, child.start_doc, child.end_doc)

    def _star_node(self, start, end, dim):
        """constructStarNode / generateRecordsForStarNode: stable sort by the dimensions after ``dim``."""
        self.num_nodes += 1
        dims = self.rec.dims[start:end].copy()
        mets = [m[start:end].copy() for m in self.rec.mets]
        dims[:, dim] = STAR_IN_FORWARD_INDEX
        after = dims[:, dim + 1:]
        order = np.lexsort(after.T[::-1]) if after.shape[1] else np.arange(len(dims))
        d2, m2 = _aggregate_runs(dims[order], [m[order] for m in mets], self.funcs)
        node = TreeNode(dim, ALL, self.rec.n, self.rec.n + len(d2))
        self.rec.append(d2, m2)
        return node

    def _merge_range(self, start, end):
        dims = self.rec.dims[start].copy()
        mets = []
        for f, m in zip(self.funcs, self.rec.mets):
            seg = m[start:end]
            mets.append(seg.sum() if f in ("sum", "count") else (seg.min() if f == "min" else seg.max(axis=0)))
        return dims, mets

    def _append_aggregated(self, node, dims, mets):
        dims = dims.copy()
        dims[node.dimension_id + 1:] = STAR_IN_FORWARD_INDEX
        node.aggregated_doc = self.rec.n
        self.rec.append(dims[None, :], [np.asarray(v)[None] for v in mets])

    def _aggregated_docs(self, node):
        """createAggregatedDocs (BaseSingleTreeBuilder.java:414-455); returns the node's aggregated record."""
        if node.children is None:
            if node.start_doc == node.end_doc - 1:
                node.aggregated_doc = node.start_doc
                return self.rec.dims[node.start_doc].copy(), [m[node.start_doc].copy() for m in self.rec.mets]
            dims, mets = self._merge_range(node.start_doc, node.end_doc)
            self._append_aggregated(node, dims, mets)
            return dims, mets
        if ALL in node.children:
            out = None
            for v, child in node.children.items():
                r = self._aggregated_docs(child)
                if v == ALL:
                    out = r
                    node.aggregated_doc = child.aggregated_doc
            return out
        acc_d, acc_m = None, None
        for child in node.children.values():
            d, m = self._aggregated_docs(child)
            if acc_d is None:
                acc_d, acc_m = d.copy(), list(m)
            else:
                acc_m = [(a + b) if f in ("sum", "count") else
                         (min(a, b) if f == "min" else (np.maximum(a, b) if f == "hll" else max(a, b)))
                         for f, a, b in zip(self.funcs, acc_m, m)]
        self._append_aggregated(node, acc_d, acc_m)
        return acc_d, acc_m


def build_star_tree(config: StarTreeIndexConfig, dims_ids: Sequence[np.ndarray], dim_columns, metric_values,
                    name: str, metric_types=None) -> StarTree:
    """Builds one star-tree over a segment: ``dims_ids`` = the dict ids of every split-order dimension,
    ``dim_columns`` = their ColumnIndexes (dictionaries and metadata are shared with the star-tree docs),
    ``metric_values`` = column -> raw values for the SUM / MIN / MAX pairs."""
    from .creator import ColumnIndexes, ColumnMetadata, ImmutableSegment, _chunk_forward, pack_bits
    b = _Builder(config, dims_ids, metric_values, metric_types or {})
    root = b.build()
    n = b.rec.n
    seg = ImmutableSegment(name, n)
    for j, dim in enumerate(b.dimensions):
        src = dim_columns[j]
        m = src.metadata
        ids = b.rec.dims[:n, j]
        meta = ColumnMetadata(dim, m.data_type, n, m.cardinality, m.bits_per_element, False, True, False,
                              m.string_width)
        seg.columns[dim] = ColumnIndexes(meta, pack_bits(ids, m.bits_per_element), src.dictionary, None)
    for (col, k, _), vals in zip(b.slots, b.rec.mets):
        if k == "hll":  # register rows, 2^log2m bytes per star-tree document
            meta = ColumnMetadata(col, DataType.LONG, n, 0, 0, False, False, False, 0, STAR_HLL_LOG2M)
            seg.columns[col] = ColumnIndexes(meta, np.ascontiguousarray(vals[:n], dtype=np.uint8).tobytes())
            continue
        dt = DataType.LONG if k == "count" else DataType.DOUBLE
        meta = ColumnMetadata(col, dt, n, 0, 0, False, False, False)
        seg.columns[col] = ColumnIndexes(meta, _chunk_forward(vals[:n], dt))
    return StarTree(config, b.dimensions, root, b.num_nodes, seg, b.pairs)


# ------------------------------------------------------------------------------------------------------
# Pinot's on-disk star-tree (segment v3: star_tree_index + star_tree_index_map, metadata.properties startree.v2.*),
# so that a server pins Pinot-written star-trees at load instead of rebuilding them.
# ------------------------------------------------------------------------------------------------------
STAR_TREE_MAGIC = 0xBADDA55B00DAD00D  # OffHeapStarTree.MAGIC_MARKER
STAR_TREE_VERSION = 1                 # OffHeapStarTree.VERSION
_NODE_INTS = 7                        # OffHeapStarTreeNode.NUM_SERIALIZABLE_FIELDS


def parse_properties(text: str) -> Dict[str, List[str]]:
    """metadata.properties / star_tree_index_map as Commons Configuration reads them: `key = value` lines,
    `#` comments, a key may repeat (a list). Values are returned unescaped of the `\\uXXXX` forms."""
    out: Dict[str, List[str]] = {}
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#") or line.startswith("!"):
            continue
        k, sep, v = line.partition("=")
        if not sep:
            continue
        v = v.strip()
        if "\\u" in v:
            v = v.encode("latin-1", "backslashreplace").decode("unicode_escape")
        out.setdefault(k.strip(), []).append(v)
    return out


def star_tree_metadata(props: Dict[str, List[str]]) -> List[dict]:
    """StarTreeV2Metadata of every tree (SegmentMetadataImpl: startree.v2.count, startree.v2.<i>.total.docs /
    split.order / function.column.pairs / skip.star.node.creation / max.leaf.records)."""
    n = int(props.get("startree.v2.count", ["0"])[0])
    out = []
    for i in range(n):
        p = f"startree.v2.{i}."
        split = [x.strip() for v in props.get(p + "split.order", []) for x in v.split(",") if x.strip()]
        pairs = [x.strip() for v in props.get(p + "function.column.pairs", []) for x in v.split(",") if x.strip()]
        skip = [x.strip() for v in props.get(p + "skip.star.node.creation", []) for x in v.split(",") if x.strip()]
        out.append({"total_docs": int(props[p + "total.docs"][0]), "split_order": split, "pairs": pairs,
                    "skip": skip, "max_leaf_records": int(props.get(p + "max.leaf.records", [DEFAULT_MAX_LEAF_RECORDS])[0])})
    return out


def parse_star_tree_index_map(text: str) -> Dict[tuple, tuple]:
    """star_tree_index_map (StarTreeIndexMapUtils): `<tree>.<column>.<STAR_TREE|FORWARD_INDEX>.OFFSET / .SIZE`
    -> {(tree, column or None, type): (offset, size)}."""
    raw: Dict[tuple, dict] = {}
    for k, vs in parse_properties(text).items():
        parts = k.split(".")
        tree, field_ = int(parts[0]), parts[-1]
        kind = parts[-2]
        col = ".".join(parts[1:-2])
        raw.setdefault((tree, None if col == "null" else col, kind), {})[field_] = int(vs[0])
    return {key: (v["OFFSET"], v["SIZE"]) for key, v in raw.items()}


def decode_off_heap_tree(buf: bytes):
    """OffHeapStarTree (OffHeapStarTree.java:38-79, little-endian): magic, version, root node offset, dimension
    names (id, utf-8 bytes), node count, then 7-int nodes (OffHeapStarTreeNode.java: dimension id, dimension value,
    start doc, end doc (exclusive), aggregated doc, first child, last child; -1 = no child). Returns
    (dimension names, root TreeNode, node count)."""
    import struct
    magic, version, root_off, ndims = struct.unpack_from("<QiiI", buf, 0)
    if magic != STAR_TREE_MAGIC:
        raise ValueError("invalid magic marker in star-tree data buffer")
    if version != STAR_TREE_VERSION:
        raise ValueError(f"star-tree version {version} is not {STAR_TREE_VERSION}")
    off = 20
    names: List[Optional[str]] = [None] * ndims
    for _ in range(ndims):
        did, nb = struct.unpack_from("<ii", buf, off)
        off += 8
        names[did] = bytes(buf[off:off + nb]).decode("utf-8")
        off += nb
    (num_nodes,) = struct.unpack_from("<i", buf, off)
    off += 4
    if off != root_off:
        raise ValueError("star-tree header length mismatch")
    if off + num_nodes * _NODE_INTS * 4 != len(buf):
        raise ValueError("star-tree buffer size mismatch")
    nd = np.frombuffer(buf, dtype="<i4", count=num_nodes * _NODE_INTS, offset=off).reshape(num_nodes, _NODE_INTS)
    if num_nodes == 0:
        raise ValueError("star-tree without nodes")

    def make(i):
        r = nd[i]
        return TreeNode(int(r[0]), int(r[1]), int(r[2]), int(r[3]), int(r[4]))

    nodes = [make(i) for i in range(num_nodes)]
    # (the writer leaves the root's doc range unset, -1 / -1: it is the span of its non-star children)
    for i in range(num_nodes):
        first, last = int(nd[i, 5]), int(nd[i, 6])
        if first < 0:
            continue
        if not (i < first <= last < num_nodes):
            raise ValueError(f"star-tree node {i}: children [{first}, {last}] out of order")
        kids = {}
        for c in range(first, last + 1):
            kids[nodes[c].dimension_value] = nodes[c]  # ALL (-1) is the star child (serialized first)
        nodes[i].children = kids
        nodes[i].child_dimension_id = int(nd[first, 0])
    root = nodes[0]
    if root.start_doc < 0 and root.children:
        kids = [c for v, c in root.children.items() if v != ALL]
        root.start_doc = min(c.start_doc for c in kids)
        root.end_doc = max(c.end_doc for c in kids)
    return [str(n) for n in names], root, num_nodes


def read_pinot_star_trees(index: bytes, index_map: str, metadata: str, parent_columns, name: str = "startree"
                          ) -> List[StarTree]:
    """Every star-tree of a Pinot v3 segment directory, as the StarTree the GPU star-tree operator traverses
    (StarTreeIndexReader.java: one buffer, the tree little-endian, forward indexes big-endian). The star-tree
    documents become an ImmutableSegment: split-order dimensions as fixed-bit dict ids sharing the parent
    column's dictionary (`parent_columns`: column -> ColumnIndexes of the segment), function-column pairs as
    the raw chunk forward indexes Pinot wrote (count__* LONG, sum / min / max DOUBLE: the ValueAggregators'
    result types)."""
    from .creator import ColumnIndexes, ColumnMetadata, ImmutableSegment
    metas = star_tree_metadata(parse_properties(metadata))
    entries = parse_star_tree_index_map(index_map)
    out = []
    for i, m in enumerate(metas):
        off, size = entries[(i, None, "STAR_TREE")]
        dims, root, num_nodes = decode_off_heap_tree(index[off:off + size])
        if dims != m["split_order"]:
            raise ValueError(f"star-tree {i}: dimensions {dims} differ from the split order {m['split_order']}")
        cfg = StarTreeIndexConfig(tuple(dims), tuple(m["pairs"]), tuple(m["skip"]), m["max_leaf_records"])
        n = m["total_docs"]
        seg = ImmutableSegment(f"{name}{i}", n)
        for d in dims:
            src = parent_columns[d].metadata
            o, sz = entries[(i, d, "FORWARD_INDEX")]
            want = (n * src.bits_per_element + 7) // 8
            if sz < want:
                raise ValueError(f"star-tree {i}: forward index of {d} holds {sz} bytes, {want} needed")
            meta = ColumnMetadata(d, src.data_type, n, src.cardinality, src.bits_per_element, False, True, False,
                                  src.string_width)
            seg.columns[d] = ColumnIndexes(meta, bytes(index[o:o + sz]), parent_columns[d].dictionary, None)
        pairs = cfg.pairs()
        for f, c in pairs:
            if f in ("avg", "distinctcounthll"):  # serialized AvgPair / HyperLogLog bytes (var-byte chunk indexes)
                raise ValueError(f"star-tree {i}: {f.upper()} pairs are serialized objects, not read here")
            col = pair_column(f, c)
            o, sz = entries[(i, col, "FORWARD_INDEX")]
            dt = DataType.LONG if f == "count" else DataType.DOUBLE
            seg.columns[col] = ColumnIndexes(ColumnMetadata(col, dt, n, 0, 0, False, False, False), bytes(index[o:o + sz]))
        out.append(StarTree(cfg, list(dims), root, num_nodes, seg, pairs))
    return out
