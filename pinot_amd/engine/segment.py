"""HBM-resident segment (the GPU side of ImmutableSegmentLoader.load).

``GpuSegment(segment)`` hands every column's index buffers to ``phip_segment_load`` — the point
where the reference maps them (ImmutableSegmentLoader.java:222-280,
PhysicalColumnIndexContainer.java:44-68) — and keeps the host-side readers the plan needs
(dictionaries for predicate evaluation, the sorted index for doc ranges).
"""
import ctypes

import numpy as np

from .. import _lib
from ..segment.creator import ImmutableSegment
from ..segment.dictionary import Dictionary


class GpuSegment:
    def __init__(self, segment: ImmutableSegment, device: int = -1):
        lib = _lib.load()
        self.segment = segment
        self.name = segment.name
        self.num_docs = segment.num_docs
        self._dicts = {}
        self._sorted = {}
        self._inv_offsets = {}
        cols = list(segment.columns.values())
        descs = (_lib.ColumnDesc * max(len(cols), 1))()
        keep = []
        for i, ci in enumerate(cols):
            m = ci.metadata
            d = descs[i]
            name = m.name.encode()
            keep.append(name)
            d.name = name
            d.data_type = int(m.data_type)
            if getattr(m, "hll_log2m", 0):  # star-tree DISTINCTCOUNTHLL pair: register rows
                d.fwd_kind = _lib.FWD_HLL_REGISTERS
            elif not m.has_dictionary:
                d.fwd_kind = _lib.FWD_RAW_CHUNK
            elif m.is_sorted:
                d.fwd_kind = _lib.FWD_SORTED
            else:
                d.fwd_kind = _lib.FWD_FIXED_BIT
            d.cardinality = m.cardinality
            d.bits_per_value = m.hll_log2m if getattr(m, "hll_log2m", 0) else m.bits_per_element
            d.string_width = m.string_width
            for attr, buf in (("forward", ci.forward), ("dictionary", ci.dictionary), ("inverted", ci.inverted),
                              ("null_vector", getattr(ci, "null_vector", None))):
                if buf is None:
                    setattr(d, attr, None)
                    setattr(d, attr + "_bytes", 0)
                else:
                    arr = np.frombuffer(buf, dtype=np.uint8)
                    keep.append(arr)
                    setattr(d, attr, arr.ctypes.data if len(arr) else None)
                    setattr(d, attr + "_bytes", len(arr))
        sd = _lib.SegmentDesc()
        nm = segment.name.encode()
        sd.name = nm
        sd.device = device
        sd.num_docs = segment.num_docs
        sd.num_columns = len(cols)
        sd.columns = descs
        handle = ctypes.c_uint64(0)
        _lib.check(lib.phip_segment_load(ctypes.byref(sd), ctypes.byref(handle)))
        self.handle = handle.value
        del keep
        # star-tree indexes load with their segment (ImmutableSegmentLoader -> StarTreeIndexReader): the star-tree
        # documents are resident like any segment's columns
        self.star_trees = list(getattr(segment, "star_trees", []) or [])
        self.star_segments = [GpuSegment(t.docs, device) for t in self.star_trees]

    # ---- host-side readers (DataSource equivalents) -----------------------------------------
    def column_metadata(self, column):
        return self.segment.columns[column].metadata

    def has_null_vector(self, column) -> bool:
        """The column has a null value vector, i.e. some doc is null (NullValueVectorCreator writes none otherwise;
        DataSource.getNullValueVector() != null)."""
        ci = self.segment.columns.get(column)
        return ci is not None and bool(getattr(ci, "null_vector", None))

    def has_column(self, column):
        return column in self.segment.columns

    def dictionary(self, column) -> Dictionary:
        d = self._dicts.get(column)
        if d is None:
            ci = self.segment.columns[column]
            m = ci.metadata
            d = Dictionary(ci.dictionary, m.data_type, m.cardinality, m.string_width)
            self._dicts[column] = d
        return d

    def inverted_bytes(self, column, dict_ids) -> int:
        """Bytes of the inverted-index bitmaps of `dict_ids` (the bytes an inverted leaf reads)."""
        if column not in self._inv_offsets:
            ci = self.segment.columns[column]
            card = ci.metadata.cardinality
            self._inv_offsets[column] = np.frombuffer(ci.inverted[:4 * (card + 1)], dtype=">u4").astype(np.int64)
        offs = self._inv_offsets[column]
        ids = np.asarray(dict_ids, dtype=np.int64)
        return int(np.sum(offs[ids + 1] - offs[ids])) if len(ids) else 0

    def sorted_doc_range(self, column, dict_id):
        """SortedIndexReaderImpl.getDocIds(dictId) (SortedIndexReaderImpl.java:114-116): inclusive pair."""
        p = self._sorted.get(column)
        if p is None:
            p = np.frombuffer(self.segment.columns[column].forward, dtype=">i4").astype(np.int64).reshape(-1, 2)
            self._sorted[column] = p
        return int(p[dict_id, 0]), int(p[dict_id, 1])

    def device_bytes(self) -> int:
        out = ctypes.c_uint64(0)
        _lib.check(_lib.load().phip_segment_device_bytes(self.handle, ctypes.byref(out)))
        return out.value

    def destroy(self):
        for s in getattr(self, "star_segments", []):
            s.destroy()
        self.star_segments = []
        if self.handle:
            _lib.check(_lib.load().phip_segment_unload(self.handle))
            self.handle = 0
