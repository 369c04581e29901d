"""Host-side immutable dictionary (BaseImmutableDictionary / IntDictionary / StringDictionary).

pinot-segment-local/.../segment/index/readers/BaseImmutableDictionary.java:70-72 (immutable
dictionaries are sorted), :124-246 (indexOf / insertionIndexOf by binary search). Used by the
host-side predicate evaluators, exactly where the reference evaluates predicates on the host.
"""
import bisect

import numpy as np

from ..spi import DataType


class Dictionary:
    def __init__(self, data: bytes, data_type: DataType, cardinality: int, string_width: int = 0):
        self.data_type = data_type
        self.cardinality = cardinality
        if data_type == DataType.STRING:
            w = string_width
            self.values = [data[i * w:(i + 1) * w].rstrip(b"\0").decode("utf-8") for i in range(cardinality)]
        else:
            self.values = np.frombuffer(data, dtype=data_type.numpy_be, count=cardinality).astype(data_type.numpy)

    def __len__(self):
        return self.cardinality

    def get(self, dict_id):
        v = self.values[dict_id]
        return v if self.data_type == DataType.STRING else v.item()

    def _key(self, value):
        if self.data_type == DataType.STRING:
            return str(value)
        if self.data_type.is_integral:
            f = float(value)
            return int(value) if f == int(f) else f
        if self.data_type == DataType.FLOAT:
            return float(np.float32(float(value)))  # FloatDictionary: Float.parseFloat of the literal
        return float(value)

    def insertion_index_of(self, value) -> int:
        """Java binarySearch contract: index if found, else -(insertionPoint) - 1."""
        key = self._key(value)
        if self.data_type == DataType.STRING:
            i = bisect.bisect_left(self.values, key)
            if i < len(self.values) and self.values[i] == key:
                return i
            return -(i + 1)
        i = int(np.searchsorted(self.values, key, side="left"))
        if i < self.cardinality and self.values[i] == key:
            return i
        return -(i + 1)

    def index_of(self, value) -> int:
        i = self.insertion_index_of(value)
        return i if i >= 0 else -1
