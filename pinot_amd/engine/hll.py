"""Host-side HyperLogLog helpers for dictionary-answered DISTINCTCOUNTHLL.

NonScanBasedAggregationOperator.getDistinctCountHLLResult (pinot-core/.../operator/query/
NonScanBasedAggregationOperator.java) answers an unfiltered DISTINCTCOUNTHLL on a dictionary
column by offering every dictionary value; this is the vectorised clearspring stream-lib 2.9.8
MurmurHash.hash(Object) + HyperLogLog.offerHashed used for that (the GPU kernels use the same
(register, rho) per dict id, precomputed by libpinot_hip at first use).
"""
import numpy as np

from ..spi import DataType

_M = np.uint32(0x5BD1E995)


def _mix_long(data: np.ndarray) -> np.ndarray:
    d = data.astype(np.int64).view(np.uint64)
    with np.errstate(over="ignore"):
        lo = (d & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (d >> np.uint64(32)).astype(np.uint32)
        k = lo * _M
        k ^= k >> np.uint32(24)
        h = k * _M
        k = hi * _M
        k ^= k >> np.uint32(24)
        h = h * _M
        h ^= k * _M
        h ^= h >> np.uint32(13)
        h = h * _M
        h ^= h >> np.uint32(15)
    return h


def _hash_bytes(b: bytes) -> int:
    m = 0x5BD1E995
    n = len(b)
    h = (0xFFFFFFFF ^ n) & 0xFFFFFFFF  # seed -1
    n4 = n >> 2
    for i in range(n4):
        k = int.from_bytes(b[4 * i:4 * i + 4], "little")
        k = (k * m) & 0xFFFFFFFF
        k ^= k >> 24
        k = (k * m) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF
        h ^= k
    left = n - (n4 << 2)
    if left:
        def sb(x):
            return x - 256 if x > 127 else x
        if left >= 3:
            h ^= (sb(b[n - 3]) << 16) & 0xFFFFFFFF
        if left >= 2:
            h ^= (sb(b[n - 2]) << 8) & 0xFFFFFFFF
        h ^= sb(b[n - 1]) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= h >> 15
    return h


def hash_values(values, data_type: DataType) -> np.ndarray:
    """MurmurHash.hash(Object) of dictionary values, as uint32."""
    if data_type == DataType.STRING:
        return np.asarray([_hash_bytes(s.encode("utf-8")) for s in values], dtype=np.uint32)
    arr = np.asarray(values)
    if data_type in (DataType.INT, DataType.LONG):
        return _mix_long(arr.astype(np.int64))
    if data_type == DataType.FLOAT:
        return _mix_long(arr.astype(np.float32).view(np.int32).astype(np.int64))
    return _mix_long(arr.astype(np.float64).view(np.int64))


def register_rho(h: np.ndarray, log2m: int):
    """HyperLogLog.offerHashed of each hash: (register index, rho) per hash."""
    h = h.astype(np.uint32)
    j = (h >> np.uint32(32 - log2m)).astype(np.int64)
    w = (h << np.uint32(log2m)) | np.uint32((1 << (log2m - 1)) + 1)
    # rho = number of leading zeros of w (32-bit) + 1
    _, bitlen = np.frexp(w.astype(np.float64))  # exact bit length for w < 2^53
    rho = (32 - bitlen.astype(np.int64)) + 1
    return j, rho


def registers_of_hashes(h: np.ndarray, log2m: int) -> np.ndarray:
    """HyperLogLog.offerHashed over all hashes -> registers (uint8)."""
    j, rho = register_rho(h, log2m)
    regs = np.zeros(1 << log2m, dtype=np.uint8)
    np.maximum.at(regs, j, rho.astype(np.uint8))
    return regs
