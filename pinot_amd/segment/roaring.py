"""Portable RoaringBitmap serialization (writer side).

The reference serializes inverted-index bitmaps with RoaringBitmap 1.3.0 (pom.xml:805-806; a
third-party jar, not vendored under /root/reference) via
``RoaringBitmapWriter.writer().get()`` + ``RoaringBitmap.serialize`` at
pinot-segment-local/.../creator/impl/inv/OffHeapBitmapInvertedIndexCreator.java:237-249 and
BitmapInvertedIndexWriter.java:78-85. This restates the public "portable" format
(RoaringFormatSpec) that RoaringBitmap writes:

  cookie   u32 LE: 12346 (no run containers) followed by u32 size,
           or 12347 | (size-1) << 16 followed by a run-flag bitset of ceil(size/8) bytes
  header   per container: u16 key (high 16 bits of the doc id), u16 cardinality-1
  offsets  per container u32 (present unless runs exist and size < 4)
  payload  array container  = card x u16 sorted low bits            (card <= 4096)
           bitmap container = 1024 x u64 LE words                   (card  > 4096)
           run container    = u16 nruns, nruns x (u16 start, u16 length-1)

The writer's default wizard run-compresses containers (``runOptimize``): a container is stored
as runs when that is strictly smaller than its array/bitmap form. Byte-level equality with the
Java library is unpinned (no golden bytes in the reference); decoders accept all
three container kinds.
"""
import struct

import numpy as np

SERIAL_COOKIE_NO_RUNCONTAINER = 12346
SERIAL_COOKIE = 12347
NO_OFFSET_THRESHOLD = 4
ARRAY_MAX = 4096


def _runs(lows: np.ndarray):
    """Runs of consecutive values in a sorted uint16 array -> (starts, lengths)."""
    if len(lows) == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    v = lows.astype(np.int64)
    brk = np.nonzero(np.diff(v) != 1)[0]
    starts = np.concatenate([[0], brk + 1])
    ends = np.concatenate([brk, [len(v) - 1]])
    return v[starts], v[ends] - v[starts] + 1


def serialize(doc_ids, run_optimize: bool = True) -> bytes:
    """Serialize a sorted, duplicate-free collection of non-negative doc ids."""
    docs = np.asarray(doc_ids, dtype=np.int64)
    if len(docs) > 1:
        assert np.all(np.diff(docs) > 0), "doc ids must be strictly increasing"
    keys = (docs >> 16).astype(np.int64)
    lows = (docs & 0xFFFF).astype(np.uint16)
    ukeys, starts = np.unique(keys, return_index=True)
    bounds = list(starts) + [len(docs)]
    containers = []  # (key, card, kind, payload bytes)
    for i, k in enumerate(ukeys):
        lo = lows[bounds[i]:bounds[i + 1]]
        card = len(lo)
        rs, rl = _runs(lo)
        nruns = len(rs)
        if card <= ARRAY_MAX:
            kind, size = "array", 2 * card
        else:
            kind, size = "bitmap", 8192
        if run_optimize and 2 + 4 * nruns < size:
            kind = "run"
        if kind == "array":
            payload = lo.astype("<u2").tobytes()
        elif kind == "bitmap":
            words = np.zeros(1024, dtype=np.uint64)
            np.bitwise_or.at(words, lo.astype(np.int64) >> 6,
                             np.left_shift(np.uint64(1), (lo.astype(np.uint64) & np.uint64(63))))
            payload = words.astype("<u8").tobytes()
        else:
            pairs = np.empty(2 * nruns, dtype="<u2")
            pairs[0::2] = rs
            pairs[1::2] = rl - 1
            payload = struct.pack("<H", nruns) + pairs.tobytes()
        containers.append((int(k), card, kind, payload))

    size = len(containers)
    has_run = any(c[2] == "run" for c in containers)
    out = bytearray()
    if has_run:
        out += struct.pack("<I", SERIAL_COOKIE | ((size - 1) << 16))
        flags = bytearray((size + 7) // 8)
        for i, c in enumerate(containers):
            if c[2] == "run":
                flags[i >> 3] |= 1 << (i & 7)
        out += flags
    else:
        out += struct.pack("<II", SERIAL_COOKIE_NO_RUNCONTAINER, size)
    for k, card, _, _ in containers:
        out += struct.pack("<HH", k, card - 1)
    if (not has_run) or size >= NO_OFFSET_THRESHOLD:
        off = len(out) + 4 * size
        for c in containers:
            out += struct.pack("<I", off)
            off += len(c[3])
    for c in containers:
        out += c[3]
    return bytes(out)
