"""Segment creation (host side): the native inverted-index writer (pinot_amd/segment/invidx.c) must
produce exactly the bytes of the Python restatement of BitmapInvertedIndexWriter + RoaringBitmap's
portable format (pinot_amd/segment/roaring.py), and both must decode back to the doc ids."""
import numpy as np
import pytest

from oracle import executor  # noqa: F401  (oracle package importable: decode helpers)
from pinot_amd.segment import creator, roaring


def _decode_index(blob: bytes, card: int):
    """Independent decode of the (card+1) BE offsets + portable Roaring bitmaps -> list of doc arrays."""
    offs = np.frombuffer(blob[:4 * (card + 1)], dtype=">u4").astype(np.int64)
    out = []
    for d in range(card):
        out.append(_decode_roaring(blob[offs[d]:offs[d + 1]]))
    return out


def _decode_roaring(b: bytes) -> np.ndarray:
    cookie = int.from_bytes(b[0:4], "little")
    if cookie & 0xFFFF == roaring.SERIAL_COOKIE:
        size = (cookie >> 16) + 1
        flags = b[4:4 + (size + 7) // 8]
        pos = 4 + (size + 7) // 8
        runs = [(flags[i >> 3] >> (i & 7)) & 1 for i in range(size)]
    else:
        assert cookie == roaring.SERIAL_COOKIE_NO_RUNCONTAINER
        size = int.from_bytes(b[4:8], "little")
        pos = 8
        runs = [0] * size
    hdr = np.frombuffer(b[pos:pos + 4 * size], dtype="<u2").reshape(-1, 2)
    pos += 4 * size
    if not any(runs) or size >= roaring.NO_OFFSET_THRESHOLD:
        pos += 4 * size
    docs = []
    for i in range(size):
        key, card = int(hdr[i, 0]), int(hdr[i, 1]) + 1
        if runs[i]:
            n = int.from_bytes(b[pos:pos + 2], "little")
            pr = np.frombuffer(b[pos + 2:pos + 2 + 4 * n], dtype="<u2").reshape(-1, 2).astype(np.int64)
            pos += 2 + 4 * n
            lows = np.concatenate([np.arange(s, s + l + 1) for s, l in pr]) if n else np.zeros(0, np.int64)
        elif card <= roaring.ARRAY_MAX:
            lows = np.frombuffer(b[pos:pos + 2 * card], dtype="<u2").astype(np.int64)
            pos += 2 * card
        else:
            words = np.frombuffer(b[pos:pos + 8192], dtype="<u8")
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")
            lows = np.nonzero(bits)[0]
            pos += 8192
        docs.append((key << 16) + lows)
    return np.concatenate(docs) if docs else np.zeros(0, np.int64)


CASES = [
    ("uniform_small_card", 1, 200_000, 7),
    ("uniform_mid_card", 2, 150_000, 1000),
    ("clustered_runs", 3, 300_000, 12),
    ("skewed_exp", 4, 200_000, 0),
    ("single_value", 5, 70_000, 1),
    ("tiny", 6, 3, 3),
]


@pytest.mark.parametrize("name,seed,n,card", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("run_optimize", [True, False])
def test_native_inverted_index_bytes_match_python(name, seed, n, card, run_optimize):
    rng = np.random.default_rng(seed)
    if name == "clustered_runs":
        ids = np.repeat(rng.integers(0, card, n // 1000), 1000)[:n]
        ids[rng.integers(0, len(ids), 500)] = rng.integers(0, card, 500)
    elif name == "skewed_exp":
        v = (-np.log(rng.random(n)) / 0.01).astype(np.int64)
        _, ids = np.unique(v, return_inverse=True)
        card = int(ids.max()) + 1
    elif name == "tiny":
        ids = np.array([2, 0, 2])
    else:
        ids = rng.integers(0, card, n)
    ids = ids.astype(np.int32)
    card = max(card, int(ids.max()) + 1)
    nat = creator.inverted_index_bytes(ids, card, run_optimize, native=True)
    py = creator.inverted_index_bytes(ids, card, run_optimize, native=False)
    assert nat == py
    if n <= 200_000:
        dec = _decode_index(nat, card)
        for d in range(card):
            assert np.array_equal(dec[d], np.nonzero(ids == d)[0])


def test_native_inverted_index_rejects_bad_ids():
    with pytest.raises(ValueError):
        creator.inverted_index_bytes(np.array([0, 5], dtype=np.int32), 3)


@pytest.mark.parametrize("bits", [1, 2, 3, 5, 7, 8, 13, 16, 21, 31])
@pytest.mark.parametrize("n", [1, 7, 95, 4097])
def test_native_pack_bits_matches_numpy(bits, n):
    rng = np.random.default_rng(bits * 1000 + n)
    ids = rng.integers(0, 1 << bits, n).astype(np.uint32)
    assert creator.pack_bits(ids, bits, native=True) == creator.pack_bits(ids, bits, native=False)
