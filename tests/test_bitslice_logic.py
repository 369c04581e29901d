"""CPU check of the bit-sliced comparison the filter kernel runs (filter.hip bs_range / bs_set over the planes of
load.hip bitslice_kernel), restated in numpy: planes of the tile-mask layout (bit 31-g of lane l = doc 64g + l),
gt/eq and lt/eq flags from the most significant plane down. Every (lo, hi, sides) of widths 1..6 and random ones
of 7..12 must give exactly lo <= x <= hi; a set of ids, the OR of the equalities."""
import numpy as np
import pytest


def planes(ids, b):
    """[b][64] u32 lane words of one 2048-doc tile: plane k = bit b-1-k."""
    ids = np.asarray(ids, dtype=np.uint32).reshape(32, 64)  # [g][lane]
    out = np.zeros((b, 64), dtype=np.uint32)
    for k in range(b):
        bit = (ids >> np.uint32(b - 1 - k)) & np.uint32(1)
        for g in range(32):
            out[k] |= bit[g] << np.uint32(31 - g)
    return out


def bs_range(pl, b, lo, hi, sides):
    full = np.uint32(0xFFFFFFFF)
    if sides == 3 and lo == hi:
        eq = np.full(64, full, dtype=np.uint32)
        for k in range(b):
            eq &= pl[k] if (lo >> (b - 1 - k)) & 1 else ~pl[k]
        return eq
    r = np.full(64, full, dtype=np.uint32)
    if sides & 1:
        gt, eq = np.zeros(64, np.uint32), np.full(64, full, np.uint32)
        for k in range(b):
            if (lo >> (b - 1 - k)) & 1:
                eq &= pl[k]
            else:
                gt |= eq & pl[k]
                eq &= ~pl[k]
        r &= gt | eq
    if sides & 2:
        lt, eq = np.zeros(64, np.uint32), np.full(64, full, np.uint32)
        for k in range(b):
            if (hi >> (b - 1 - k)) & 1:
                lt |= eq & ~pl[k]
                eq &= pl[k]
            else:
                eq &= ~pl[k]
        r &= lt | eq
    return r


def bs_set(pl, b, ids):
    r = np.zeros(64, np.uint32)
    for i in ids:
        eq = np.full(64, np.uint32(0xFFFFFFFF), np.uint32)
        for k in range(b):
            eq &= pl[k] if (i >> (b - 1 - k)) & 1 else ~pl[k]
        r |= eq
    return r


def lane_major(mask):
    m = np.asarray(mask, dtype=np.uint32).reshape(32, 64)
    out = np.zeros(64, np.uint32)
    for g in range(32):
        out |= m[g] << np.uint32(31 - g)
    return out


@pytest.mark.parametrize("b", range(1, 13))
def test_bitsliced_ranges(b):
    rng = np.random.default_rng(b)
    card = 1 << b
    ids = rng.integers(0, card, 2048)
    pl = planes(ids, b)
    cases = [(lo, hi) for lo in range(card) for hi in range(lo, card)] if b <= 6 else \
        [tuple(sorted(rng.integers(0, card, 2))) for _ in range(300)] + [(0, card - 1), (5, 5), (card - 1, card - 1)]
    for lo, hi in cases:
        lo, hi = int(lo), int(hi)
        sides = (1 if lo > 0 else 0) | (2 if hi < card - 1 else 0)
        want = lane_major((ids >= lo) & (ids <= hi))
        got = bs_range(pl, b, lo, hi, sides)
        assert np.array_equal(got, want), (b, lo, hi, sides)


@pytest.mark.parametrize("b", range(1, 7))
def test_bitsliced_sets(b):
    rng = np.random.default_rng(100 + b)
    card = 1 << b
    ids = rng.integers(0, card, 2048)
    pl = planes(ids, b)
    for _ in range(50):
        s = sorted(set(int(x) for x in rng.integers(0, card, rng.integers(1, 5))))
        assert np.array_equal(bs_set(pl, b, s), lane_major(np.isin(ids, s))), (b, s)


def bs_runs(pl, b, runs):
    """filter.hip bs_runs: OR over runs [a, b] of (gt | eq_a) & (lt | eq_b), both bounds tested in one plane pass."""
    full = np.uint32(0xFFFFFFFF)
    res = np.zeros(64, np.uint32)
    for a, z in runs:
        gt, lt = np.zeros(64, np.uint32), np.zeros(64, np.uint32)
        eqa, eqb = np.full(64, full, np.uint32), np.full(64, full, np.uint32)
        for k in range(b):
            if (a >> (b - 1 - k)) & 1:
                eqa &= pl[k]
            else:
                gt |= eqa & pl[k]
                eqa &= ~pl[k]
            if (z >> (b - 1 - k)) & 1:
                lt |= eqb & ~pl[k]
                eqb &= pl[k]
            else:
                eqb &= ~pl[k]
        res |= (gt | eqa) & (lt | eqb)
    return res


def id_runs(ids_in, card, exclusive):
    """runtime.cpp DICT_SET -> DevNode.bs_runs: the matching ids (complemented when exclusive) as runs."""
    member = np.zeros(card, bool)
    member[list(ids_in)] = True
    if exclusive:
        member = ~member
    runs, start = [], None
    for i in range(card + 1):
        on = i < card and member[i]
        if on and start is None:
            start = i
        elif not on and start is not None:
            runs.append((start, i - 1))
            start = None
    return runs


@pytest.mark.parametrize("b", [1, 3, 5, 8, 10, 12])
@pytest.mark.parametrize("exclusive", [False, True])
def test_bitsliced_id_runs(b, exclusive):
    """IN / NOT IN sets of at most 4 runs (OR of EQ predicates merged into one IN, SSB Q3.3's two cities, Q4.1's
    P_MFGR pair): the OR of plane ranges equals membership for every doc."""
    rng = np.random.default_rng(100 + b)
    card = max(2, (1 << b) - int(rng.integers(0, 2)))
    ids = rng.integers(0, card, 2048)
    pl = planes(ids, b)
    for _ in range(60):
        n = int(rng.integers(1, min(card, 9)))
        chosen = set(int(x) for x in rng.choice(card, n, replace=False))
        runs = id_runs(chosen, card, exclusive)
        if not runs or len(runs) > 4:
            continue
        want = lane_major(np.isin(ids, list(chosen)) != exclusive)
        assert np.array_equal(bs_runs(pl, b, runs), want), (b, sorted(chosen), exclusive, runs)
