"""The bit-sliced conjunctive filter path (ConjLeaf kind 2; filter.hip eval_conj_bs over the planes built at load by
load.hip bitslice_kernel): doc sets bit-exact against the oracle and against the packed-word path
(PHIP_NO_BITSLICE=1) for every column width it serves (1..12 bits), one- and two-sided ranges, single-value ranges,
ranges touching the dictionary ends, small IN sets, ragged last tiles, and ANDs with sorted-index doc ranges."""
import numpy as np
import pytest

from oracle import executor
from oracle.executor import OracleSegment
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType

pytestmark = pytest.mark.gpu

WIDTHS = list(range(1, 13))


def _segment(n, seed):
    rng = np.random.default_rng(seed)
    c = SegmentCreator(f"bs{seed}")
    for b in WIDTHS:
        card = (1 << b) if b < 12 else 3000  # a dictionary that does not fill its width too
        c.add_column(f"c{b}", DataType.INT, rng.integers(0, card, n).astype(np.int32) * 3 - 7)
    c.add_column("srt", DataType.INT, np.sort(rng.integers(0, 50, n)).astype(np.int32))
    c.add_column("m", DataType.LONG, rng.integers(-10 ** 9, 10 ** 9, n))
    return c.build()


def _filters():
    out = []
    for b in WIDTHS:
        card = (1 << b) if b < 12 else 3000
        vmax = (card - 1) * 3 - 7
        mid = (card // 2) * 3 - 7
        out += [f"c{b} = {mid}", f"c{b} BETWEEN -7 AND {mid}", f"c{b} >= {mid}", f"c{b} < {vmax}",
                f"c{b} > -7 AND c{b} <= {vmax}"]
    out += ["c3 BETWEEN 2 AND 11 AND c5 < 40 AND c9 >= 100", "c1 = -7 AND c12 > 4000 AND srt BETWEEN 10 AND 30",
            "c4 = 8 AND c6 BETWEEN 20 AND 80 AND c7 > 100 AND c8 < 300 AND c10 >= 1000 AND c11 < 5000",
            # IN sets of <= 4 ids over a dictionary of <= 64 (OR of equalities on the planes), and ones that are not
            "c3 IN (-4, 8, 14)", "c5 IN (-7, 2, 89) AND c2 = -1 AND c9 > 500", "c6 IN (-7, 182) AND c4 BETWEEN 5 AND 20",
            "c6 NOT IN (-7, 182) AND c4 > 5", "c6 IN (-7, -4, -1, 2, 5, 8) AND c3 < 8",
            # OR of EQ / IN / ranges on one column, merged into one IN (MergeEqInFilterOptimizer) and tested on the
            # planes as an OR of <= 4 id runs (ConjLeaf kind 4) over dictionaries of any size up to 12 bits
            "(c8 = 8 OR c8 = 80) AND c5 < 40", "(c12 = -4 OR c12 = 2000 OR c12 = 8990) AND c3 > 2",
            "(c10 BETWEEN 100 AND 200 OR c10 = 2000) AND c7 < 300", "c9 NOT IN (-7, 500) AND c6 > 50",
            "(c11 = 5 OR c11 IN (11, 14, 17)) AND c4 < 20", "c8 IN (-7, 2, 89, 300, 500) AND c2 = -1",
            "(c7 = -7 OR c7 = 374) AND (c9 = 20 OR c9 = 1000)"]
    return out


def _cases():
    out = []
    for f in _filters():
        out += [pytest.param(f, "default", id=f"{f}-default"), pytest.param(f, "no-runs", id=f"{f}-no-runs")]
        if " IN " in f:  # IN sets of <= 64-entry dictionaries as ids on the planes (opt-in PHIP_BS_SETS)
            out.append(pytest.param(f, "bs-sets", id=f"{f}-bs-sets"))
    return out


@pytest.fixture(scope="module")
def segs(gpu_lib):
    from pinot_amd.engine.segment import GpuSegment
    raws = [_segment(n, s) for n, s in ((5000, 1), (2048 * 3, 2), (70001, 3))]
    gs = [GpuSegment(r) for r in raws]
    yield raws, gs
    for g in gs:
        g.destroy()


@pytest.mark.parametrize("flt,mode", _cases())
def test_gpu_bitsliced_doc_sets(flt, mode, segs, monkeypatch):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from tests.test_gpu_parity import _assert_intermediates_equal, _words_from_mask
    raws, gs = segs
    if mode == "bs-sets":  # IN sets on the planes as id masks (opt-in: PHIP_BS_SETS, read when a plan is prepared)
        monkeypatch.setenv("PHIP_BS_SETS", "1")
        monkeypatch.setenv("PHIP_BS_RUNS", "0")
    elif mode == "no-runs":  # sets off the planes: the packed-word conjunction or the interpreter
        monkeypatch.setenv("PHIP_BS_RUNS", "0")
    qc = parse(f"SELECT COUNT(*), SUM(m) FROM t WHERE {flt}")
    for raw, g in zip(raws, gs):
        want = _words_from_mask(executor.eval_filter(OracleSegment(raw), qc.filter))
        for off in (False, True):
            if off:
                monkeypatch.setenv("PHIP_NO_BITSLICE", "1")
            else:
                monkeypatch.delenv("PHIP_NO_BITSLICE", raising=False)
            op = GpuInstancePlanMaker().make_instance_plan(qc, [g])
            assert np.array_equal(op.filter_bitmap(), want), (flt, raw.name, off)
            op.close()
    monkeypatch.delenv("PHIP_NO_BITSLICE", raising=False)
    op = GpuInstancePlanMaker().make_instance_plan(qc, gs)
    blk = op.next_block()
    op.close()
    oblk, ex = executor.execute(qc, raws)
    _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
