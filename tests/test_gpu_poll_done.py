"""Aggregation-only executions without timing markers (PHIP_KERNEL_TIMING=0, how bench.py's timed steps and a server
run): the host takes the results when finalize_all_kernel has published the execution's sequence number in the plan's
mapped result area (PHIP_POLL_DONE, default on), not when the stream completes. The answers must be the oracle's on
every execution -- repeated executions of one plan (the sequence number advances, the device counters reset), several
plans interleaved, and concurrent client threads on separate execution lanes -- and equal to the stream-wait path's."""
import threading

import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.plan import GpuInstancePlanMaker
from pinot_amd.query.sql import parse
from tests.test_gpu_parity import _assert_intermediates_equal

pytestmark = pytest.mark.gpu

QUERIES = ["Q1.1", "Q1.2", "Q1.3"]
EXTRA = ["SELECT COUNT(*), SUM(LO_REVENUE), MIN(LO_DISCOUNT), MAX(LO_QUANTITY) FROM lineorder WHERE D_YEAR = 1995",
         "SELECT SUM(LO_EXTENDEDPRICE * LO_DISCOUNT), DISTINCTCOUNTHLL(LO_CUSTKEY) FROM lineorder WHERE LO_QUANTITY < 10",
         "SELECT COUNT(*) FROM lineorder WHERE D_YEAR > 2100"]  # (nothing matches: no kernel, no poll)


@pytest.fixture(scope="module")
def ssb(gpu_lib):
    from pinot_amd.engine.segment import GpuSegment
    from tools import ssb
    cols = sorted(set(ssb.columns_for(QUERIES)) | {"LO_REVENUE", "LO_QUANTITY", "LO_CUSTKEY"})
    raws = ssb.make_segments(1, cols, seed=13, segment_rows=1_500_000)
    segs = [GpuSegment(r) for r in raws]
    yield raws, segs
    for s in segs:
        s.destroy()


def _sqls():
    from tools import ssb
    return [ssb.SSB_QUERIES[q] for q in QUERIES] + EXTRA


def _check(qc, blk, raws):
    oblk, exact = executor.execute(qc, raws)
    assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
    _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, exact)


@pytest.mark.parametrize("poll", ["1", "0"])
def test_gpu_poll_done_sequential(poll, ssb, monkeypatch):
    monkeypatch.setenv("PHIP_KERNEL_TIMING", "0")
    monkeypatch.setenv("PHIP_POLL_DONE", poll)
    raws, segs = ssb
    qcs = [parse(s) for s in _sqls()]
    ops = [GpuInstancePlanMaker().make_instance_plan(qc, segs) for qc in qcs]
    first = [op.next_block() for op in ops]
    for qc, blk in zip(qcs, first):
        _check(qc, blk, raws)
        assert blk.filter_kernel_ms == 0.0 and blk.agg_kernel_ms == 0.0  # (no markers recorded)
    for _ in range(25):  # interleaved re-executions: every one equals the first
        for op, blk in zip(ops, first):
            again = op.next_block()
            assert again.stats.num_docs_scanned == blk.stats.num_docs_scanned
            for a, b in zip(again.results, blk.results):
                assert np.array_equal(np.asarray(a), np.asarray(b))
    for op in ops:
        op.close()


def test_gpu_poll_done_concurrent(ssb, monkeypatch):
    monkeypatch.setenv("PHIP_KERNEL_TIMING", "0")
    raws, segs = ssb
    qcs = [parse(s) for s in _sqls()]
    want = []
    for qc in qcs:
        oblk, exact = executor.execute(qc, raws)
        want.append((oblk, exact))
    errors = []

    def worker(i):
        try:
            op = GpuInstancePlanMaker().make_instance_plan(qcs[i % len(qcs)], segs)
            oblk, exact = want[i % len(qcs)]
            for _ in range(30):
                blk = op.next_block()
                assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
                _assert_intermediates_equal(qcs[i % len(qcs)].aggregations, blk.results, oblk.results, exact)
            op.close()
        except Exception as e:  # surfaced below
            errors.append((i, repr(e)))

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in threads), "a worker hung"
    assert not errors, errors[:3]
