"""Concurrent queries (SURVEY.md §8b threading contract): the server's worker threads call the library at
once (BaseCombineOperator.java:87-92, default 2 x cores workers ResourceManager.java:59-60). Every execution
takes its own lane (stream + scratch) of the device, so queries overlap instead of serialising on a device
lock; results must stay bit-exact vs the oracle under any interleaving."""
import threading

import numpy as np
import pytest

from oracle import executor
from pinot_amd.query.sql import parse
from tests import fixtures

QUERIES = [
    "SELECT COUNT(*), SUM(column1), MIN(column3), MAX(column9) FROM testTable WHERE column1 > 100000000",
    "SELECT column9, COUNT(*), SUM(column3) FROM testTable WHERE column11 IN ('t', 'P') GROUP BY column9 LIMIT 100000",
    "SELECT DISTINCTCOUNTHLL(column1), COUNT(*) FROM testTable WHERE column6 <> 296467636 OR column9 < 50000",
    "SELECT column11, column12, SUM(column1), MAX(column7) FROM testTable GROUP BY column11, column12 LIMIT 100000",
    "SELECT column1, COUNT(*) FROM testTable GROUP BY column1 ORDER BY COUNT(*) DESC, column1 LIMIT 10",
    "SELECT SUM(column3), COUNT(*) FROM testTable WHERE NOT column11 IN ('t', 'P') AND daysSinceEpoch <> 126164076",
]


@pytest.mark.gpu
def test_gpu_concurrent_mixed_queries(gpu_lib):
    from pinot_amd.engine.plan import GpuInstancePlanMaker
    from pinot_amd.engine.segment import GpuSegment
    from tests.test_gpu_limits import _check
    from tests.test_gpu_parity import _assert_intermediates_equal
    seg = GpuSegment(fixtures.segment_for("test_data_sv"))
    try:
        want = {q: executor.execute(parse(q), [seg.segment, seg.segment]) for q in QUERIES}
        errors = []

        def worker(tid):
            try:
                rng = np.random.default_rng(tid)
                for i in range(24):
                    q = QUERIES[int(rng.integers(0, len(QUERIES)))]
                    qc = parse(q)
                    op = GpuInstancePlanMaker(num_groups_limit=10 ** 9 if tid % 2 else 100_000).make_instance_plan(
                        qc, [seg, seg])
                    blk = op.next_block()
                    if i % 3 == 0:  # a prepared plan re-executed
                        blk = op.next_block()
                    op.close()
                    oblk, ex = want[q]
                    if qc.group_by:
                        if getattr(blk, "num_groups_trimmed", False):
                            from pinot_amd.engine.reduce import trim_groups
                            oblk = trim_groups(qc, oblk)
                        _check(qc, blk, oblk, ex)
                    else:
                        assert blk.stats.num_docs_scanned == oblk.stats.num_docs_scanned
                        _assert_intermediates_equal(qc.aggregations, blk.results, oblk.results, ex)
            except Exception as e:  # noqa: BLE001
                errors.append((tid, repr(e)))

        threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in threads), "a worker hung"
        assert not errors, errors[:3]
    finally:
        seg.destroy()
