"""CPU: the bench's cpu_baseline restatement (oracle/cpu_scan.c, OpenMP) answers the headline queries exactly
like the oracle on both SSB layouts (matched docs and the SUM, which is integral here)."""
import pytest

from oracle import cpu_baseline, executor
from pinot_amd.query.sql import parse


@pytest.mark.parametrize("layout", ["unsorted", "sorted"])
def test_cpu_baseline_matches_oracle(layout):
    from tools import ssb
    qs = ["Q1.1", "Q1.2", "Q1.3"]
    raws = ssb.make_segments(1, ssb.columns_for(qs), seed=11, segment_rows=1_500_000, layout=layout)
    for q in qs:
        qc = parse(ssb.SSB_QUERIES[q])
        ob, ex = executor.execute(qc, raws)
        total, matched = cpu_baseline.Prepared(qc, raws).run(4)
        assert matched == ob.stats.num_docs_scanned
        assert total == ob.results[0] == float(ex[0])
    v, threads, reps, el, res = cpu_baseline.time_queries([parse(ssb.SSB_QUERIES[q]) for q in qs], raws, 2, 0.1, 2)
    assert v > 0 and threads == 2 and reps >= 1


GROUP_BY_QUERIES = ["Q2.1", "Q2.2", "Q2.3", "Q3.1", "Q3.2", "Q3.3", "Q3.4", "Q4.1", "Q4.2", "Q4.3", "C5"]


@pytest.mark.parametrize("layout", ["unsorted", "sorted"])
def test_cpu_group_by_matches_oracle(layout):
    """oracle/cpu_scan.c's group-by (bench.py's C3 / C5 parity check and group-by cpu_baseline) against the oracle
    executor: the same group set, exact SUMs, HLL registers and numDocsScanned, on both layouts."""
    import numpy as np

    from tools import ssb
    raws = ssb.make_segments(1, ssb.columns_for(GROUP_BY_QUERIES), seed=7, segment_rows=1_500_000, layout=layout)
    for q in GROUP_BY_QUERIES:
        qc = parse(ssb.SSB_QUERIES[q])
        ob, ex = executor.execute(qc, raws)
        p = cpu_baseline.PreparedGroupBy(qc, raws)
        out = p.run(3)
        assert out[3] == ob.stats.num_docs_scanned, q
        got = p.groups(out)
        assert set(got) == set(ob.groups), q
        assert len(got) > 0, q
        si, hi = p.sum_agg, p.hll_agg
        for k, (s, c, regs) in got.items():
            assert s == ex[k][si], (q, k)
            if hi is not None:
                assert np.array_equal(regs, ob.groups[k][hi]), (q, k)
    v, threads, reps, el = cpu_baseline.time_group_by([parse(ssb.SSB_QUERIES[q]) for q in ("Q2.1", "C5")], raws, 2,
                                                      0.1, 2)
    assert v > 0 and threads == 2 and reps >= 1
