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
