"""Pin the CPU oracle against the reference's own known answers (CPU only).

Segments are rebuilt from the committed fixtures; queries and expected rows/stats are transcribed in
tests/golden/expected.json with the reference file:line of each assertion. The harness mirrors
BaseQueriesTest.getBrokerResponse: the server runs over two copies of the segment and the response
is reduced as OFFLINE + REALTIME (x4 for COUNT/SUM).
"""
import numpy as np
import pytest

from oracle import executor
from pinot_amd.engine.reduce import reduce_blocks
from pinot_amd.query.sql import parse
from tests import fixtures

CASES = fixtures.expected()["queries"]


def _oracle_broker(query, seg, num_segments):
    qc = parse(query)
    block, _ = executor.execute(qc, [seg] * num_segments)
    return reduce_blocks(qc, [block, block])


@pytest.mark.parametrize("case", CASES, ids=[f"{c['ref'].split('/')[-1]}|{c['query'][:60]}" for c in CASES])
def test_oracle_known_answers(case):
    seg = fixtures.segment_for(case["data"])
    if case["data"] == "test_data_sv":
        rt = _oracle_broker(case["query"], seg, 2)
        # the non-scan shortcut (dictionary-answered MIN/MAX/HLL) is a plan choice, not in the oracle
        docs, post, total = case["stats"]
        assert rt.stats.num_docs_scanned == docs
        assert rt.stats.num_total_docs == total
        if post != 0:
            assert rt.stats.num_entries_scanned_post_filter == post
    else:
        # FastFilteredCountTest asserts the single-segment operator result
        qc = parse(case["query"])
        block, _ = executor.execute(qc, [seg])
        rt = reduce_blocks(qc, [block])
    assert fixtures.rows_match(rt.rows, case["rows"]), (rt.rows, case["rows"])


@pytest.mark.parametrize("case", fixtures.expected()["docsets"], ids=lambda c: c["ref"].split("/")[-1])
@pytest.mark.parametrize("prefix", ["s", "t"])
def test_oracle_docset_kats(case, prefix):
    seg = fixtures.docset_segment(case["sets"], case["num_docs"])
    q = parse("SELECT COUNT(*) FROM t WHERE " + fixtures.docset_filter(case["op"], len(case["sets"]), prefix))
    mask = executor.filter_mask(q, seg)
    assert np.nonzero(mask)[0].tolist() == case["expected"]
