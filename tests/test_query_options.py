"""Result-changing query options of the GPU plan maker (InstancePlanMakerImplV2.applyQueryOptions,
pinot-core/.../plan/maker/InstancePlanMakerImplV2.java:230-300). Host-only: the option resolution, the trim
arithmetic pinned by the reference's GroupByUtilsTest known answers, the oracle's segment-level trim, and the
combine checks of GpuGroupByCombineOperator driven by a stub operator (the GPU parity of the same options is
tests/test_gpu_query_options.py)."""
from types import SimpleNamespace

import pytest

from oracle import executor
from pinot_amd.engine.plan import (GpuGroupByCombineOperator, GpuInstancePlanMaker, GpuPlanWithCpuFallback,
                                   QueryOptionError, UnsupportedOnGpu, indexed_table_trim_threshold, table_capacity)
from pinot_amd.engine.results import ExecutionStatistics, GroupByResultsBlock
from pinot_amd.query.sql import parse
from pinot_amd.segment.creator import SegmentCreator
from pinot_amd.spi import DataType

INT_MAX = (1 << 31) - 1


def test_table_capacity_known_answers():
    """GroupByUtilsTest.testGetTableCapacity (pinot-core/src/test/.../util/GroupByUtilsTest.java:28-39)."""
    for limit, want in [(0, 5000), (1, 5000), (1000, 5000), (10000, 50000), (100000, 500000), (1000000, 5000000),
                        (10000000, 50000000), (100000000, 500000000), (1000000000, INT_MAX)]:
        assert table_capacity(limit, 5000) == want


def test_indexed_table_trim_threshold_known_answers():
    """GroupByUtilsTest.getIndexedTableTrimThreshold (:41-57)."""
    cases = [(5000, -1, INT_MAX), (5000, 0, INT_MAX), (5000, 10, 10000), (5000, 100, 10000), (5000, 1000, 10000),
             (5000, 10000, 10000), (5000, 100000, 100000), (5000, 1000000, 1000000), (5000, 10000000, 10000000),
             (5000, 100000000, 100000000), (5000, 1000000000, 1000000000), (5000, 1000000001, INT_MAX),
             (INT_MAX, 10, INT_MAX), (500000000, 10, 1000000000), (500000001, 10, INT_MAX)]
    for size, thr, want in cases:
        assert indexed_table_trim_threshold(size, thr) == want, (size, thr)


def test_apply_query_options_resolves_group_by_options():
    pm = GpuInstancePlanMaker(num_groups_limit=777, min_segment_group_trim_size=-1, group_trim_threshold=123456)
    q = pm.apply_query_options(parse("SELECT a, COUNT(*) FROM t GROUP BY a"))
    assert q.options == {"numGroupsLimit": "777", "minSegmentGroupTrimSize": "-1", "minServerGroupTrimSize": "5000",
                         "groupTrimThreshold": "123456"}
    q = pm.apply_query_options(parse("SET numGroupsLimit = 10; SET minSegmentGroupTrimSize = 50; "
                                     "SET groupTrimThreshold = 0; SET minServerGroupTrimSize = -1; "
                                     "SELECT a, COUNT(*) FROM t GROUP BY a"))
    assert (q.options["numGroupsLimit"], q.options["minSegmentGroupTrimSize"], q.options["groupTrimThreshold"],
            q.options["minServerGroupTrimSize"]) == ("10", "50", "0", "-1")
    # keys resolve case-insensitively (QueryOptionsUtils.resolveCaseInsensitiveOptions)
    q = pm.apply_query_options(parse("SET NUMGROUPSLIMIT = 3; SELECT a, COUNT(*) FROM t GROUP BY a"))
    assert q.options["numGroupsLimit"] == "3"
    # aggregation-only queries never read the group-by options (applyQueryOptions :230)
    q0 = parse("SET numGroupsLimit = 0; SELECT COUNT(*) FROM t")
    assert pm.apply_query_options(q0) is q0


@pytest.mark.parametrize("opt", ["numGroupsLimit = 0", "numGroupsLimit = -5", "numGroupsLimit = abc",
                                 "numGroupsLimit = 3000000000", "minSegmentGroupTrimSize = 1.5",
                                 "groupTrimThreshold = ten"])
def test_malformed_options_are_bad_requests(opt):
    with pytest.raises(QueryOptionError):
        GpuInstancePlanMaker().apply_query_options(parse(f"SET {opt}; SELECT a, COUNT(*) FROM t GROUP BY a"))


def test_server_config_threshold_must_be_positive():
    with pytest.raises(ValueError):
        GpuInstancePlanMaker(group_trim_threshold=0)


class _CpuMaker:
    def __init__(self):
        self.calls = []

    def make_instance_plan(self, query, segments):
        self.calls.append(query)
        return SimpleNamespace(next_block=lambda: "cpu-block", close=lambda: None)


@pytest.mark.parametrize("opt", ["serverReturnFinalResult = true", "serverReturnFinalResultKeyUnpartitioned = true"])
def test_options_outside_the_gpu_semantics_fall_back(opt):
    sql = f"SET {opt}; SELECT a, COUNT(*) FROM t GROUP BY a"
    with pytest.raises(UnsupportedOnGpu):
        GpuInstancePlanMaker().make_instance_plan(sql, [])
    cpu = _CpuMaker()
    assert GpuInstancePlanMaker(cpu_plan_maker=cpu).make_instance_plan(sql, []).next_block() == "cpu-block"
    assert len(cpu.calls) == 1


def test_null_handling_false_stays_on_the_gpu_path():
    q = GpuInstancePlanMaker().apply_query_options(parse("SET enableNullHandling = false; SELECT COUNT(*) FROM t"))
    assert q.options["enableNullHandling"] == "false"


# ---------------------------------------------------------------------------------------------- oracle
def test_oracle_segment_trim():
    """Each segment keeps its top getTableCapacity(limit, minSegmentGroupTrimSize) groups before the merge: a key
    that ranks high in one segment and low in another keeps only the first segment's share."""
    raws = []
    for s, rows in enumerate([[(k, 100 - k) for k in range(20)], [(k, k + 1) for k in range(20)]]):
        c = SegmentCreator(f"st{s}")
        c.add_column("k", DataType.INT, [r[0] for r in rows])
        c.add_column("m", DataType.LONG, [r[1] for r in rows])
        raws.append(c.build())
    qc = parse("SELECT k, SUM(m) FROM t GROUP BY k ORDER BY SUM(m) DESC LIMIT 1")
    full, _ = executor.execute(qc, raws)
    assert len(full.groups) == 20 and full.groups[(0,)][0] == 101
    trimmed, ex = executor.execute(qc, raws, min_segment_group_trim_size=5)  # trimSize max(5 x 1, 5) = 5
    # segment 0 keeps k = 0..4 (100..96), segment 1 keeps k = 15..19 (16..20)
    assert sorted(trimmed.groups) == [(k,) for k in list(range(5)) + list(range(15, 20))]
    assert ex[(0,)][0] == 100 and ex[(19,)][0] == 20
    same, _ = executor.execute(qc, raws, min_segment_group_trim_size=20)  # no segment holds more than 20 groups
    assert same.groups == full.groups


# ---------------------------------------------------------------------------------------------- combine checks
class _Seg:
    def __init__(self, n, card):
        self.num_docs = n
        self.card = card

    def column_metadata(self, c):
        return SimpleNamespace(cardinality=self.card, has_dictionary=True)


class _Op:
    def __init__(self, segments, matched, groups=None):
        self.segments = segments
        self.matched = matched
        self.groups = groups or {}
        self.runs = 0
        self.segment_trim = None

    def next_block(self):
        self.runs += 1
        b = GroupByResultsBlock([], [], dict(self.groups), ExecutionStatistics(), False)
        b.segment_docs_matched = list(self.matched)
        return b

    def close(self):
        pass


def _resolved(sql, **kw):
    return GpuInstancePlanMaker(**kw).apply_query_options(parse(sql))


def test_combine_checks_pass_through_when_no_trim_can_fire():
    q = _resolved("SET minSegmentGroupTrimSize = 100; SELECT k, COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) LIMIT 5")
    assert GpuGroupByCombineOperator.needed(q)
    segs = [_Seg(1000, 90), _Seg(1000, 500)]
    inner = _Op(segs, [1000, 60])  # bounds min(1000, 90) = 90 and min(60, 500) = 60: both <= trimSize 100
    op = GpuGroupByCombineOperator(q, inner, lambda s: pytest.fail("no per-segment plan expected"))
    op.next_block()
    assert inner.runs == 1


def test_combine_runs_per_segment_when_a_segment_trims():
    q = _resolved("SET minSegmentGroupTrimSize = 100; SELECT k, COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) LIMIT 5")
    segs = [_Seg(1000, 90), _Seg(1000, 500)]
    inner = _Op(segs, [1000, 200])  # segment 1 may hold 200 > 100 groups
    made = []

    def make(s):
        o = _Op(s, [0], {(len(made),): [1]})
        made.append(o)
        return o

    op = GpuGroupByCombineOperator(q, inner, make)
    op.aggs = []
    blk = op.next_block()
    assert len(made) == 2 and all(o.segment_trim == 100 for o in made)
    assert blk.segment_trimmed


def test_combine_threshold_refuses_multi_segment_resizes():
    # trimSize max(5 x 10, 5000) = 5000 -> threshold max(10, 2 x 5000) = 10000
    sql = "SET groupTrimThreshold = 10; SELECT k, COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) LIMIT 10"
    q = _resolved(sql)
    assert GpuGroupByCombineOperator.needed(q)
    segs = [_Seg(100000, 8000), _Seg(100000, 8000)]
    op = GpuGroupByCombineOperator(q, _Op(segs, [9000, 9000]), None)
    with pytest.raises(UnsupportedOnGpu):
        op.next_block()
    # one segment with records: every group is upserted once, resizes keep the exact top trimSize
    GpuGroupByCombineOperator(q, _Op(segs, [100000, 0]), None).next_block()
    # under the threshold
    GpuGroupByCombineOperator(q, _Op(segs, [4000, 4000]), None).next_block()
    # the default threshold (10^6) and no ORDER BY: nothing to check
    assert not GpuGroupByCombineOperator.needed(_resolved("SELECT k, COUNT(*) FROM t GROUP BY k LIMIT 10"))
    assert not GpuGroupByCombineOperator.needed(_resolved("SET groupTrimThreshold = -1; " + sql.split("; ")[1]))


def test_execution_time_refusal_goes_to_the_cpu_plan():
    sql = "SET groupTrimThreshold = 10; SELECT k, COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) LIMIT 10"
    q = _resolved(sql)
    segs = [_Seg(100000, 8000), _Seg(100000, 8000)]
    cpu = _CpuMaker()
    op = GpuPlanWithCpuFallback(GpuGroupByCombineOperator(q, _Op(segs, [9000, 9000]), None), cpu, q, segs)
    assert op.next_block() == "cpu-block" and cpu.calls == [q]


def test_combine_threshold_counts_distinct_keys():
    """ConcurrentIndexedTable resizes on the number of DISTINCT keys in its map (ConcurrentIndexedTable.java:63-67):
    per-segment bounds that sum past the threshold do not refuse the query when the merged result (untrimmed) or the
    query-global key space holds fewer keys than the threshold."""
    sql = "SET groupTrimThreshold = 10; SELECT k, COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) LIMIT 10"
    q = _resolved(sql)
    segs = [_Seg(100000, 8000), _Seg(100000, 8000)]

    class _Untrimmed(_Op):
        def __init__(self, segments, matched, groups, trimmed, key_space):
            super().__init__(segments, matched, groups)
            self.trimmed, self.key_space = trimmed, key_space

        def next_block(self):
            b = super().next_block()
            b.num_groups_trimmed, b.key_space = self.trimmed, self.key_space
            return b

    few = {(k,): [1] for k in range(9000)}  # 9000 distinct keys < threshold 10000, bounds sum to 18000
    GpuGroupByCombineOperator(q, _Untrimmed(segs, [9000, 9000], few, False, 20000), None).next_block()
    # trimmed block: the distinct count is unknown, the key space (8000 < 10000) still bounds it
    GpuGroupByCombineOperator(q, _Untrimmed(segs, [9000, 9000], few, True, 8000), None).next_block()
    with pytest.raises(UnsupportedOnGpu):  # trimmed, key space 20000: the combine may resize
        GpuGroupByCombineOperator(q, _Untrimmed(segs, [9000, 9000], few, True, 20000), None).next_block()
    many = {(k,): [1] for k in range(12000)}
    with pytest.raises(UnsupportedOnGpu):  # 12000 distinct keys >= 10000
        GpuGroupByCombineOperator(q, _Untrimmed(segs, [9000, 9000], many, False, 20000), None).next_block()


def test_timeout_option_validated_and_applied():
    """timeoutMs is QueryOptionsUtils.getTimeoutMs (a positive long); a query whose end time passed raises
    QueryTimeoutError before it runs, and one with time left runs its operator."""
    import time as _time

    from pinot_amd.engine import plan as _plan
    from pinot_amd.engine.plan import QueryOptionError, QueryTimeoutError
    for bad in ("0", "-5", "abc", "1.5"):
        with pytest.raises(QueryOptionError):
            GpuInstancePlanMaker().apply_query_options(parse(f"SET timeoutMs = {bad}; SELECT COUNT(*) FROM t"))

    class _Inner:
        def next_block(self):
            _plan.check_deadline("inside")
            return "ran"

        def close(self):
            pass

    assert _plan._DeadlineOperator(_Inner(), 10_000).next_block() == "ran"
    slow = _plan._DeadlineOperator(type("S", (), {"next_block": lambda s: (_time.sleep(0.02), _plan.check_deadline(
        "after sleeping"))[1], "close": lambda s: None})(), 1)
    with pytest.raises(QueryTimeoutError):
        slow.next_block()
    _plan.check_deadline("outside any query")  # no end time: no-op
