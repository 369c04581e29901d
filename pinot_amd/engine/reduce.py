"""Broker-side reduce of server results blocks into a result table.

Mirrors what the reference tests observe through BrokerReduceService (pinot-core/.../query/reduce/):
AggregationDataTableReducer / GroupByDataTableReducer merge intermediates across server responses
(AggregationFunction.merge), extract final results (extractFinalResult), apply ORDER BY / LIMIT, and
name columns by alias or by the canonical expression. ``broker_response`` mirrors
BaseQueriesTest.getBrokerResponse (pinot-core/src/test/java/org/apache/pinot/queries/BaseQueriesTest.java:207-247):
the server response is reduced as if it came from an OFFLINE and a REALTIME server.
"""
import math
from dataclasses import dataclass, field
from typing import List

import numpy as np

from ..query.context import FilterClause, Function, Identifier, Literal, QueryContext, SUPPORTED_AGGREGATIONS
from ..spi import DEFAULT_HYPERLOGLOG_LOG2M
from .results import AggregationResultsBlock, ExecutionStatistics, GroupByResultsBlock, merge_intermediate


def hll_cardinality(regs: np.ndarray) -> int:
    """clearspring HyperLogLog.cardinality() (stream-lib 2.9.8; DistinctCountHLLAggregationFunction.java:362-365)."""
    m = len(regs)
    log2m = m.bit_length() - 1
    if log2m == 4:
        alpha_mm = 0.673 * m * m
    elif log2m == 5:
        alpha_mm = 0.697 * m * m
    elif log2m == 6:
        alpha_mm = 0.709 * m * m
    else:
        alpha_mm = (0.7213 / (1 + 1.079 / m)) * m * m
    s = 0.0
    zeros = 0
    for r in regs.tolist():
        s += 1.0 / (1 << r)
        zeros += r == 0
    est = alpha_mm * (1.0 / s)
    if est <= 2.5 * m:
        if zeros == 0:  # linearCounting(m, 0) = m * log(m / 0.0) = +Infinity; Math.round(+Infinity) = Long.MAX_VALUE
            return 2 ** 63 - 1
        return int(math.floor(m * math.log(m / zeros) + 0.5))
    return int(math.floor(est + 0.5))


def order_key(ob, value):
    """Sort key of one ORDER BY expression over records (used with reverse = DESC): a null (None) value -- a null
    group key or a null aggregation result under enableNullHandling -- goes last or first as ob.is_nulls_last says
    (OrderByExpressionContext.isNullsLast; the comparator of TableResizer / the broker's reduce)."""
    high = ob.is_nulls_last != (not ob.ascending)  # where nulls sit before the DESC reversal

    def key(rec):
        v = value(rec)
        return ((v is None) if high else (v is not None), v)
    return key


def final_result(function: str, v):
    """AggregationFunction.extractFinalResult (a null intermediate stays null)."""
    if v is None:
        return None
    if function == "count":
        return int(v)
    if function == "sum":
        return float(v)
    if function in ("min", "max"):
        return float(v)
    if function == "avg":
        s, c = v
        return float(s) / c if c else float("-inf")
    if function == "minmaxrange":
        return float(v[1]) - float(v[0])
    if function in ("distinctcounthll", "distinctcountrawhll"):
        return hll_cardinality(v)
    raise NotImplementedError(function)


@dataclass
class ResultTable:
    columns: List[str]
    rows: List[list]
    stats: ExecutionStatistics = field(default_factory=ExecutionStatistics)
    num_groups_limit_reached: bool = False


def _agg_index(query: QueryContext, expr):
    flt = None
    if isinstance(expr, FilterClause):
        expr, flt = expr.function, expr.filter
    if not isinstance(expr, Function):
        return None
    for i, a in enumerate(query.aggregations):  # exact argument first (COUNT(col) under enableNullHandling)
        if expr.name == a.function and a.filter == flt and expr.args and expr.args[0] == a.argument:
            return i
    for i, a in enumerate(query.aggregations):
        if expr.name == a.function == "count" and a.filter == flt and a.argument is None:
            return i
    return None


def _column_name(expr, alias, query=None):
    if alias:
        return alias
    if isinstance(expr, Function) and expr.name == "count":
        i = _agg_index(query, expr) if query is not None else None
        if i is not None and query.aggregations[i].argument is not None:
            return f"count({query.aggregations[i].argument})"  # (enableNullHandling: CountAggregationFunction.java:64-66)
        return "count(*)"
    return str(expr)


def reduce_blocks(query: QueryContext, blocks) -> ResultTable:
    stats = ExecutionStatistics()
    for b in blocks:
        stats.merge(b.stats)
    if query.is_selection:
        return _reduce_selection(query, blocks, stats)
    names = [_column_name(e, a, query) for e, a in query.select]
    if not query.group_by:
        merged = None
        for b in blocks:
            if merged is None:
                merged = list(b.results)
            else:
                merged = [merge_intermediate(a.function, x, y) for a, x, y in zip(query.aggregations, merged, b.results)]
        finals = [final_result(a.function, v) for a, v in zip(query.aggregations, merged)]
        row = []
        for e, _ in query.select:
            i = _agg_index(query, e)
            if i is None:
                raise NotImplementedError(f"post-aggregation expression {e}")
            row.append(finals[i])
        return ResultTable(names, [row], stats)

    groups = {}
    limit_reached = False
    for b in blocks:
        limit_reached |= b.num_groups_limit_reached
        for k, v in b.groups.items():
            if k in groups:
                groups[k] = [merge_intermediate(a.function, x, y) for a, x, y in zip(query.aggregations, groups[k], v)]
            else:
                groups[k] = list(v)
    gb_index = {str(e): i for i, e in enumerate(query.group_by)}
    records = []
    for k, v in groups.items():
        finals = [final_result(a.function, x) for a, x in zip(query.aggregations, v)]
        records.append((k, finals))

    def value_of(expr, rec):
        k, finals = rec
        if str(expr) in gb_index:
            return k[gb_index[str(expr)]]
        i = _agg_index(query, expr)
        if i is None:
            raise NotImplementedError(f"order-by/select expression {expr}")
        return finals[i]

    for ob in reversed(query.order_by):
        records.sort(key=order_key(ob, lambda rec: value_of(ob.expression, rec)), reverse=not ob.ascending)
    records = records[:query.limit]
    rows = [[value_of(e, rec) for e, _ in query.select] for rec in records]
    return ResultTable(names, rows, stats, limit_reached)


def _reduce_selection(query: QueryContext, blocks, stats) -> ResultTable:
    """SelectionOnlyReducer (pinot-core/.../query/reduce/SelectionOnlyReducer): the servers' rows concatenated up to
    LIMIT, each row mapped to the select list (SelectionOperatorUtils.getSelectionColumns: SELECT * keeps the data
    schema's columns; duplicated expressions read the same schema column)."""
    schema = next((b for b in blocks if b.column_names), None)
    if schema is None:
        return ResultTable([], [], stats)
    index = {n: i for i, n in enumerate(schema.column_names)}
    star = len(query.select) == 1 and str(query.select[0][0]) == "*"
    if star:
        names, picks = list(schema.column_names), list(range(len(schema.column_names)))
    else:
        names = [_column_name(e, a, query) for e, a in query.select]
        picks = [index[str(e)] for e, _ in query.select]
    rows = []
    for b in blocks:
        for r in b.rows:
            if len(rows) >= query.limit:
                break
            rows.append([r[i] for i in picks])
    return ResultTable(names, rows, stats)


def trim_size(query: QueryContext, min_trim=None) -> int:
    """GroupByUtils.getTableCapacity(limit, minServerGroupTrimSize) (GroupByUtils.java:55-58,96-140); 0 = no trim.
    ``min_trim``: a segment's minSegmentGroupTrimSize instead (GroupByOperator.java:118-133)."""
    if min_trim is None:
        min_trim = int(query.options.get("minServerGroupTrimSize", 5000))
    if not query.group_by or not query.order_by or min_trim <= 0:
        return 0
    return min(max(5 * int(query.limit), min_trim), 2 ** 31 - 1)


def trim_groups(query: QueryContext, block, min_trim=None):
    """Server-level trim on the host (IndexedTable.finish -> TableResizer.getTopRecords): the merged
    group-by block of a multi-GPU server keeps its top trimSize groups by the full ORDER BY. Ties at the
    boundary keep the smallest keys (the reference's choice is heap-order dependent). ``min_trim``: the
    segment-level trim of one segment's block (minSegmentGroupTrimSize, TableResizer.trimInSegmentResults)."""
    k = trim_size(query, min_trim)
    if not k or len(block.groups) <= k:
        return block
    gb_index = {str(e): i for i, e in enumerate(query.group_by)}
    recs = [(key, [final_result(a.function, x) for a, x in zip(query.aggregations, v)]) for key, v in block.groups.items()]
    recs.sort(key=lambda r: tuple((x is None, x) for x in r[0]))  # (a null key after the values)

    def value_of(expr, rec):
        if str(expr) in gb_index:
            return rec[0][gb_index[str(expr)]]
        return rec[1][_agg_index(query, expr)]

    for ob in reversed(query.order_by):
        recs.sort(key=order_key(ob, lambda r: value_of(ob.expression, r)), reverse=not ob.ascending)
    keep = {r[0] for r in recs[:k]}
    block.groups = {key: v for key, v in block.groups.items() if key in keep}
    block.num_groups_trimmed = True
    return block


def broker_response(plan_maker, query, segments) -> ResultTable:
    """BaseQueriesTest.getBrokerResponse: server over ``segments``, reduced as OFFLINE + REALTIME."""
    from ..query.sql import parse
    qc = parse(query) if isinstance(query, str) else query
    block = plan_maker.make_instance_plan(qc, segments).next_block()
    return reduce_blocks(qc, [block, block])
