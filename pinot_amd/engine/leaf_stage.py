"""Multi-stage engine leaf stage over the GPU server path.

The multi-stage engine runs the single-stage server executor on a leaf stage's segments and ships its results
blocks to the next stage as row blocks (pinot-query-runtime/.../runtime/operator/LeafStageTransferableBlockOperator.java):

  getNextBlock            :160-183   one TransferableBlock per results block, then an end-of-stream metadata block
                                     carrying the merged execution statistics
  composeTransferableBlock :490-500  rows of BaseResultsBlock.getRows() converted to the stage's desired DataSchema
  composeDirectTransferableBlock / convertRow :595-617   per column, when the stored types differ, TypeUtils.convert
                                     (…/operator/utils/TypeUtils.java:40-60: Number.intValue / longValue / floatValue /
                                     doubleValue, toString for STRING)

Selection leaves (the lineorder side of a joined SSB query: a filter plus a projection of join keys and metrics,
SelectionOnlyOperator) arrive as SelectionResultsBlocks: composeSelectTransferableBlock (:505-560) maps the stage's
select expressions onto the block's DataSchema columns (reordering when they differ) and converts the stored types.

Rows follow the results blocks: AggregationResultsBlock.getRows (…/blocks/results/AggregationResultsBlock.java:99-101)
is one row of intermediate results; GroupByResultsBlock.getRows (:173-183) is one row per group, group-by values
then intermediates. Intermediates keep their single-stage types: SUM / MIN / MAX as DOUBLE (the library's exact
integer sums are handed over as the double the reference holds), COUNT as LONG, AVG / MINMAXRANGE / HLL as OBJECT
(the (sum, count) / (min, max) pairs and the register arrays of this package's results containers).

GpuLeafStageOperator replaces the per-segment server plan of a leaf stage with the GPU combine operator of
GpuInstancePlanMaker (one launch over all of the stage's segments); everything after it -- exchange, joins,
the intermediate aggregate -- stays with the multi-stage engine.
"""
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .results import AggregationResultsBlock, GroupByResultsBlock, SelectionResultsBlock

# DataSchema.ColumnDataType stored types on this path
INT, LONG, FLOAT, DOUBLE, STRING, OBJECT = "INT", "LONG", "FLOAT", "DOUBLE", "STRING", "OBJECT"


@dataclass
class DataSchema:
    column_names: List[str]
    column_types: List[str]   # stored ColumnDataType names


@dataclass
class TransferableBlock:
    """DataBlock.Type.ROW (rows + schema) or the end-of-stream metadata block (stats)."""
    rows: Optional[List[list]]
    schema: Optional[DataSchema]
    is_end_of_stream: bool = False
    stats: dict = field(default_factory=dict)


def _java_d2i(x, bits):
    """Java's double -> int / long narrowing (JLS 5.1.3): NaN -> 0, saturating at the type's range."""
    if x != x:
        return 0
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    return lo if x <= lo else (hi if x >= hi else int(x))


def convert(value, stored_type):
    """TypeUtils.convert (TypeUtils.java:40-60): Number.intValue / longValue / floatValue / doubleValue."""
    if stored_type in (INT, LONG):
        bits = 32 if stored_type == INT else 64
        if isinstance(value, (int, np.integer)):  # long -> int wraps (two's complement)
            v = int(value) & ((1 << bits) - 1)
            return v - (1 << bits) if v >> (bits - 1) else v
        return _java_d2i(float(value), bits)
    if stored_type == FLOAT:
        return float(np.float32(value))
    if stored_type == DOUBLE:
        return float(value)
    if stored_type == STRING:
        return str(value)
    return value


def _stored_type(function):
    """getIntermediateResultColumnType of the functions on the path (stored types)."""
    if function == "count":
        return LONG
    if function in ("sum", "min", "max"):
        return DOUBLE
    return OBJECT


def _intermediate(function, v):
    if function == "count":
        return int(v)
    if function in ("sum", "min", "max"):
        return float(v)
    return v


def block_schema(block) -> DataSchema:
    """The results block's own schema (group-by columns first, then one column per function; a selection block's
    DataSchema as it is). Group-by column types are the columns' stored types from the segment metadata
    (GroupByResultsBlock's DataSchema: the group-by expressions' result types), never guessed from the values."""
    if isinstance(block, SelectionResultsBlock):
        return DataSchema(list(block.column_names), list(block.column_types))
    aggs = block.aggregations
    names = [a.result_column_name for a in aggs]
    types = [_stored_type(a.function) for a in aggs]
    if isinstance(block, GroupByResultsBlock):
        keys = [str(e) for e in block.group_by]
        if block.key_types is None:
            raise ValueError("group-by block without key types (the plan records them from the column metadata)")
        return DataSchema(keys + names, list(block.key_types) + types)
    return DataSchema(names, types)


def block_rows(block) -> List[list]:
    """BaseResultsBlock.getRows."""
    if isinstance(block, SelectionResultsBlock):
        return block.rows
    fns = [a.function for a in block.aggregations]
    if isinstance(block, AggregationResultsBlock):
        return [[_intermediate(f, v) for f, v in zip(fns, block.results)]]
    return [list(k) + [_intermediate(f, v) for f, v in zip(fns, vals)] for k, vals in block.groups.items()]


def compose_select_transferable_block(block: SelectionResultsBlock, select_exprs, desired: DataSchema):
    """composeSelectTransferableBlock (LeafStageTransferableBlockOperator.java:505-583): the column of every stage
    select expression in the block's DataSchema; in order -> composeDirectTransferableBlock, else
    composeColumnIndexedTransferableBlock (reorder, converting where the stored types differ)."""
    index = {n: i for i, n in enumerate(block.column_names)}
    idx = [index[str(e)] for e in select_exprs]
    if idx == list(range(len(idx))) and len(idx) == len(block.column_names):
        return compose_transferable_block(block, desired)
    have = block.column_types
    conv = [have[i] != t for i, t in zip(idx, desired.column_types)]
    cols = [c.tolist() if hasattr(c, "tolist") else list(c) for c in block.columns]
    rows = []
    for r in range(block.num_rows):
        row = []
        for j, i in enumerate(idx):
            v = cols[i][r]
            row.append(convert(v, desired.column_types[j]) if conv[j] and v is not None else v)
        rows.append(row)
    return TransferableBlock(rows, desired)


def compose_transferable_block(block, desired: DataSchema) -> TransferableBlock:
    """composeDirectTransferableBlock: convert the columns whose stored type differs from the desired one."""
    rows = block_rows(block)
    have = block_schema(block).column_types
    if len(have) != len(desired.column_types):
        raise ValueError(f"leaf stage schema has {len(desired.column_types)} columns, the block {len(have)}")
    diff = [i for i, (a, b) in enumerate(zip(have, desired.column_types)) if a != b]
    for r in rows:
        for i in diff:
            if r[i] is not None:
                r[i] = convert(r[i], desired.column_types[i])
    return TransferableBlock(rows, desired)


class GpuLeafStageOperator:
    """LeafStageTransferableBlockOperator with the GPU server path underneath: next_block() returns the data
    block, then the end-of-stream block with the execution statistics (numDocsScanned, numEntriesScanned*,
    numSegments*, totalDocs) the leaf stage reports upward."""

    def __init__(self, query, segments, desired_schema: Optional[DataSchema] = None, plan_maker=None):
        from .plan import GpuInstancePlanMaker
        from ..query.sql import parse
        self.query = parse(query) if isinstance(query, str) else query
        self.segments = list(segments)
        self.desired = desired_schema
        self.plan_maker = plan_maker or GpuInstancePlanMaker()
        self._state = 0
        self._stats = {}

    def next_block(self) -> TransferableBlock:
        if self._state == 0:
            op = self.plan_maker.make_instance_plan(self.query, self.segments)
            try:
                blk = op.next_block()
            finally:
                if hasattr(op, "close"):
                    op.close()
            s = blk.stats
            self._stats = {"numDocsScanned": s.num_docs_scanned,
                           "numEntriesScannedInFilter": s.num_entries_scanned_in_filter,
                           "numEntriesScannedPostFilter": s.num_entries_scanned_post_filter,
                           "numSegmentsProcessed": s.num_segments_processed,
                           "numSegmentsMatched": s.num_segments_matched,
                           "totalDocs": s.num_total_docs,
                           "numGroupsLimitReached": bool(getattr(blk, "num_groups_limit_reached", False))}
            self._state = 1
            if isinstance(blk, SelectionResultsBlock):
                exprs = [e for e, _ in self.query.select]
                if len(exprs) == 1 and str(exprs[0]) == "*":
                    exprs = list(blk.column_names)
                return compose_select_transferable_block(blk, exprs, self.desired or block_schema(blk))
            return compose_transferable_block(blk, self.desired or block_schema(blk))
        self._state = 2
        return TransferableBlock(None, None, is_end_of_stream=True, stats=dict(self._stats))
