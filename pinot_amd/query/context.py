"""Query context types (host side).

Mirrors the shapes the reference's server consumes (all in pinot-common / pinot-core, used as
inputs to the hot path, not rebuilt):
  ExpressionContext      pinot-common/.../request/context/ExpressionContext.java
  FilterContext          pinot-common/.../request/context/FilterContext.java:37-39 (AND/OR/NOT/PREDICATE/CONSTANT)
  Predicate.Type         pinot-common/.../request/context/predicate/Predicate.java:30-42
  RangePredicate         pinot-common/.../request/context/predicate/RangePredicate.java:38-143
  QueryContext           pinot-core/.../query/request/context/QueryContext.java:74-757
"""
from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Union


# ----------------------------------------------------------------------------- expressions
@dataclass(frozen=True)
class Identifier:
    name: str

    def __str__(self):
        return self.name


@dataclass(frozen=True)
class Literal:
    value: Union[int, float, str]

    def __str__(self):
        return repr(self.value) if isinstance(self.value, str) else str(self.value)


@dataclass(frozen=True)
class Function:
    name: str  # lower-case canonical name
    args: Tuple["Expression", ...]

    def __str__(self):
        return f"{self.name}({','.join(str(a) for a in self.args)})"


@dataclass(frozen=True)
class FilterClause:
    """`agg(...) FILTER(WHERE ...)`: an aggregation with its own filter (QueryContext's
    filtered-aggregation pairs, pinot-core/.../query/request/context/QueryContext.java)."""
    function: "Function"
    filter: "FilterContext"

    def __str__(self):
        return f"{self.function} FILTER(WHERE {self.filter})"


Expression = Union[Identifier, Literal, Function, FilterClause]


def columns_of(expr) -> List[str]:
    if isinstance(expr, Identifier):
        return [expr.name]
    if isinstance(expr, FilterContext):  # a CASE condition
        return expr.columns()
    if isinstance(expr, FilterClause):
        return columns_of(expr.function)
    if isinstance(expr, Function):
        out = []
        for a in expr.args:
            for c in columns_of(a):
                if c not in out:
                    out.append(c)
        return out
    return []


# ----------------------------------------------------------------------------- predicates
class PredicateType:
    EQ = "EQ"
    NOT_EQ = "NOT_EQ"
    IN = "IN"
    NOT_IN = "NOT_IN"
    RANGE = "RANGE"
    IS_NULL = "IS_NULL"          # the column's null value vector (FilterPlanNode.java:294-307)
    IS_NOT_NULL = "IS_NOT_NULL"


UNBOUNDED = "*"  # RangePredicate.UNBOUNDED


@dataclass(frozen=True)
class Predicate:
    type: str
    lhs: Expression
    values: Tuple = ()                 # EQ/NOT_EQ: (v,), IN/NOT_IN: (v1, ...)
    lower: object = UNBOUNDED          # RANGE
    upper: object = UNBOUNDED
    lower_inclusive: bool = False
    upper_inclusive: bool = False

    @property
    def column(self) -> str:
        if not isinstance(self.lhs, Identifier):
            raise NotImplementedError("predicates on expressions are out of scope")
        return self.lhs.name


@dataclass(frozen=True)
class FilterContext:
    type: str  # AND / OR / NOT / PREDICATE / CONSTANT
    children: Tuple["FilterContext", ...] = ()
    predicate: Optional[Predicate] = None
    constant: Optional[bool] = None

    @staticmethod
    def AND(*children):
        return FilterContext("AND", tuple(children))

    @staticmethod
    def OR(*children):
        return FilterContext("OR", tuple(children))

    @staticmethod
    def NOT(child):
        return FilterContext("NOT", (child,))

    @staticmethod
    def PRED(p: Predicate):
        return FilterContext("PREDICATE", predicate=p)

    def columns(self) -> List[str]:
        if self.type == "PREDICATE":
            return [self.predicate.column]
        out = []
        for c in self.children:
            for x in c.columns():
                if x not in out:
                    out.append(x)
        return out


# ----------------------------------------------------------------------------- aggregations
SUPPORTED_AGGREGATIONS = ("count", "sum", "min", "max", "avg", "minmaxrange", "distinctcounthll",
                          "distinctcountrawhll", "distinctcount")


@dataclass(frozen=True)
class AggregationInfo:
    function: str           # canonical lower-case name, e.g. "sum"
    argument: Optional[Expression]  # None for COUNT(*)
    log2m: int = 8
    filter: Optional["FilterContext"] = None  # FILTER(WHERE ...) of a filtered aggregation

    @property
    def result_column_name(self) -> str:
        """AggregationFunction.getResultColumnName(): lower-case function name + argument; COUNT(col) keeps its
        argument only under enableNullHandling (the argument is then set: CountAggregationFunction.java:44-66)."""
        if self.function == "count":
            base = "count(*)" if self.argument is None else f"count({self.argument})"
        else:
            base = f"{self.function}({self.argument})"
        return base if self.filter is None else f"{base} FILTER(WHERE {self.filter})"

    def unfiltered(self) -> "AggregationInfo":
        return AggregationInfo(self.function, self.argument, self.log2m)


@dataclass
class OrderByExpression:
    expression: Expression
    ascending: bool = True
    nulls_last: Optional[bool] = None  # NULLS FIRST / LAST; None = the default

    @property
    def is_nulls_last(self) -> bool:
        """OrderByExpressionContext.isNullsLast (pinot-core/.../request/context/OrderByExpressionContext.java:53-61):
        nulls sort as if larger than every value unless NULLS FIRST / LAST says otherwise."""
        return self.ascending if self.nulls_last is None else self.nulls_last


@dataclass
class QueryContext:
    table: str
    select: List[Tuple[Expression, Optional[str]]]
    aggregations: List[AggregationInfo]
    filter: Optional[FilterContext]
    group_by: List[Expression]
    order_by: List[OrderByExpression] = field(default_factory=list)
    limit: int = 10
    options: dict = field(default_factory=dict)

    @property
    def is_aggregation(self) -> bool:
        return bool(self.aggregations) and not self.group_by

    @property
    def is_group_by(self) -> bool:
        return bool(self.group_by)

    @property
    def is_selection(self) -> bool:
        """A selection (row-returning) query: no aggregation, no group-by (QueryContext.isSelectionQuery)."""
        return not self.aggregations and not self.group_by

    def select_expressions(self, segment_columns=None):
        """SelectionOperatorUtils.extractExpressions (pinot-core/.../query/selection/SelectionOperatorUtils.java:
        83-124) without ORDER BY: the select expressions, deduplicated in order; SELECT * expands to the segment's
        columns sorted by name (columns starting with '$' excluded)."""
        exprs = [e for e, _ in self.select]
        if len(exprs) == 1 and isinstance(exprs[0], Identifier) and exprs[0].name == "*":
            return [Identifier(c) for c in sorted(c for c in (segment_columns or []) if not c.startswith("$"))]
        out = []
        for e in exprs:
            if e not in out:
                out.append(e)
        return out
