"""A small SQL front end for the query shapes on the hot path.

The reference compiles SQL with Calcite (CalciteSqlParser, pinot-common/.../sql/parsers/) into a
PinotQuery, then QueryContextConverterUtils builds a QueryContext. This is a recursive-descent
parser for the subset the parity tests and SSB use: SELECT <aggregations / group columns>
FROM t [WHERE <boolean expr>] [GROUP BY ...] [ORDER BY ...] [LIMIT n], with predicates
=, <>, !=, <, <=, >, >=, [NOT] BETWEEN, [NOT] IN, IS [NOT] NULL and NOT/AND/OR, and +, -, *, / and CAST in
expressions. The reference optimizer's flattening of nested AND/OR
(pinot-core/.../query/optimizer/filter/FlattenAndOrFilterOptimizer.java) is applied.
"""
import re

from .context import (AggregationInfo, FilterClause, FilterContext, Function, Identifier, Literal, OrderByExpression,
                      Predicate, PredicateType, QueryContext, SUPPORTED_AGGREGATIONS, UNBOUNDED)

_TOKEN = re.compile(r"""\s*(?:
    (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?|\.\d+)
  | (?P<str>'(?:[^']|'')*')
  | (?P<ident>[A-Za-z_][A-Za-z0-9_$.]*|"[^"]+")
  | (?P<op><>|!=|<=|>=|[(),*+\-/=<>])
)""", re.VERBOSE)

_KEYWORDS = {"select", "from", "where", "group", "by", "order", "limit", "and", "or", "not", "between",
             "in", "asc", "desc", "as", "cast", "option", "case", "when", "then", "else", "end", "is", "null"}


class SqlError(ValueError):
    pass


def _tokenize(sql):
    pos = 0
    out = []
    sql = sql.strip().rstrip(";")
    while pos < len(sql):
        m = _TOKEN.match(sql, pos)
        if not m or m.end() == pos:
            if sql[pos:].strip() == "":
                break
            raise SqlError(f"cannot tokenize at {sql[pos:pos + 20]!r}")
        pos = m.end()
        if m.group("num") is not None:
            t = m.group("num")
            out.append(("num", float(t) if any(c in t for c in ".eE") else int(t)))
        elif m.group("str") is not None:
            out.append(("str", m.group("str")[1:-1].replace("''", "'")))
        elif m.group("ident") is not None:
            t = m.group("ident")
            if t.startswith('"'):
                out.append(("ident", t[1:-1]))
            elif t.lower() in _KEYWORDS:
                out.append(("kw", t.lower()))
            else:
                out.append(("ident", t))
        else:
            out.append(("op", m.group("op")))
    out.append(("eof", None))
    return out


class _Parser:
    def __init__(self, sql):
        self.toks = _tokenize(sql)
        self.i = 0

    def peek(self, k=0):
        return self.toks[self.i + k]

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind, val=None):
        t = self.peek()
        if t[0] == kind and (val is None or t[1] == val):
            self.i += 1
            return t
        return None

    def expect(self, kind, val=None):
        t = self.accept(kind, val)
        if t is None:
            raise SqlError(f"expected {val or kind}, got {self.peek()}")
        return t

    # expressions -------------------------------------------------------------------------
    def expr(self):
        e = self.term()
        while True:
            if self.accept("op", "+"):
                e = Function("plus", (e, self.term()))
            elif self.accept("op", "-"):
                e = Function("minus", (e, self.term()))
            else:
                return e

    def term(self):
        e = self.factor()
        while True:
            if self.accept("op", "*"):
                e = Function("times", (e, self.factor()))
            elif self.accept("op", "/"):
                e = Function("divide", (e, self.factor()))
            else:
                return e

    def factor(self):
        t = self.peek()
        if self.accept("op", "-"):
            v = self.factor()
            if isinstance(v, Literal) and not isinstance(v.value, str):
                return Literal(-v.value)
            return Function("minus", (Literal(0), v))
        if self.accept("op", "("):
            e = self.expr()
            self.expect("op", ")")
            return e
        if t[0] == "num":
            self.next()
            return Literal(t[1])
        if t[0] == "str":
            self.next()
            return Literal(t[1])
        if t[0] == "kw" and t[1] == "case":
            # CASE WHEN c1 THEN e1 [WHEN c2 THEN e2 ...] ELSE e END -> case(c1, e1, c2, e2, ..., e)
            # (CalciteSqlParser's CASE -> the "case" transform function, CaseTransformFunction)
            self.next()
            args = []
            while self.accept("kw", "when"):
                args.append(self.bool_or())
                self.expect("kw", "then")
                args.append(self.expr())
            if not args:
                raise SqlError("CASE needs WHEN")
            if not self.accept("kw", "else"):
                raise SqlError("CASE without ELSE (a null default) is outside the subset")
            args.append(self.expr())
            self.expect("kw", "end")
            return Function("case", tuple(args))
        if t[0] == "kw" and t[1] == "cast":
            self.next()
            self.expect("op", "(")
            e = self.expr()
            self.expect("kw", "as")
            typ = self.next()[1]
            self.expect("op", ")")
            return Function("cast", (e, Literal(str(typ).upper())))
        if t[0] == "ident":
            self.next()
            if self.accept("op", "("):
                name = t[1].lower()
                args = []
                if self.accept("op", "*"):
                    args = [Identifier("*")]
                elif not self.accept("op", ")"):
                    args.append(self.expr())
                    while self.accept("op", ","):
                        args.append(self.expr())
                    self.expect("op", ")")
                    return self._func(name, args)
                else:
                    return self._func(name, args)
                self.expect("op", ")")
                return self._func(name, args)
            return Identifier(t[1])
        raise SqlError(f"unexpected token {t}")

    @staticmethod
    def _func(name, args):
        alias = {"sub": "minus", "add": "plus", "mult": "times", "div": "divide"}
        return Function(alias.get(name, name), tuple(args))

    # boolean expressions ------------------------------------------------------------------
    def bool_or(self):
        kids = [self.bool_and()]
        while self.accept("kw", "or"):
            kids.append(self.bool_and())
        if len(kids) == 1:
            return kids[0]
        flat = []
        for k in kids:
            flat.extend(k.children if k.type == "OR" else [k])
        return FilterContext.OR(*flat)

    def bool_and(self):
        kids = [self.bool_not()]
        while self.accept("kw", "and"):
            kids.append(self.bool_not())
        if len(kids) == 1:
            return kids[0]
        flat = []
        for k in kids:
            flat.extend(k.children if k.type == "AND" else [k])
        return FilterContext.AND(*flat)

    def bool_not(self):
        if self.accept("kw", "not"):
            return FilterContext.NOT(self.bool_not())
        if self.peek() == ("op", "(") and self._paren_is_boolean():
            self.next()
            f = self.bool_or()
            self.expect("op", ")")
            return f
        return self.predicate()

    def _paren_is_boolean(self):
        depth = 0
        j = self.i
        while True:
            k, v = self.toks[j]
            if k == "eof":
                return False
            if (k, v) == ("op", "("):
                depth += 1
            elif (k, v) == ("op", ")"):
                depth -= 1
                if depth == 0:
                    return False
            elif depth == 1 and k == "kw" and v in ("and", "or", "not", "between", "in", "is"):
                return True
            elif depth == 1 and k == "op" and v in ("=", "<>", "!=", "<", "<=", ">", ">="):
                return True
            j += 1

    def _lit(self):
        e = self.expr()
        if not isinstance(e, Literal):
            raise SqlError("predicate right-hand side must be a literal")
        return e.value

    def predicate(self):
        lhs = self.expr()
        if self.accept("kw", "is"):  # IS [NOT] NULL (Predicate.Type.IS_NULL / IS_NOT_NULL)
            neg = bool(self.accept("kw", "not"))
            self.expect("kw", "null")
            return FilterContext.PRED(Predicate(PredicateType.IS_NOT_NULL if neg else PredicateType.IS_NULL, lhs))
        neg = bool(self.accept("kw", "not"))
        if self.accept("kw", "between"):
            lo = self._lit()
            self.expect("kw", "and")
            hi = self._lit()
            p = FilterContext.PRED(Predicate(PredicateType.RANGE, lhs, lower=lo, upper=hi,
                                             lower_inclusive=True, upper_inclusive=True))
            return FilterContext.NOT(p) if neg else p
        if self.accept("kw", "in"):
            self.expect("op", "(")
            vals = [self._lit()]
            while self.accept("op", ","):
                vals.append(self._lit())
            self.expect("op", ")")
            return FilterContext.PRED(Predicate(PredicateType.NOT_IN if neg else PredicateType.IN, lhs,
                                                values=tuple(vals)))
        if neg:
            raise SqlError("NOT must precede BETWEEN or IN")
        op = self.expect("op")[1]
        v = self._lit()
        if op == "=":
            return FilterContext.PRED(Predicate(PredicateType.EQ, lhs, values=(v,)))
        if op in ("<>", "!="):
            return FilterContext.PRED(Predicate(PredicateType.NOT_EQ, lhs, values=(v,)))
        if op == "<":
            return FilterContext.PRED(Predicate(PredicateType.RANGE, lhs, upper=v))
        if op == "<=":
            return FilterContext.PRED(Predicate(PredicateType.RANGE, lhs, upper=v, upper_inclusive=True))
        if op == ">":
            return FilterContext.PRED(Predicate(PredicateType.RANGE, lhs, lower=v))
        if op == ">=":
            return FilterContext.PRED(Predicate(PredicateType.RANGE, lhs, lower=v, lower_inclusive=True))
        raise SqlError(f"unsupported operator {op}")

    # query ------------------------------------------------------------------------------
    def query(self):
        self.expect("kw", "select")
        select = [self._select_item()]
        while self.accept("op", ","):
            select.append(self._select_item())
        self.expect("kw", "from")
        table = self.expect("ident")[1]
        filt = None
        if self.accept("kw", "where"):
            filt = self.bool_or()
        group_by = []
        if self.accept("kw", "group"):
            self.expect("kw", "by")
            group_by.append(self.expr())
            while self.accept("op", ","):
                group_by.append(self.expr())
        order_by = []
        if self.accept("kw", "order"):
            self.expect("kw", "by")
            order_by.append(self._order_item())
            while self.accept("op", ","):
                order_by.append(self._order_item())
        limit = 10
        if self.accept("kw", "limit"):
            limit = int(self.expect("num")[1])
        self.expect("eof")
        return table, select, filt, group_by, order_by, limit

    def _select_item(self):
        if self.accept("op", "*"):  # SELECT * (expanded per segment: SelectionOperatorUtils.extractExpressions)
            return Identifier("*"), None
        e = self.expr()
        if self.peek()[0] == "ident" and str(self.peek()[1]).lower() == "filter":
            # agg(...) FILTER(WHERE ...) (CalciteSqlParser's FILTER clause -> filtered aggregation)
            if not (isinstance(e, Function) and e.name in SUPPORTED_AGGREGATIONS):
                raise SqlError("FILTER applies to an aggregation")
            self.next()
            self.expect("op", "(")
            self.expect("kw", "where")
            f = self.bool_or()
            self.expect("op", ")")
            e = FilterClause(e, f)
        alias = None
        if self.accept("kw", "as"):
            alias = self.next()[1]
        elif self.peek()[0] == "ident":
            alias = self.next()[1]
        return e, alias

    def _order_item(self):
        e = self.expr()
        asc = True
        if self.accept("kw", "desc"):
            asc = False
        else:
            self.accept("kw", "asc")
        nulls_last = None
        t = self.peek()
        if t[0] == "ident" and str(t[1]).lower() == "nulls":  # NULLS FIRST | NULLS LAST
            self.i += 1
            w = self.expect("ident")[1].lower()
            if w not in ("first", "last"):
                raise SqlError(f"NULLS {w}: expected FIRST or LAST")
            nulls_last = w == "last"
        return OrderByExpression(e, asc, nulls_last)


def _collect_aggs(expr, out, flt=None, null_handling=False):
    if isinstance(expr, FilterClause):
        _collect_aggs(expr.function, out, expr.filter, null_handling)
        return
    if isinstance(expr, Function):
        if expr.name in SUPPORTED_AGGREGATIONS:
            arg = None
            if expr.name == "count":
                # COUNT(col) counts the non-null values under enableNullHandling (an identifier or a function
                # argument; COUNT(*) and COUNT(literal) stay COUNT(*): CountAggregationFunction.java:44-52)
                a0 = expr.args[0] if expr.args else None
                if null_handling and a0 is not None and not isinstance(a0, Literal) and a0 != Identifier("*"):
                    arg = a0
            else:
                if len(expr.args) < 1:
                    raise SqlError(f"{expr.name} needs an argument")
                arg = expr.args[0]
            log2m = 8
            if expr.name in ("distinctcounthll", "distinctcountrawhll") and len(expr.args) > 1:
                log2m = int(expr.args[1].value)
            info = AggregationInfo(expr.name, arg, log2m, flt)
            if info not in out:
                out.append(info)
            return
        for a in expr.args:
            _collect_aggs(a, out, None, null_handling)


_SET = re.compile(r"\s*SET\s+([A-Za-z_][A-Za-z0-9_.]*)\s*=\s*('(?:[^']|'')*'|[^;]*?)\s*;", re.IGNORECASE)


# CommonConstants.Broker.Request.QueryOptionKey names this path reads: SET keys resolve to them case-insensitively
# (QueryOptionsUtils.resolveCaseInsensitiveOptions, pinot-common/.../utils/config/QueryOptionsUtils.java:80-95)
QUERY_OPTION_KEYS = ("useGpu", "numGroupsLimit", "minSegmentGroupTrimSize", "minServerGroupTrimSize",
                     "groupTrimThreshold", "enableNullHandling", "filteredAggregationsSkipEmptyGroups", "useStarTree",
                     "serverReturnFinalResult", "serverReturnFinalResultKeyUnpartitioned",
                     "maxInitialResultHolderCapacity", "minInitialIndexedTableCapacity", "timeoutMs")
_OPTION_RESOLVER = {k.lower(): k for k in QUERY_OPTION_KEYS}


def parse(sql: str) -> QueryContext:
    """SQL -> QueryContext; leading ``SET key = value;`` statements become query options (as the broker's
    CalciteSqlParser.compileToPinotQuery collects them)."""
    options = {}
    while True:
        m = _SET.match(sql)
        if not m:
            break
        v = m.group(2)
        key = _OPTION_RESOLVER.get(m.group(1).lower(), m.group(1))
        options[key] = v[1:-1].replace("''", "'") if v.startswith("'") else v
        sql = sql[m.end():]
    table, select, filt, group_by, order_by, limit = _Parser(sql).query()
    aggs = []
    nh = str(options.get("enableNullHandling", "false")).strip().lower() == "true"
    for e, _ in select:
        _collect_aggs(e, aggs, None, nh)
    # ORDER BY may reference aggregations absent from the select list (InterSegmentGroupBy tests)
    alias_map = {a: e for e, a in select if a}
    resolved_order = []
    for ob in order_by:
        e = ob.expression
        if isinstance(e, Identifier) and e.name in alias_map:
            e = alias_map[e.name]
        _collect_aggs(e, aggs, None, nh)
        resolved_order.append(OrderByExpression(e, ob.ascending, ob.nulls_last))
    for e, _ in select:
        if isinstance(e, FilterClause):
            continue
        if not isinstance(e, Function) or e.name not in SUPPORTED_AGGREGATIONS:
            if group_by and e not in group_by:
                raise SqlError(f"select expression {e} is neither an aggregation nor a group-by expression")
    if not aggs and not group_by:
        # selection (SelectionOnlyOperator): columns and arithmetic over them; SELECT * stays a single '*'
        for e, _ in select:
            if isinstance(e, FilterClause) or (isinstance(e, Identifier) and e.name == "*" and len(select) > 1):
                raise SqlError(f"select expression {e} in a selection query")
    return QueryContext(table, select, aggs, filt, group_by, resolved_order, limit, options)
