"""Query model for the segment execution path: a Python mirror of the parts of Pinot's
``QueryContext`` / ``FilterContext`` / ``Predicate`` that the filter -> aggregation / group-by
path consumes, plus a parser for the SQL subset the reference's own tests use.

Reference anchors
-----------------
* ``QueryContext`` getters: pinot-core/.../core/query/request/context/QueryContext.java:190-357
  (filter, group-by expressions, aggregation functions, order-by, limit, numGroupsLimit).
* ``FilterContext`` {AND, OR, NOT, PREDICATE}: pinot-common/.../request/context/FilterContext.java.
* Predicates (values are kept as *strings*, exactly as Pinot stores them):
  ``EqPredicate``, ``NotEqPredicate``, ``InPredicate``, ``NotInPredicate``, ``RangePredicate``
  (pinot-common/.../request/context/predicate/*.java; RangePredicate.UNBOUNDED = "*").
* SQL -> QueryContext: CalciteSqlParser + RequestContextUtils (comparison operators become RANGE,
  ``=`` EQ, ``<>``/``!=`` NOT_EQ, ``BETWEEN`` inclusive RANGE); default LIMIT 10
  (CommonConstants.Broker.DEFAULT_BROKER_QUERY_LIMIT... QueryContext limit default).
* Query options ``numGroupsLimit`` / ``minSegmentGroupTrimSize`` / ``minServerGroupTrimSize`` /
  ``groupTrimThreshold`` (CommonConstants.java:328-350, InstancePlanMakerImplV2.applyQueryOptions :166-229).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple, Union

UNBOUNDED = "*"

# Aggregation function types supported on this path (AggregationFunctionFactory.java:186-263).
COUNT, SUM, MIN, MAX, DISTINCTCOUNTHLL = "COUNT", "SUM", "MIN", "MAX", "DISTINCTCOUNTHLL"
SUPPORTED_AGGREGATIONS = (COUNT, SUM, MIN, MAX, DISTINCTCOUNTHLL)
DEFAULT_HLL_LOG2M = 8  # CommonConstants.Helix.DEFAULT_HYPERLOGLOG_LOG2M (CommonConstants.java:96-97)
DEFAULT_NUM_GROUPS_LIMIT = 100_000  # InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT (:72-73)
DEFAULT_QUERY_LIMIT = 10


# --------------------------------------------------------------------------- predicates
@dataclass(frozen=True)
class Predicate:
    column: str

    @property
    def type(self) -> str:
        return self.TYPE  # type: ignore[attr-defined]


@dataclass(frozen=True)
class EqPredicate(Predicate):
    value: str
    TYPE = "EQ"


@dataclass(frozen=True)
class NotEqPredicate(Predicate):
    value: str
    TYPE = "NOT_EQ"


@dataclass(frozen=True)
class InPredicate(Predicate):
    values: Tuple[str, ...]
    TYPE = "IN"


@dataclass(frozen=True)
class NotInPredicate(Predicate):
    values: Tuple[str, ...]
    TYPE = "NOT_IN"


@dataclass(frozen=True)
class RangePredicate(Predicate):
    lower: str = UNBOUNDED
    upper: str = UNBOUNDED
    lower_inclusive: bool = False
    upper_inclusive: bool = False
    TYPE = "RANGE"


# --------------------------------------------------------------------------- filter tree
@dataclass(frozen=True)
class FilterContext:
    type: str  # "AND" | "OR" | "NOT" | "PREDICATE"
    children: Tuple["FilterContext", ...] = ()
    predicate: Optional[Predicate] = None

    @staticmethod
    def pred(p: Predicate) -> "FilterContext":
        return FilterContext("PREDICATE", (), p)

    # FlattenAndOrFilterOptimizer (QueryOptimizer.java:47): an AND child of an AND (an OR child of an OR) is spliced
    # into its parent, as the reference's query optimizer does before planning

    @staticmethod
    def and_(*c: "FilterContext") -> "FilterContext":
        return FilterContext("AND", tuple(x for k in c for x in (k.children if k.type == "AND" else (k,))))

    @staticmethod
    def or_(*c: "FilterContext") -> "FilterContext":
        return FilterContext("OR", tuple(x for k in c for x in (k.children if k.type == "OR" else (k,))))

    @staticmethod
    def not_(c: "FilterContext") -> "FilterContext":
        return FilterContext("NOT", (c,))

    def columns(self) -> List[str]:
        if self.type == "PREDICATE":
            return [self.predicate.column]
        out: List[str] = []
        for c in self.children:
            for col in c.columns():
                if col not in out:
                    out.append(col)
        return out


# --------------------------------------------------------------------------- aggregations
# 2-operand expressions inside aggregates (SSB Q1.x SUM(lo_extendedprice * lo_discount), Q4.x
# SUM(lo_revenue - lo_supplycost)), computed per row as double arithmetic (MultiplicationTransformFunction.java:89-104).
# Their names in result columns are the parser's canonical SqlKind names (CalciteSqlParser.java:798
# canonicalizeFunctionNamePreservingSpecialKey(functionKind.name()): TIMES -> "times", MINUS -> "minus", PLUS -> "plus"),
# so SUM(a*b) is reported as `sum(times(a,b))`, the same name datatable.cpp's agg_column_name writes.
EXPR_OPS = {"*": "times", "-": "minus", "+": "plus"}


@dataclass(frozen=True)
class AggregationSpec:
    function: str           # COUNT | SUM | MIN | MAX | DISTINCTCOUNTHLL
    column: Optional[str]   # None for COUNT(*); the first operand of an expression
    log2m: int = DEFAULT_HLL_LOG2M
    column2: Optional[str] = None  # second operand of `column <op> column2`
    op: Optional[str] = None       # "*", "-" or "+" (None: plain column)

    def columns(self) -> List[str]:
        return [c for c in (self.column, self.column2) if c]

    def result_name(self) -> str:
        arg = "*" if self.column is None else self.column
        if self.op:
            arg = f"{EXPR_OPS[self.op]}({self.column},{self.column2})"
        if self.function == DISTINCTCOUNTHLL and self.log2m != DEFAULT_HLL_LOG2M:
            arg = f"{arg},{self.log2m}"
        return f"{self.function.lower()}({arg})"


@dataclass(frozen=True)
class OrderByExpression:
    kind: str        # "column" | "aggregation"
    ref: Union[str, int]   # column name or index into QueryContext.aggregations
    asc: bool = True


@dataclass
class SelectItem:
    kind: str        # "column" | "aggregation"
    ref: Union[str, int]
    alias: Optional[str] = None


@dataclass
class QueryContext:
    table: str = "testTable"
    select: List[SelectItem] = field(default_factory=list)
    filter: Optional[FilterContext] = None
    group_by: List[str] = field(default_factory=list)
    aggregations: List[AggregationSpec] = field(default_factory=list)
    order_by: List[OrderByExpression] = field(default_factory=list)
    limit: int = DEFAULT_QUERY_LIMIT
    options: dict = field(default_factory=dict)

    @property
    def num_groups_limit(self) -> int:
        return int(self.options.get("numGroupsLimit", DEFAULT_NUM_GROUPS_LIMIT))

    def add_aggregation(self, a: AggregationSpec) -> int:
        if a in self.aggregations:
            return self.aggregations.index(a)
        self.aggregations.append(a)
        return len(self.aggregations) - 1

    def result_columns(self) -> List[str]:
        out = []
        for s in self.select:
            if s.alias:
                out.append(s.alias)
            elif s.kind == "column":
                out.append(s.ref)
            else:
                out.append(self.aggregations[s.ref].result_name())
        return out


# --------------------------------------------------------------------------- SQL subset parser
_TOKEN = re.compile(
    r"\s*(?:(?P<num>-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?)|(?P<str>'(?:[^']|'')*')|(?P<id>[A-Za-z_][A-Za-z0-9_.$]*)"
    r"|(?P<op><>|!=|<=|>=|=|<|>|\(|\)|,|\*|;|\+|-))")

_KEYWORDS = {"SELECT", "FROM", "WHERE", "GROUP", "BY", "ORDER", "LIMIT", "AND", "OR", "NOT", "IN",
             "BETWEEN", "AS", "ASC", "DESC", "SET", "TOP"}


class SqlParseError(ValueError):
    pass


class _Parser:
    def __init__(self, sql: str):
        self.toks: List[Tuple[str, str]] = []
        pos = 0
        sql = sql.strip()
        while pos < len(sql):
            m = _TOKEN.match(sql, pos)
            if not m or m.end() == pos:
                if sql[pos:].strip() == "":
                    break
                raise SqlParseError(f"bad token at {sql[pos:pos + 20]!r}")
            pos = m.end()
            kind = m.lastgroup
            text = m.group(kind)
            if kind == "id" and text.upper() in _KEYWORDS:
                self.toks.append(("kw", text.upper()))
            else:
                self.toks.append((kind, text))
        self.i = 0

    def peek(self, k=0):
        j = self.i + k
        return self.toks[j] if j < len(self.toks) else ("eof", "")

    def take(self):
        t = self.peek()
        self.i += 1
        return t

    def accept(self, kind, text=None):
        t = self.peek()
        if t[0] == kind and (text is None or t[1] == text):
            self.i += 1
            return t
        return None

    def expect(self, kind, text=None):
        t = self.accept(kind, text)
        if t is None:
            raise SqlParseError(f"expected {text or kind}, got {self.peek()}")
        return t

    # literal -> Pinot string form
    def literal(self) -> str:
        t = self.take()
        if t[0] == "num":
            return t[1]
        if t[0] == "str":
            return t[1][1:-1].replace("''", "'")
        raise SqlParseError(f"expected literal, got {t}")

    def ident(self) -> str:
        t = self.take()
        if t[0] != "id":
            raise SqlParseError(f"expected identifier, got {t}")
        return t[1]

    def agg_call(self) -> Optional[AggregationSpec]:
        t, n = self.peek(), self.peek(1)
        if t[0] == "id" and n == ("op", "(") and t[1].upper() in SUPPORTED_AGGREGATIONS:
            fn = t[1].upper()
            self.i += 2
            col2 = op = None
            if self.accept("op", "*"):
                col = None
            else:
                col = self.ident()
                t2 = self.peek()
                if t2[0] == "op" and t2[1] in EXPR_OPS:
                    self.i += 1
                    op = t2[1]
                    col2 = self.ident()
                    if fn not in (SUM, MIN, MAX):
                        raise SqlParseError(f"expressions are supported in SUM/MIN/MAX, not {fn}")
            log2m = DEFAULT_HLL_LOG2M
            if self.accept("op", ","):
                log2m = int(self.literal())
            self.expect("op", ")")
            if fn != COUNT and col is None:
                raise SqlParseError(f"{fn}(*) not supported")
            if fn == COUNT:
                col = None
            return AggregationSpec(fn, col, log2m, col2, op)
        if t[0] == "id" and n == ("op", "("):
            raise SqlParseError(f"unsupported function {t[1]}")
        return None

    def filter_expr(self) -> FilterContext:
        children = [self.and_expr()]
        while self.accept("kw", "OR"):
            children.append(self.and_expr())
        return children[0] if len(children) == 1 else FilterContext.or_(*children)

    def and_expr(self) -> FilterContext:
        children = [self.not_expr()]
        while self.accept("kw", "AND"):
            children.append(self.not_expr())
        return children[0] if len(children) == 1 else FilterContext.and_(*children)

    def not_expr(self) -> FilterContext:
        if self.accept("kw", "NOT"):
            return FilterContext.not_(self.not_expr())
        if self.accept("op", "("):
            f = self.filter_expr()
            self.expect("op", ")")
            return f
        return self.predicate()

    def predicate(self) -> FilterContext:
        col = self.ident()
        negate = bool(self.accept("kw", "NOT"))
        if self.accept("kw", "IN"):
            self.expect("op", "(")
            vals = [self.literal()]
            while self.accept("op", ","):
                vals.append(self.literal())
            self.expect("op", ")")
            p = NotInPredicate(col, tuple(vals)) if negate else InPredicate(col, tuple(vals))
            return FilterContext.pred(p)
        if self.accept("kw", "BETWEEN"):
            lo = self.literal()
            self.expect("kw", "AND")
            hi = self.literal()
            f = FilterContext.pred(RangePredicate(col, lo, hi, True, True))
            return FilterContext.not_(f) if negate else f
        if negate:
            raise SqlParseError("NOT must precede IN/BETWEEN")
        op = self.take()
        if op[0] != "op":
            raise SqlParseError(f"expected comparison, got {op}")
        v = self.literal()
        o = op[1]
        if o == "=":
            p = EqPredicate(col, v)
        elif o in ("<>", "!="):
            p = NotEqPredicate(col, v)
        elif o == ">":
            p = RangePredicate(col, v, UNBOUNDED, False, False)
        elif o == ">=":
            p = RangePredicate(col, v, UNBOUNDED, True, False)
        elif o == "<":
            p = RangePredicate(col, UNBOUNDED, v, False, False)
        elif o == "<=":
            p = RangePredicate(col, UNBOUNDED, v, False, True)
        else:
            raise SqlParseError(f"bad operator {o}")
        return FilterContext.pred(p)


def parse_sql(sql: str) -> QueryContext:
    """Parse the SQL subset (SET options; SELECT aggregations / group-by columns FROM t
    [WHERE filter] [GROUP BY cols] [ORDER BY exprs] [LIMIT n])."""
    p = _Parser(sql)
    q = QueryContext()
    while p.accept("kw", "SET"):
        key = p.ident()
        p.expect("op", "=")
        # (QueryOptionsUtils reads boolean options such as skipStarTree=true as strings)
        q.options[key] = p.ident() if p.peek()[0] == "id" else p.literal()
        p.accept("op", ";")
    p.expect("kw", "SELECT")
    while True:
        agg = p.agg_call()
        if agg is not None:
            item = SelectItem("aggregation", q.add_aggregation(agg))
        else:
            item = SelectItem("column", p.ident())
        if p.accept("kw", "AS"):
            item.alias = p.ident()
        q.select.append(item)
        if not p.accept("op", ","):
            break
    p.expect("kw", "FROM")
    q.table = p.ident()
    if p.accept("kw", "WHERE"):
        q.filter = p.filter_expr()
    if p.accept("kw", "GROUP"):
        p.expect("kw", "BY")
        q.group_by.append(p.ident())
        while p.accept("op", ","):
            q.group_by.append(p.ident())
    if p.accept("kw", "ORDER"):
        p.expect("kw", "BY")
        while True:
            agg = p.agg_call()
            if agg is not None:
                ob = OrderByExpression("aggregation", q.add_aggregation(agg))
            else:
                name = p.ident()
                alias = [s for s in q.select if s.alias == name]
                if alias:
                    ob = OrderByExpression(alias[0].kind, alias[0].ref)
                else:
                    ob = OrderByExpression("column", name)
            if p.accept("kw", "DESC"):
                ob = OrderByExpression(ob.kind, ob.ref, False)
            else:
                p.accept("kw", "ASC")
            q.order_by.append(ob)
            if not p.accept("op", ","):
                break
    if p.accept("kw", "LIMIT"):
        q.limit = int(p.literal())
    p.accept("op", ";")
    if p.peek()[0] != "eof":
        raise SqlParseError(f"trailing input {p.peek()}")
    for s in q.select:
        if s.kind == "column" and q.group_by and s.ref not in q.group_by:
            raise SqlParseError(f"column {s.ref} not in GROUP BY")
    if not q.group_by and any(s.kind == "column" for s in q.select):
        raise SqlParseError("selection queries are out of scope for this path")
    return q
