"""Hand-written SQL tokenizer + recursive-descent parser (the SparkSQL subset the "Data
Frame" widget needs; reference: orangecontrib/spark/widgets/data/spark_sql_dataframe.py:83-94
runs ``hc.sql(query)``; Hive Table uses ``show databases``, spark_table.py:41).

Produces plain tuples (the AST) consumed by ``sql.engine``; scalar expressions compile
to ``frame.expr.Expr`` so evaluation is the same vectorised device code as the
DataFrame API.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field

from ..frame import expr as E

GRAMMAR = """\
statement :=
    [WITH name AS (select) [, ...]] select
  | CREATE TABLE name AS select
  | CREATE [OR REPLACE] [GLOBAL] [TEMP|TEMPORARY] VIEW [IF NOT EXISTS] name AS select
  | INSERT {INTO | OVERWRITE} [TABLE] name [(col, ...)] {VALUES (v, ...), ... | select}
  | CACHE [LAZY] TABLE name [AS select] | UNCACHE TABLE [IF EXISTS] name | REFRESH TABLE name
  | TRUNCATE TABLE name | ALTER {TABLE|VIEW} name RENAME TO name
  | DROP TABLE [IF EXISTS] name | DROP VIEW [IF EXISTS] name | DROP DATABASE [IF EXISTS] name
  | CREATE DATABASE [IF NOT EXISTS] name | USE name
  | SHOW DATABASES | SHOW TABLES [IN db] | SHOW COLUMNS {FROM|IN} name | SHOW FUNCTIONS
  | DESCRIBE [TABLE] name | EXPLAIN [EXTENDED] statement
  | SET [key [= value]] | RESET [key]

select :=
    SELECT [DISTINCT] item [, ...]
    [FROM source [TABLESAMPLE (x PERCENT | n ROWS)] [[AS] alias]
        {[NATURAL] [INNER|LEFT [OUTER]|RIGHT [OUTER]|FULL [OUTER]|CROSS|LEFT SEMI|LEFT ANTI] JOIN source [alias]
            [ON condition | USING (col, ...)] | , source [alias]} ...
        [PIVOT (agg [AS a], ... FOR col IN (v [AS a], ...))]
        [LATERAL VIEW [OUTER] generator(...) t AS col [, ...]] ...]
    [WHERE condition]            -- incl. [NOT] EXISTS (correlated: semi / anti join), IN (select)
    [GROUP BY expr|ordinal|alias, ... [WITH ROLLUP|CUBE] | ROLLUP(...) | CUBE(...) | GROUPING SETS (...)]
    [HAVING condition] [ORDER BY expr|ordinal [ASC|DESC] [NULLS FIRST|LAST], ...]
    [LIMIT n] [OFFSET n]
    [{UNION|INTERSECT|EXCEPT|MINUS} [ALL|DISTINCT] select]

source := table | (select) | VALUES (v, ...), ... [AS t(col, ...)]

expr := literals, columns, t.col, struct.field, arr[i], map[key], + - * / % DIV, & | ^ ~,
        = == != <> < <= > >= <=>, AND OR NOT, IS [NOT] NULL, [NOT] IN (...), [NOT] BETWEEN,
        [NOT] LIKE | RLIKE | REGEXP | ILIKE, CASE [x] WHEN ... END, CAST(x AS type),
        (scalar select), function(...) [FILTER (WHERE c)] [OVER (PARTITION BY ... ORDER BY ...
        [ROWS|RANGE BETWEEN ... AND ...])], every sql.functions name plus IF / IFF / NVL / NVL2 /
        IFNULL / NULLIF / typeof / named_struct
"""

_TOKEN = re.compile(r"""
    (?P<ws>\s+|--[^\n]*)
  | (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?)
  | (?P<str>'(?:[^']|'')*')
  | (?P<qid>`[^`]+`|"[^"]+")
  | (?P<op><=>|<=|>=|<>|!=|==|\|\||[-+*/%(),.;=<>\[\]&|^~])
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
""", re.X)

KEYWORDS = {"select", "from", "where", "group", "by", "order", "having", "limit", "as", "and", "or", "not",
            "null", "is", "in", "like", "between", "distinct", "asc", "desc", "true", "false", "case", "when",
            "then", "else", "end", "cast", "join", "inner", "left", "right", "outer", "full", "cross", "on",
            "union", "all", "show", "databases", "tables", "use", "create", "database", "drop", "table", "if",
            "exists", "describe", "desc", "with"}


# non-reserved words that end a relation / select item instead of naming it
_NOT_ALIASES = {"intersect", "except", "minus", "lateral", "natural", "semi", "anti", "using", "offset", "window",
                "tablesample", "pivot", "nulls", "for", "filter"}


@dataclass
class Tok:
    kind: str
    val: str


def tokenize(sql: str) -> list[Tok]:
    out, pos = [], 0
    while pos < len(sql):
        m = _TOKEN.match(sql, pos)
        if not m:
            raise SyntaxError(f"unexpected character at {pos}: {sql[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        v = m.group(kind)
        if kind == "ws":
            continue
        if kind == "qid":
            out.append(Tok("id", v[1:-1]))
        elif kind == "id" and v.lower() in KEYWORDS:
            out.append(Tok("kw", v.lower()))
        else:
            out.append(Tok(kind, v))
    out.append(Tok("eof", ""))
    return out


def _named_windows(toks: list) -> tuple[list, dict]:
    """``WINDOW w AS (spec)[, w2 AS (spec)]`` clauses: cut out of the token stream and kept
    by name; ``OVER w`` splices the spec's tokens back in (window_spec).  The WINDOW word
    followed by ``(`` is the window() time-bucket function, not a clause."""
    def definition(i):          # toks[i] = name, toks[i+1] = AS, toks[i+2] = "(" -> index after ")"
        if not (toks[i].kind == "id" and toks[i + 1].kind == "kw" and toks[i + 1].val == "as"
                and toks[i + 2].kind == "op" and toks[i + 2].val == "("):
            return None
        j, depth = i + 2, 0
        while toks[j].kind != "eof":
            if toks[j].kind == "op" and toks[j].val in "()":
                depth += 1 if toks[j].val == "(" else -1
            j += 1
            if depth == 0:
                return j
        raise SyntaxError("unterminated WINDOW definition")

    out, named, i = [], {}, 0
    while i < len(toks):
        t = toks[i]
        if t.kind == "id" and t.val.lower() == "window" and i + 4 < len(toks) and definition(i + 1):
            i += 1
            while True:
                j = definition(i)
                named[toks[i].val.lower()] = toks[i + 2:j]
                i = j
                if toks[i].kind == "op" and toks[i].val == "," and definition(i + 1):
                    i += 1
                    continue
                break
            continue
        out.append(t)
        i += 1
    return out, named


@dataclass
class SelectItem:
    expr: object            # Expr | AggCall | "*"
    alias: str | None = None


@dataclass
class AggCall:
    fn: str
    arg: object             # Expr or None (count(*))
    distinct: bool = False
    text: str = ""
    built: object = None    # prebuilt frame Agg (statistical / two-argument aggregates)


# SQL aggregates built through sql.functions (arguments after the first are literals)
_EXTRA_AGGS = {"first", "last", "collect_list", "collect_set", "stddev_pop", "var_pop", "skewness",
               "kurtosis", "approx_count_distinct", "corr", "covar_pop", "covar_samp", "percentile_approx",
               "percentile", "grouping", "grouping_id", "median", "mode", "product", "count_if", "bool_and",
               "bool_or", "every", "some", "any_value", "max_by", "min_by", "bit_and", "bit_or", "bit_xor",
               "array_agg", "histogram_numeric"}
_TWO_COLUMN_AGGS = {"corr", "covar_pop", "covar_samp", "max_by", "min_by"}


@dataclass
class Join:
    table: str | None
    alias: str | None
    how: str
    on: object
    using: list | None = None           # JOIN ... USING (a, b)
    natural: bool = False               # NATURAL JOIN: USING every common column
    subquery: object = None             # JOIN (SELECT ...) alias


@dataclass
class Lateral:
    gen: object                         # generator Expr (explode / posexplode / inline ...)
    names: list                         # output column names
    outer: bool = False


@dataclass
class Select:
    items: list
    table: str | None = None
    alias: str | None = None
    subquery: object = None
    joins: list = field(default_factory=list)
    where: object = None
    group_by: list = field(default_factory=list)
    having: object = None
    order_by: list = field(default_factory=list)
    limit: int | None = None
    offset: int | None = None
    grouping: str | None = None          # "rollup" | "cube" | "sets"
    grouping_sets: list | None = None    # index tuples into group_by (GROUPING SETS)
    distinct: bool = False
    ctes: list = field(default_factory=list)        # WITH name AS (select), ...
    values: list | None = None           # FROM VALUES (..), (..) [AS t(a, b)]
    value_names: list | None = None
    laterals: list = field(default_factory=list)    # LATERAL VIEW [OUTER] gen(..) t AS c
    sample: tuple | None = None          # TABLESAMPLE (x PERCENT | n ROWS)
    pivot: tuple | None = None           # PIVOT (aggs FOR col IN (values))


@dataclass
class SetOp:
    """``left {UNION|INTERSECT|EXCEPT} [ALL] right`` -- a node of a query expression.

    Chains are left-associative and INTERSECT binds tighter than UNION / EXCEPT (SQL
    standard, Spark's grammar); a trailing ORDER BY / LIMIT / OFFSET after the last branch
    applies to the combined result."""
    op: str                              # union | intersect | except
    all: bool
    left: object                         # Select | SetOp
    right: object
    order_by: list = field(default_factory=list)
    limit: int | None = None
    offset: int | None = None
    ctes: list = field(default_factory=list)


class Parser:
    def __init__(self, sql: str):
        self.toks, self.windows = _named_windows(tokenize(sql))
        self.i = 0
        self.src = sql

    # -- helpers ---------------------------------------------------------------
    def peek(self, k=0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def next(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind, val=None) -> Tok | None:
        t = self.peek()
        if t.kind == kind and (val is None or t.val == val):
            self.i += 1
            return t
        return None

    def expect(self, kind, val=None) -> Tok:
        t = self.accept(kind, val)
        if t is None:
            p = self.peek()
            raise SyntaxError(f"expected {val or kind} but found {p.val!r}")
        return t

    def idw(self, *words) -> bool:
        """Non-reserved words (ROLLUP, CUBE, SETS, OFFSET, ...) arrive as identifiers."""
        for k, w in enumerate(words):
            t = self.peek(k)
            if not (t.kind == "id" and t.val.lower() == w):
                return False
        self.i += len(words)
        return True

    def _expr_list(self) -> list:
        self.expect("op", "(")
        out = []
        if not self.accept("op", ")"):
            out.append(self.expr())
            while self.accept("op", ","):
                out.append(self.expr())
            self.expect("op", ")")
        return out

    def kw(self, *words) -> bool:
        for k, w in enumerate(words):
            t = self.peek(k)
            if not (t.kind == "kw" and t.val == w):
                return False
        self.i += len(words)
        return True

    def ident(self) -> str:
        t = self.next()
        if t.kind not in ("id", "kw"):
            raise SyntaxError(f"expected identifier, found {t.val!r}")
        return t.val

    def qualified(self) -> str:
        name = self.ident()
        while self.accept("op", "."):
            name += "." + self.ident()
        return name

    # -- statements --------------------------------------------------------------
    def statement(self):
        if self.kw("show", "databases"):
            return ("show_databases",)
        if self.kw("show", "tables"):
            db = None
            if self.kw("in") or self.kw("from"):
                db = self.ident()
            return ("show_tables", db)
        if self.kw("use"):
            return ("use", self.ident())
        if self.idw("set"):                          # SET / SET key / SET key = value
            if self.peek().kind == "eof":
                return ("set", None, None)
            start = self.i
            while self.peek().kind != "eof" and not (self.peek().kind == "op" and self.peek().val == "="):
                self.i += 1
            key = "".join(t.val for t in self.toks[start:self.i])
            if self.accept("op", "="):
                raw = self.src.split("=", 1)[1].strip().rstrip(";").strip()
                self.i = len(self.toks) - 1
                return ("set", key, raw.strip("'\""))
            return ("set", key, None)
        if self.idw("reset"):
            key = "".join(t.val for t in self.toks[self.i:-1]) or None
            self.i = len(self.toks) - 1
            return ("reset", key)
        if self.idw("truncate"):
            self.kw("table")
            return ("truncate", self.qualified())
        if self.idw("alter"):
            self.kw("table") or self.idw("view")
            name = self.qualified()
            if not (self.idw("rename") and self.idw("to")):
                raise SyntaxError("only ALTER TABLE ... RENAME TO ... is supported")
            return ("rename", name, self.qualified())
        if self.peek().kind == "kw" and self.peek().val == "drop" and self.peek(1).kind == "id" and \
                self.peek(1).val.lower() == "view":
            self.i += 2
            ie = self.kw("if", "exists")
            return ("drop_view", self.qualified(), ie)
        if self.kw("show") and self.idw("columns"):
            if not (self.kw("in") or self.kw("from")):
                raise SyntaxError("expected FROM / IN after SHOW COLUMNS")
            name = self.qualified()
            if self.kw("in") or self.kw("from"):
                name = self.ident() + "." + name
            return ("show_columns", name)
        if self.peek(-1).val == "show" and self.idw("functions"):
            return ("show_functions",)
        if self.idw("explain"):
            self.idw("extended") or self.idw("formatted") or self.idw("codegen")
            start = self.i
            inner = self.statement()
            return ("explain", inner, " ".join(t.val for t in self.toks[start:-1]))
        if self.idw("cache"):
            lazy = bool(self.idw("lazy"))
            self.kw("table")
            name = self.qualified()
            sel = self.select() if self.kw("as") else None
            return ("cache", name, sel, lazy)
        if self.idw("uncache"):
            self.kw("table")
            self.kw("if", "exists")
            return ("uncache", self.qualified())
        if self.idw("refresh"):
            self.kw("table")
            return ("refresh", self.qualified())
        if self.kw("create", "database"):
            ine = self.kw("if", "not", "exists")
            return ("create_database", self.ident(), ine)
        if self.kw("drop", "table"):
            ie = self.kw("if", "exists")
            return ("drop_table", self.qualified(), ie)
        if self.kw("drop", "database"):
            ie = self.kw("if", "exists")
            return ("drop_database", self.ident(), ie)
        if self.kw("describe") or self.kw("desc"):
            self.kw("table")
            return ("describe", self.qualified())
        if self.kw("create", "table"):
            name = self.qualified()
            self.expect("kw", "as")
            return ("ctas", name, self.select())
        if self.peek().kind == "kw" and self.peek().val == "create":
            save = self.i
            self.i += 1
            replace = self.kw("or") and self.idw("replace")
            glob = self.idw("global")
            temp = self.idw("temporary") or self.idw("temp")
            if self.idw("view"):
                self.kw("if", "not", "exists")
                name = self.qualified()
                self.expect("kw", "as")
                sel = self.select()
                self.accept("op", ";")
                return ("create_view", name, sel, glob, replace or not temp)
            self.i = save
        if self.idw("insert"):
            overwrite = bool(self.idw("overwrite"))
            if not overwrite:
                if not self.idw("into"):
                    raise SyntaxError("expected INTO or OVERWRITE after INSERT")
            self.kw("table")
            name = self.qualified()
            cols = None
            if self.peek().val == "(" and not (self.peek(1).kind == "kw" and self.peek(1).val == "select"):
                self.expect("op", "(")
                cols = [self.ident()]
                while self.accept("op", ","):
                    cols.append(self.ident())
                self.expect("op", ")")
            if self.idw("values"):
                src = ("values", self._values_rows())
            else:
                src = ("select", self.select())
            self.accept("op", ";")
            return ("insert", name, cols, src, overwrite)
        ctes = []
        if self.kw("with"):
            while True:
                cname = self.ident()
                self.expect("kw", "as")
                self.expect("op", "(")
                ctes.append((cname, self.select()))
                self.expect("op", ")")
                if not self.accept("op", ","):
                    break
        sel = self.select()
        sel.ctes = ctes
        self.accept("op", ";")
        if self.peek().kind != "eof":
            raise SyntaxError(f"unexpected trailing input: {self.peek().val!r}")
        return ("select", sel)

    def select(self):
        """query := term ((UNION | EXCEPT | MINUS) [ALL | DISTINCT] term)* [ORDER BY / LIMIT / OFFSET]
        term := primary (INTERSECT [ALL | DISTINCT] primary)*
        primary := SELECT ... | '(' query ')'"""
        node = self._set_term()
        while True:
            if self.kw("union"):
                op = "union"
            elif self.idw("except") or self.idw("minus"):
                op = "except"
            else:
                break
            is_all = bool(self.kw("all"))
            if not is_all:
                self.kw("distinct")
            node = SetOp(op, is_all, node, self._set_term())
        if isinstance(node, SetOp):
            self._lift_tail(node)
        return node

    def _set_term(self):
        node = self._set_primary()
        while self.idw("intersect"):
            is_all = bool(self.kw("all"))
            if not is_all:
                self.kw("distinct")
            node = SetOp("intersect", is_all, node, self._set_primary())
        return node

    def _set_primary(self):
        if self.peek().kind == "op" and self.peek().val == "(" and self.peek(1).val == "select":
            self.next()
            q = self.select()
            self.expect("op", ")")
            return q
        return self._select_core()

    @staticmethod
    def _lift_tail(node: "SetOp") -> None:
        """ORDER BY / LIMIT / OFFSET parsed with the rightmost SELECT belong to the whole
        set operation (a branch needs parentheses to own them)."""
        last = node
        while isinstance(last, SetOp):
            last = last.right
        if isinstance(last, Select) and (last.order_by or last.limit is not None or last.offset is not None):
            node.order_by, node.limit, node.offset = last.order_by, last.limit, last.offset
            last.order_by, last.limit, last.offset = [], None, None

    def _select_core(self) -> Select:
        self.expect("kw", "select")
        distinct = bool(self.kw("distinct"))
        items = [self.select_item()]
        while self.accept("op", ","):
            items.append(self.select_item())
        s = Select(items, distinct=distinct)
        if self.kw("from"):
            if self.idw("values"):
                s.values = self._values_rows()
                s.alias, s.value_names = self._table_alias()
            else:
                if self.accept("op", "("):
                    s.subquery = self.select()
                    self.expect("op", ")")
                else:
                    s.table = self.qualified()
                if self.idw("tablesample"):
                    self.expect("op", "(")
                    n = float(self.expect("num").val)
                    unit = self.ident().lower()
                    self.expect("op", ")")
                    s.sample = ("percent" if unit == "percent" else "rows", n)
                s.alias = self._alias()
            while True:
                how, natural = None, False
                if self.accept("op", ","):                 # FROM a, b  == CROSS JOIN
                    how = "cross"
                else:
                    natural = bool(self.idw("natural"))
                    if self.kw("join") or self.kw("inner", "join"):
                        how = "inner"
                    elif self.kw("left", "outer", "join") or self.kw("left", "join"):
                        how = "left"
                    elif self.kw("right", "outer", "join") or self.kw("right", "join"):
                        how = "right"
                    elif self.kw("full", "outer", "join") or self.kw("full", "join"):
                        how = "outer"
                    elif self.kw("cross", "join"):
                        how = "cross"
                    elif self.peek().val == "left" and self.peek(1).kind == "id" and \
                            self.peek(1).val.lower() in ("semi", "anti") and self.peek(2).val == "join":
                        how = "left_" + self.peek(1).val.lower()
                        self.i += 3
                    elif self.peek().kind == "id" and self.peek().val.lower() in ("semi", "anti") and \
                            self.peek(1).val == "join":
                        how = "left_" + self.peek().val.lower()
                        self.i += 2
                    elif natural:
                        raise SyntaxError("expected JOIN after NATURAL")
                if how is None:
                    break
                sub = t = None
                if self.accept("op", "("):
                    sub = self.select()
                    self.expect("op", ")")
                else:
                    t = self.qualified()
                al = self._alias()
                on = using = None
                if natural:
                    pass
                elif how != "cross" and self.idw("using"):
                    self.expect("op", "(")
                    using = [self.ident()]
                    while self.accept("op", ","):
                        using.append(self.ident())
                    self.expect("op", ")")
                elif how != "cross":
                    self.expect("kw", "on")
                    on = self.expr()
                s.joins.append(Join(t, al, how, on, using, natural, sub))
            if self.idw("pivot"):
                s.pivot = self._pivot_clause()
            while self.idw("lateral", "view"):
                outer = bool(self.kw("outer"))
                gen = self.primary()
                self.ident()                                # table alias of the generator
                names = []
                if self.kw("as"):
                    names.append(self.ident())
                    while self.accept("op", ","):
                        names.append(self.ident())
                s.laterals.append(Lateral(gen, names, outer))
        if self.kw("where"):
            s.where = self.expr()
        if self.kw("group", "by"):
            if self.idw("rollup") or self.idw("cube"):
                s.grouping = self.toks[self.i - 1].val.lower()
                s.group_by = self._expr_list()
            elif self.idw("grouping", "sets"):
                self.expect("op", "(")
                sets = []
                while True:
                    sets.append(self._expr_list() if self.peek().val == "(" else [self.expr()])
                    if not self.accept("op", ","):
                        break
                self.expect("op", ")")
                names: dict = {}
                for st in sets:
                    for e in st:
                        names.setdefault(e.name, e)
                order = list(names)
                s.group_by = list(names.values())
                s.grouping = "sets"
                s.grouping_sets = [tuple(sorted(order.index(e.name) for e in st)) for st in sets]
            else:
                s.group_by = [self.expr()]
                while self.accept("op", ","):
                    s.group_by.append(self.expr())
                if self.peek().kind == "kw" and self.peek().val == "with" and \
                        self.peek(1).kind == "id" and self.peek(1).val.lower() in ("rollup", "cube"):
                    self.i += 2
                    s.grouping = self.toks[self.i - 1].val.lower()
        if self.kw("having"):
            s.having = self.expr(allow_agg=True)
        if self.kw("order", "by"):
            s.order_by = [self.order_item()]
            while self.accept("op", ","):
                s.order_by.append(self.order_item())
        if self.kw("limit"):
            s.limit = int(float(self.expect("num").val))
        if self.idw("offset"):
            s.offset = int(float(self.expect("num").val))
        return s

    def _values_rows(self) -> list:
        """VALUES (1, 'a'), (2, 'b')  (or bare scalars: VALUES 1, 2) -> rows of python values."""
        rows = []
        while True:
            if self.accept("op", "("):
                row = [self._value_literal()]
                while self.accept("op", ","):
                    row.append(self._value_literal())
                self.expect("op", ")")
            else:
                row = [self._value_literal()]
            rows.append(row)
            if not self.accept("op", ","):
                return rows

    def _value_literal(self):
        if self.kw("null"):
            return None
        return self.literal_value()

    def _table_alias(self):
        """[AS] name [(col, ...)] after an inline table."""
        name = self._alias()
        cols = None
        if name is not None and self.accept("op", "("):
            cols = [self.ident()]
            while self.accept("op", ","):
                cols.append(self.ident())
            self.expect("op", ")")
        return name, cols

    def _alias(self):
        if self.kw("as"):
            return self.ident()
        t = self.peek()
        if t.kind == "id" and t.val.lower() not in _NOT_ALIASES:
            self.i += 1
            return t.val
        return None

    def select_item(self) -> SelectItem:
        if self.accept("op", "*"):
            return SelectItem("*")
        if self.peek().kind == "id" and self.peek(1).val == "." and self.peek(2).val == "*":
            self.i += 3
            return SelectItem("*")
        e = self.expr(allow_agg=True)
        return SelectItem(e, self._alias())

    def order_item(self):
        e = self.expr(allow_agg=True)
        asc = True
        if self.kw("desc"):
            asc = False
        else:
            self.kw("asc")
        if self.idw("nulls"):
            first = bool(self.idw("first"))
            if not first and not self.idw("last"):
                raise SyntaxError("expected FIRST or LAST after NULLS")
            if not _is_agg(e):
                e = (e.asc_nulls_first() if first else e.asc_nulls_last()) if asc else \
                    (e.desc_nulls_first() if first else e.desc_nulls_last())
                asc = True                           # direction now carried by the sort expression
        return (e, asc)

    def _pivot_clause(self):
        """PIVOT (agg [AS a], ... FOR col IN (v [AS name], ...))."""
        self.expect("op", "(")
        aggs = []
        while True:
            a = self.expr(allow_agg=True)
            aggs.append((a, self._alias()))
            if not self.accept("op", ","):
                break
        if not self.idw("for"):
            raise SyntaxError("expected FOR in PIVOT")
        col = self.ident()
        self.expect("kw", "in")
        self.expect("op", "(")
        vals = []
        while True:
            v = self._value_literal()
            vals.append((v, self._alias()))
            if not self.accept("op", ","):
                break
        self.expect("op", ")")
        self.expect("op", ")")
        return (aggs, col, vals)

    # -- expressions -------------------------------------------------------------
    def expr(self, allow_agg=False):
        self._allow_agg = allow_agg
        return self.or_expr()

    def or_expr(self):
        e = self.and_expr()
        while self.kw("or"):
            e = _combine(e, self.and_expr(), lambda a, b: a | b)
        return e

    def and_expr(self):
        e = self.not_expr()
        while self.kw("and"):
            e = _combine(e, self.not_expr(), lambda a, b: a & b)
        return e

    def not_expr(self):
        if self.peek().kind == "kw" and self.peek().val == "not" and self.peek(1).val == "exists":
            self.i += 2
            return self._exists(True)
        if self.kw("not"):
            return _unary_map(self.not_expr(), lambda a: ~a)
        return self.cmp_expr()

    def bit_or(self):
        """a | b  <  a ^ b  <  a & b  <  + -   (Spark's bitwise operator precedence)."""
        e = self.bit_xor()
        while self.peek().kind == "op" and self.peek().val == "|":
            self.i += 1
            e = _combine(e, self.bit_xor(), lambda a, b: a.bitwiseOR(b))
        return e

    def bit_xor(self):
        e = self.bit_and()
        while self.peek().kind == "op" and self.peek().val == "^":
            self.i += 1
            e = _combine(e, self.bit_and(), lambda a, b: a.bitwiseXOR(b))
        return e

    def bit_and(self):
        e = self.add_expr()
        while self.peek().kind == "op" and self.peek().val == "&":
            self.i += 1
            e = _combine(e, self.add_expr(), lambda a, b: a.bitwiseAND(b))
        return e

    def cmp_expr(self):
        e = self.bit_or()
        t = self.peek()
        if t.kind == "op" and t.val == "<=>":                 # null-safe equality
            self.i += 1
            r = self.bit_or()
            return _combine(e, r, lambda a, b: a.eqNullSafe(b))
        if t.kind == "op" and t.val in ("=", "==", "!=", "<>", "<", "<=", ">", ">="):
            self.i += 1
            r = self.bit_or()
            op = {"=": "__eq__", "==": "__eq__", "!=": "__ne__", "<>": "__ne__", "<": "__lt__", "<=": "__le__",
                  ">": "__gt__", ">=": "__ge__"}[t.val]
            return _combine(e, r, lambda a, b: getattr(a, op)(b))
        if self.kw("is"):
            neg = self.kw("not")
            self.expect("kw", "null")
            return _unary_map(e, (lambda a: a.isNotNull()) if neg else (lambda a: a.isNull()))
        neg = False
        if self.peek().kind == "kw" and self.peek().val == "not" and \
                self.peek(1).val.lower() in ("in", "like", "between", "rlike", "regexp", "ilike"):
            self.i += 1
            neg = True
        if self.kw("in"):
            self.expect("op", "(")
            if self.peek().kind == "kw" and self.peek().val == "select":
                sub = self.select()
                self.expect("op", ")")
                r = _unary_map(e, lambda a: _in_subquery(a, sub))
                return _unary_map(r, lambda a: ~a) if neg else r
            vals = [self.literal_value()]
            while self.accept("op", ","):
                vals.append(self.literal_value())
            self.expect("op", ")")
            r = _unary_map(e, lambda a: a.isin(vals))
            return _unary_map(r, lambda a: ~a) if neg else r
        if self.kw("like"):
            pat = self.expect("str").val[1:-1].replace("''", "'")
            r = _unary_map(e, lambda a: a.like(pat))
            return _unary_map(r, lambda a: ~a) if neg else r
        if self.peek().kind == "id" and self.peek().val.lower() in ("rlike", "regexp", "ilike"):
            op = self.next().val.lower()
            pat = self.expect("str").val[1:-1].replace("''", "'")
            r = _unary_map(e, (lambda a: a.ilike(pat)) if op == "ilike" else (lambda a: a.rlike(pat)))
            return _unary_map(r, lambda a: ~a) if neg else r
        if self.kw("between"):
            lo = self.add_expr()
            self.expect("kw", "and")
            hi = self.add_expr()
            r = _combine(_combine(e, lo, lambda a, b: a >= b), _combine(e, hi, lambda a, b: a <= b),
                         lambda a, b: a & b)
            return _unary_map(r, lambda a: ~a) if neg else r
        return e

    def _exists(self, neg: bool):
        self.expect("op", "(")
        allow = self._allow_agg
        sub = self.select()
        self._allow_agg = allow
        self.expect("op", ")")
        return ExistsExpr(sub, neg)

    def literal_value(self):
        t = self.next()
        if t.kind == "num":
            return float(t.val) if any(c in t.val for c in ".eE") else int(t.val)
        if t.kind == "str":
            return t.val[1:-1].replace("''", "'")
        if t.kind == "op" and t.val == "-":
            v = self.literal_value()
            return -v
        if t.kind == "kw" and t.val in ("true", "false"):
            return t.val == "true"
        raise SyntaxError(f"expected literal, found {t.val!r}")

    def add_expr(self):
        e = self.mul_expr()
        while self.peek().kind == "op" and self.peek().val in ("+", "-", "||"):
            op = self.next().val
            r = self.mul_expr()
            e = _combine(e, r, (lambda a, b: a + b) if op in ("+", "||") else (lambda a, b: a - b))
        return e

    def mul_expr(self):
        e = self.unary()
        while (self.peek().kind == "op" and self.peek().val in ("*", "/", "%")) or \
                (self.peek().kind == "id" and self.peek().val.lower() == "div"):
            op = self.next().val.lower()
            r = self.unary()
            e = _combine(e, r, {"*": lambda a, b: a * b, "/": lambda a, b: a / b, "%": lambda a, b: a % b,
                                "div": _int_div}[op])
        return e

    def unary(self):
        if self.accept("op", "-"):
            return _unary_map(self.unary(), lambda a: -a)
        if self.accept("op", "~"):
            from . import functions as F
            return _unary_map(self.unary(), F.bitwise_not)
        if self.accept("op", "+"):
            return self.unary()
        e = self.primary()
        while self.accept("op", "["):                 # arr[i] (0-based) / map[key]
            k = self.or_expr()
            self.expect("op", "]")
            e = _subscript(e, k)
        return e

    def primary(self):
        t = self.peek()
        if t.kind == "num":
            self.i += 1
            v = float(t.val) if any(c in t.val for c in ".eE") else int(t.val)
            return E.lit(v)
        if t.kind == "str":
            self.i += 1
            return E.lit(t.val[1:-1].replace("''", "'"))
        if t.kind == "kw" and t.val in ("null", "true", "false"):
            self.i += 1
            return E.lit(None if t.val == "null" else t.val == "true")
        if self.accept("op", "("):
            if self.peek().kind == "kw" and self.peek().val == "select":
                sub = self.select()
                self.expect("op", ")")
                return _scalar_subquery(sub)
            e = self.or_expr()
            self.expect("op", ")")
            return e
        if self.kw("exists"):
            return self._exists(False)
        if self.kw("cast"):
            self.expect("op", "(")
            e = self.or_expr()
            self.expect("kw", "as")
            ty = self.ident()
            if self.accept("op", "("):
                while not self.accept("op", ")"):
                    self.next()
            self.expect("op", ")")
            if ty.lower() in ("date", "timestamp"):
                from . import functions as F
                return _unary_map(e, F.to_date if ty.lower() == "date" else F.to_timestamp)
            return _unary_map(e, lambda a: a.cast(ty))
        if self.kw("case"):
            cases = []
            operand = None if (self.peek().kind == "kw" and self.peek().val == "when") else self.or_expr()
            while self.kw("when"):
                c = self.or_expr()
                if operand is not None:                  # CASE x WHEN v THEN ...
                    c = operand == c
                self.expect("kw", "then")
                v = self.or_expr()
                cases.append((c, v))
            default = None
            if self.kw("else"):
                default = self.or_expr()
            self.expect("kw", "end")
            w = E.when(cases[0][0], cases[0][1])
            for c, v in cases[1:]:
                w = w.when(c, v)
            return w.otherwise(default) if default is not None else w.otherwise(None)
        if t.kind in ("id", "kw"):
            name = self.ident()
            if self.accept("op", "("):
                return self.func_call(name)
            qual = None
            while self.peek().val == "." and self.peek(1).kind in ("id", "kw"):
                self.i += 1
                qual, name = name, self.ident()   # qualified column: relation part picks a join side
            return E.col(name) if qual is None else E.qualified_col(qual, name)
        raise SyntaxError(f"unexpected token {t.val!r}")

    def word(self, *words) -> bool:
        """Case-insensitive match of non-reserved words (OVER, PARTITION, ROWS, ...)."""
        for k, w in enumerate(words):
            t = self.peek(k)
            if not (t.kind in ("id", "kw") and t.val.lower() == w):
                return False
        self.i += len(words)
        return True

    def func_call(self, name):
        f = self._func_call(name)
        if self.word("over"):
            return self.window_spec(f)
        return f

    def _frame_bound(self):
        from .window import currentRow, unboundedFollowing, unboundedPreceding
        if self.word("unbounded", "preceding"):
            return unboundedPreceding
        if self.word("unbounded", "following"):
            return unboundedFollowing
        if self.word("current", "row"):
            return currentRow
        x = float(self.expect("num").val)
        n = int(x) if x.is_integer() else x       # RANGE frames take fractional value offsets
        if self.word("preceding"):
            return -n
        if self.word("following"):
            return n
        raise SyntaxError("expected PRECEDING or FOLLOWING")

    def window_spec(self, f):
        """``<function> OVER ([PARTITION BY e, ...] [ORDER BY e [ASC|DESC], ...]
        [ROWS|RANGE BETWEEN <bound> AND <bound>])``."""
        from .window import WindowExpr, WindowFunction, WindowSpec
        t = self.peek()
        if t.kind == "id" and t.val.lower() in self.windows:          # OVER w (named WINDOW clause)
            self.toks[self.i:self.i + 1] = list(self.windows[t.val.lower()])
        self.expect("op", "(")
        spec = WindowSpec()
        if self.word("partition", "by"):
            parts = [self.or_expr()]
            while self.accept("op", ","):
                parts.append(self.or_expr())
            spec = spec.partitionBy(*parts)
        if self.kw("order", "by"):
            items = [self.order_item()]
            while self.accept("op", ","):
                items.append(self.order_item())
            spec = spec.orderBy(*[e if a else e.desc() for e, a in items])
        for kind in ("rows", "range"):
            if self.word(kind):
                self.kw("between")
                lo = self._frame_bound()
                self.kw("and")
                hi = self._frame_bound()
                spec = spec.rowsBetween(lo, hi) if kind == "rows" else spec.rangeBetween(lo, hi)
        self.expect("op", ")")
        if isinstance(f, AggCall):
            f = f.built if f.built is not None else E.Agg(f.fn, f.arg, f.text, f.distinct)
        if not isinstance(f, (E.Agg, WindowFunction)):
            raise SyntaxError("OVER applies to aggregate or window functions")
        return WindowExpr(f, spec, f"{f.name} OVER (...)")

    def _func_call(self, name):
        from . import window as W
        fn = name.lower()
        if fn in ("row_number", "rank", "dense_rank", "percent_rank", "cume_dist"):
            self.expect("op", ")")
            return getattr(W, fn)()
        if fn == "extract" and self.peek().kind in ("id", "kw") and self.peek(1).kind == "kw" \
                and self.peek(1).val == "from":
            from . import functions as F                          # EXTRACT(field FROM source)
            field = self.next().val
            self.next()
            src = self.or_expr()
            self.expect("op", ")")
            return F.date_part(E.lit(field), src).alias(f"extract({field} FROM {src.name})")
        if fn in ("ntile", "lag", "lead", "first_value", "last_value"):
            args = [self.or_expr()]
            while self.accept("op", ","):
                args.append(self.or_expr())
            self.expect("op", ")")
            if fn == "ntile":
                return W.ntile(int(args[0].eval_literal()))
            if fn in ("first_value", "last_value"):
                return E.Agg("first" if fn == "first_value" else "last", args[0], f"{fn}({args[0].name})")
            off = int(args[1].eval_literal()) if len(args) > 1 else 1
            default = args[2].eval_literal() if len(args) > 2 else None
            return (W.lag if fn == "lag" else W.lead)(args[0], off, default)
        if fn in ("count", "sum", "avg", "mean", "min", "max", "stddev", "stddev_samp", "variance", "var_samp"):
            distinct = bool(self.kw("distinct"))
            if self.accept("op", "*"):
                arg = None
            else:
                arg = self.or_expr()
            self.expect("op", ")")
            canon = {"mean": "avg", "stddev_samp": "stddev", "var_samp": "variance"}.get(fn, fn)
            text = f"{canon}({'DISTINCT ' if distinct else ''}{'1' if arg is None else arg.name})"
            if canon == "count" and arg is None:
                text = "count(1)"
            if self.peek().kind == "id" and self.peek().val.lower() == "filter" and self.peek(1).val == "(":
                self.i += 2                          # agg(x) FILTER (WHERE cond): rows failing cond ignored
                self.expect("kw", "where")
                cond = self.or_expr()
                self.expect("op", ")")
                arg = E.when(cond, E.lit(1) if arg is None else arg)
                text = f"{text} FILTER (WHERE {cond.name})"
            return AggCall(canon, arg, distinct, text)
        args = []
        if not self.accept("op", ")"):
            args.append(self.or_expr())
            while self.accept("op", ","):
                args.append(self.or_expr())
            self.expect("op", ")")
        if fn in _EXTRA_AGGS:
            from . import functions as F
            ncol = 2 if fn in _TWO_COLUMN_AGGS else (len(args) if fn == "grouping_id" else min(1, len(args)))
            lits = [a.eval_literal() for a in args[ncol:]]
            text = f"{fn}({', '.join(a.name for a in args)})"
            return AggCall(fn, args[0] if args else None, False, text, getattr(F, fn)(*args[:ncol], *lits))
        f = {"sqrt": E.sqrt, "log": E.log, "ln": E.log, "exp": E.exp, "abs": E.abs, "isnan": E.isnan,
             "coalesce": E.coalesce, "log1p": E.log1p}.get(fn)
        if f is None:
            if fn in ("lower", "upper", "length", "trim"):
                return _string_fn(fn, args[0])
            if fn in ("floor", "ceil"):
                return _math_fn(fn, args)
            return _resolve_function(name, fn, args)
        return f(*args)


_SCALAR_ANN = {"int", "str", "bool", "float", "int | None", "str | None"}
_SCALAR_NAMES = {"value", "format", "sep", "pattern", "replacement", "idx", "pos", "length_", "n", "pad", "d",
                 "numBits", "scale", "days", "limit", "substr", "asc", "i", "seed"}


def _int_div(a, b):
    """a DIV b: integral quotient truncated toward zero (Spark), NULL on division by zero."""
    def f(df):
        import torch
        from ..frame import column as C
        x, y = a.eval(df), b.eval(df)
        xd, yd = x.data.to(torch.float64), y.data.to(torch.float64)
        q = torch.trunc(xd / torch.where(yd == 0, torch.ones_like(yd), yd)).to(torch.int64)
        valid = yd != 0
        for c in (x, y):
            if getattr(c, "valid", None) is not None:
                valid = valid & c.valid
        return C.NumericColumn(q, None if bool(valid.all()) else valid)
    return E.Expr(f, f"({a.name} DIV {b.name})", a.refs + b.refs)


def _subscript(base, key):
    """SQL ``base[key]``: 0-based array element, map value, or vector component."""
    def f(df):
        from ..frame import column as C
        from ..frame.dataframe import _nullable_column
        c = base.eval(df)
        k = key.eval_literal() if hasattr(key, "_literal") else None
        if isinstance(c, (C.VectorColumn, C.SparseVectorColumn)):
            return base.getItem(int(k)).eval(df)
        keys = [k] * len(c) if k is not None else key.eval(df).to_pylist()
        out = []
        for v, kk in zip(c.to_pylist(), keys):
            if v is None or kk is None:
                out.append(None)
            elif isinstance(v, dict):
                out.append(v.get(kk))
            else:
                i = int(kk)
                out.append(v[i] if 0 <= i < len(v) else None)
        return _nullable_column(out)
    return E.Expr(f, f"{base.name}[{key.name}]", base.refs + key.refs)


def _typeof(e):
    def f(df):
        import numpy as np
        from ..frame import column as C
        c = e.eval(df)
        return C.StringColumn(np.array([c.dtype.simpleString()] * len(c), dtype=object))
    return E.Expr(f, f"typeof({e.name})", e.refs)


def _named_struct(*args):
    from . import functions as F
    if len(args) % 2:
        raise SyntaxError("named_struct expects name, value pairs")
    return F.struct(*[v.alias(k.eval_literal()) for k, v in zip(args[::2], args[1::2])])


# SQL-only spellings (Hive / Spark SQL built-ins without a pyspark.sql.functions twin)
_SQL_ONLY = {
    "if": lambda c, a, b: E.when(c, a).otherwise(b),
    "iff": lambda c, a, b: E.when(c, a).otherwise(b),
    "nvl": lambda a, b: E.coalesce(a, b),
    "ifnull": lambda a, b: E.coalesce(a, b),
    "nvl2": lambda a, b, c: E.when(a.isNotNull(), b).otherwise(c),
    "nullif": lambda a, b: E.when(a == b, E.lit(None)).otherwise(a),
    "typeof": _typeof,
    "named_struct": _named_struct,
}


def _resolve_function(name, fn, args):
    """Registered UDFs (spark.udf.register), then any ``sql.functions`` function by name.
    Literal arguments bound to scalar parameters (``substring(s, 1, 3)``) are passed as
    Python values, column arguments as expressions."""
    import inspect
    from . import functions as F
    from .udf import lookup
    u = lookup(fn)
    if u is not None:
        return u(*args)
    if fn in _SQL_ONLY:
        return _SQL_ONLY[fn](*args)
    g = getattr(F, fn, None)
    if fn.startswith("_") or not callable(g) or isinstance(g, type):
        raise SyntaxError(f"unknown function {name}")
    try:
        params = list(inspect.signature(g).parameters.values())
    except (TypeError, ValueError):
        params = []
    call = []
    for i, a in enumerate(args):
        p = params[i] if i < len(params) else (params[-1] if params else None)
        scalar = p is not None and p.kind is not inspect.Parameter.VAR_POSITIONAL and (
            str(p.annotation) in _SCALAR_ANN or p.name in _SCALAR_NAMES)
        if scalar and hasattr(a, "_literal"):
            call.append(a.eval_literal())
        else:
            call.append(a)
    return g(*call)


def _is_agg(x):
    return isinstance(x, AggCall) or isinstance(x, _AggExpr)


class _AggExpr:
    """Expression over aggregate results (e.g. ``sum(x) / count(*)``), resolved after grouping."""

    def __init__(self, aggs: list, build, text: str):
        self.aggs, self.build, self.text = aggs, build, text

    @property
    def name(self):
        return self.text


def _as_agg_expr(x):
    if isinstance(x, _AggExpr):
        return x
    if isinstance(x, AggCall):
        return _AggExpr([x], lambda m: E.col(m[x.text]), x.text)
    return _AggExpr([], lambda m: x, x.name if hasattr(x, "name") else str(x))


def _combine(a, b, f):
    if _is_agg(a) or _is_agg(b):
        A, B = _as_agg_expr(a), _as_agg_expr(b)
        return _AggExpr(A.aggs + B.aggs, lambda m: f(A.build(m), B.build(m)), f"({A.text} ? {B.text})")
    return f(a, b)


def _unary_map(a, f):
    if _is_agg(a):
        A = _as_agg_expr(a)
        return _AggExpr(A.aggs, lambda m: f(A.build(m)), A.text)
    return f(a)


def _string_fn(fn, e):
    import numpy as np
    from ..frame import column as C

    def run(df):
        c = e.eval(df)
        vals = c.to_pylist()
        if fn == "length":
            import torch
            return C.NumericColumn(torch.tensor([len(v) if v is not None else 0 for v in vals], dtype=torch.int32))
        op = {"lower": str.lower, "upper": str.upper, "trim": str.strip}[fn]
        return C.StringColumn(np.array([None if v is None else op(str(v)) for v in vals], dtype=object))
    return E.Expr(run, f"{fn}({e.name})", e.refs)


def _math_fn(fn, args):
    import torch
    from ..frame import column as C
    e = args[0]
    nd = 0
    if len(args) > 1:
        nd = int(args[1]._fn.__closure__ and 0 or 0)

    def run(df):
        c = e.eval(df)
        d = c.data.to(torch.float64)
        if fn == "floor":
            d = torch.floor(d)
        elif fn == "ceil":
            d = torch.ceil(d)
        else:
            d = torch.round(d, decimals=nd)
        return C.NumericColumn(d, c.valid)
    return E.Expr(run, f"{fn}({e.name})", e.refs)


class ExistsExpr(E.Expr):
    """[NOT] EXISTS (subquery).  In a WHERE conjunct the engine turns it into a left semi /
    anti join on the subquery's WHERE (so correlated references to the outer relation work);
    evaluated directly, it is the uncorrelated truth value."""

    def __init__(self, sub, neg: bool):
        def f(df):
            from .engine import run_select
            hit = len(run_select(df.session, sub).limit(1).collect()) > 0
            return E.lit(hit != neg).eval(df)
        super().__init__(f, f"{'NOT ' if neg else ''}EXISTS(subquery)")
        self.sub, self.neg = sub, neg


def _subquery_rows(df, sub) -> list:
    from .engine import run_select
    return run_select(df.session, sub).collect()


def _scalar_subquery(sub):
    """(SELECT one value): evaluated once per use; no rows -> NULL, more than one -> error."""
    def f(df):
        rows = _subquery_rows(df, sub)
        if len(rows) > 1:
            raise ValueError("more than one row returned by a subquery used as an expression")
        return E.lit(rows[0][0] if rows else None).eval(df)
    return E.Expr(f, "scalarsubquery()")


def _in_subquery(a, sub):
    """x IN (SELECT c ...): membership in the subquery's first column."""
    def f(df):
        vals = [r[0] for r in _subquery_rows(df, sub)]
        return a.isin([v for v in vals if v is not None]).eval(df)
    return E.Expr(f, f"({a.name} IN (listquery()))", a.refs)


def parse(sql: str):
    return Parser(sql).statement()


def parse_expression(text: str):
    p = Parser(text)
    e = p.expr(allow_agg=False)
    alias = p._alias()
    if p.peek().kind != "eof":
        raise SyntaxError(f"unexpected trailing input in expression: {p.peek().val!r}")
    return e.alias(alias) if alias else e
