"""Column expressions (the ``pyspark.sql.Column`` / ``functions`` surface the widgets use).

An expression is a small tree evaluated eagerly against one partition
(``expr.eval(df) -> column.Column``).  Used by ``withColumn(name, df[c].cast('double'))``
(reference: orangecontrib/spark/widgets/ml/spark_ml_dataset.py:578), ``filter``,
``select`` and the SQL engine.
"""
from __future__ import annotations

import math
import re
from typing import Any, Callable

import numpy as np
import torch

from . import column as C
from . import types as T


class Expr:
    def __init__(self, fn: Callable, name: str, refs: tuple = ()):
        self._fn = fn
        self._name = name
        self.refs = refs  # referenced source column names

    # evaluation ---------------------------------------------------------------
    def eval(self, df) -> C.Column:
        return self._fn(df)

    @property
    def name(self) -> str:
        return self._name

    def __repr__(self):
        return f"Column<'{self._name}'>"

    def alias(self, name: str) -> "Expr":
        out = Expr(self._fn, name, self.refs)
        if getattr(self, "_generator", None):
            out._generator = self._generator
        return out

    name_ = alias

    def cast(self, dataType) -> "Expr":
        dt = T.parse_type(dataType)

        def f(df):
            c = self.eval(df)
            if isinstance(c, (C.NumericColumn, C.StringColumn)):
                return c.cast(dt)
            raise TypeError(f"cannot cast {c.dtype.simpleString()} to {dt.simpleString()}")
        return Expr(f, f"CAST({self._name} AS {dt.simpleString().upper()})", self.refs)

    astype = cast

    # arithmetic ---------------------------------------------------------------
    def _bin(self, other, op: str, torch_op, bool_out=False):
        o = other if isinstance(other, Expr) else lit(other)

        def f(df):
            a, b = self.eval(df), o.eval(df)
            return _binary(a, b, op, torch_op, bool_out, len(df))
        out = Expr(f, f"({self._name} {op} {o._name})", self.refs + o.refs)
        out._tree = (op, self, o)        # kept for join planning (equi-key extraction)
        return out

    def __add__(self, o): return self._bin(o, "+", torch.add)
    def __radd__(self, o): return lit(o)._bin(self, "+", torch.add)
    def __sub__(self, o): return self._bin(o, "-", torch.sub)
    def __rsub__(self, o): return lit(o)._bin(self, "-", torch.sub)
    def __mul__(self, o): return self._bin(o, "*", torch.mul)
    def __rmul__(self, o): return lit(o)._bin(self, "*", torch.mul)
    def __truediv__(self, o): return self._bin(o, "/", _div)
    def __rtruediv__(self, o): return lit(o)._bin(self, "/", _div)
    def __mod__(self, o): return self._bin(o, "%", torch.remainder)
    def __pow__(self, o): return self._bin(o, "**", _pow)
    def __eq__(self, o): return self._bin(o, "=", torch.eq, True)  # noqa: E721
    def __ne__(self, o): return self._bin(o, "!=", torch.ne, True)
    def __lt__(self, o): return self._bin(o, "<", torch.lt, True)
    def __le__(self, o): return self._bin(o, "<=", torch.le, True)
    def __gt__(self, o): return self._bin(o, ">", torch.gt, True)
    def __ge__(self, o): return self._bin(o, ">=", torch.ge, True)
    def __and__(self, o): return self._bin(o, "AND", torch.logical_and, True)
    def __or__(self, o): return self._bin(o, "OR", torch.logical_or, True)
    __hash__ = object.__hash__

    def __invert__(self):
        def f(df):
            c = self.eval(df)
            return C.NumericColumn(~c.data.bool(), c.valid, T.BooleanType())
        return Expr(f, f"(NOT {self._name})", self.refs)

    def __neg__(self):
        def f(df):
            c = self.eval(df)
            return C.NumericColumn(-c.data, c.valid, c.dtype)
        out = Expr(f, f"(- {self._name})", self.refs)
        if isinstance(getattr(self, "_literal", None), (int, float)):
            out._literal = -self._literal
        return out

    def eval_literal(self):
        """Python value of a literal expression (SQL function arguments such as ntile(4))."""
        if not hasattr(self, "_literal"):
            raise SyntaxError(f"expected a literal, found {self._name}")
        return self._literal

    def __bool__(self):
        raise ValueError("Cannot convert column into bool: use '&' for 'and', '|' for 'or', '~' for 'not'")

    # predicates ---------------------------------------------------------------
    def isNull(self):
        def f(df):
            c = self.eval(df)
            if isinstance(c, C.NumericColumn):
                m = torch.zeros_like(c.data, dtype=torch.bool) if c.valid is None else ~c.valid
            elif isinstance(c, C.HostColumn):
                m = c.null_mask()
            else:
                m = torch.zeros(len(c), dtype=torch.bool)
            return C.NumericColumn(m, None, T.BooleanType())
        return Expr(f, f"({self._name} IS NULL)", self.refs)

    def isNotNull(self):
        return ~self.isNull()

    def isin(self, *vals):
        vals = list(vals[0]) if len(vals) == 1 and isinstance(vals[0], (list, tuple, set)) else list(vals)

        def f(df):
            c = self.eval(df)
            if isinstance(c, C.NumericColumn):
                ref = torch.tensor(vals, dtype=c.data.dtype, device=c.data.device)
                return C.NumericColumn(torch.isin(c.data, ref), c.valid, T.BooleanType())
            s = set(vals)
            return C.NumericColumn(torch.tensor([v in s for v in c.values], dtype=torch.bool), None, T.BooleanType())
        return Expr(f, f"({self._name} IN {tuple(vals)})", self.refs)

    def between(self, lo, hi):
        return (self >= lo) & (self <= hi)

    def _str_pred(self, fn, label: str):
        """Boolean predicate over a string column, vectorised through pandas' string
        methods; a null input gives a null result (Spark)."""
        def f(df):
            import pandas as pd
            c = self.eval(df)
            vals = c.values if isinstance(c, C.HostColumn) else np.asarray(c.to_pylist(), dtype=object)
            ser = pd.Series(vals, dtype=object)
            null = ser.isna().to_numpy()
            res = fn(ser.astype(str)).to_numpy(dtype=bool, na_value=False) & ~null
            return C.NumericColumn(torch.from_numpy(res), torch.from_numpy(~null) if null.any() else None,
                                   T.BooleanType())
        return Expr(f, label, self.refs)

    @staticmethod
    def _like_rx(pattern: str) -> str:
        out = []
        i = 0
        while i < len(pattern):                  # SQL LIKE: % and _ wildcards, backslash escapes
            ch = pattern[i]
            if ch == "\\" and i + 1 < len(pattern):
                out.append(re.escape(pattern[i + 1]))
                i += 2
                continue
            out.append(".*" if ch == "%" else "." if ch == "_" else re.escape(ch))
            i += 1
        return "".join(out)

    def like(self, pattern: str):
        rx = re.compile(self._like_rx(pattern), re.S)
        return self._str_pred(lambda s: s.str.fullmatch(rx), f"({self._name} LIKE '{pattern}')")

    def ilike(self, pattern: str):
        rx = re.compile(self._like_rx(pattern), re.S | re.I)
        return self._str_pred(lambda s: s.str.fullmatch(rx), f"({self._name} ILIKE '{pattern}')")

    def rlike(self, pattern: str):
        rx = re.compile(pattern)
        return self._str_pred(lambda s: s.str.contains(rx, regex=True), f"RLIKE({self._name}, {pattern})")

    def contains(self, other):
        v = other.eval_literal() if isinstance(other, Expr) else other
        return self._str_pred(lambda s: s.str.contains(str(v), regex=False), f"contains({self._name}, {v})")

    def startswith(self, other):
        v = other.eval_literal() if isinstance(other, Expr) else other
        return self._str_pred(lambda s: s.str.startswith(str(v)), f"startswith({self._name}, {v})")

    def endswith(self, other):
        v = other.eval_literal() if isinstance(other, Expr) else other
        return self._str_pred(lambda s: s.str.endswith(str(v)), f"endswith({self._name}, {v})")

    def substr(self, startPos, length):
        """1-based substring (Spark ``Column.substr``)."""
        def f(df):
            c = self.eval(df)
            vals = c.values if isinstance(c, C.HostColumn) else np.asarray(c.to_pylist(), dtype=object)
            st = int(startPos) - 1 if int(startPos) > 0 else int(startPos)
            out = np.array([None if v is None else
                            (str(v)[st:st + int(length)] if st >= 0 else str(v)[len(str(v)) + st:][:int(length)])
                            for v in vals], dtype=object)
            return C.StringColumn(out)
        return Expr(f, f"substring({self._name}, {startPos}, {length})", self.refs)

    def eqNullSafe(self, other):
        """``<=>``: true when both sides are null, false when exactly one is, else ==."""
        o = other if isinstance(other, Expr) else lit(other)

        def f(df):
            a, b = self.eval(df), o.eval(df)
            eq = (self == o).eval(df)
            na, nb = a.null_mask(), b.null_mask()
            if nb.numel() == 1 and na.numel() != 1:
                nb = nb.expand_as(na)
            d = eq.data.to(torch.bool) if isinstance(eq, C.NumericColumn) else eq
            res = torch.where(na.to(d.device) | nb.to(d.device), na.to(d.device) & nb.to(d.device), d)
            return C.NumericColumn(res, None, T.BooleanType())
        return Expr(f, f"({self._name} <=> {o._name})", tuple(self.refs) + tuple(o.refs))

    def bitwiseAND(self, other):
        return self._bin(other, "&", torch.bitwise_and)

    def bitwiseOR(self, other):
        return self._bin(other, "|", torch.bitwise_or)

    def bitwiseXOR(self, other):
        return self._bin(other, "^", torch.bitwise_xor)

    def _ordered(self, desc: bool, nulls_first=None):
        e = Expr(self._fn, self._name, self.refs)
        e._desc = desc
        if nulls_first is not None:
            e._nulls_first = nulls_first
        return e

    def desc(self):
        return self._ordered(True)

    def asc(self):
        return self._ordered(False)

    def asc_nulls_first(self):
        return self._ordered(False, True)

    def asc_nulls_last(self):
        return self._ordered(False, False)

    def desc_nulls_first(self):
        return self._ordered(True, True)

    def desc_nulls_last(self):
        return self._ordered(True, False)

    def otherwise(self, value):
        if not hasattr(self, "_cases"):
            raise ValueError("otherwise() only valid after when()")
        return _when_expr(self._cases, value)

    def when(self, cond, value):
        if not hasattr(self, "_cases"):
            raise ValueError("when() only valid after functions.when()")
        return _make_when(self._cases + [(cond, value)])

    def getItem(self, i: int):
        def f(df):
            c = self.eval(df)
            if isinstance(c, C.VectorColumn):
                return C.NumericColumn(c.data[:, i].to(torch.float64))
            if isinstance(c, C.SparseVectorColumn):
                return C.NumericColumn(c.to_dense(torch.float64)[:, i])
            if isinstance(c, C.ArrayColumn):
                return C.StringColumn(np.array([None if v is None or i >= len(v) else v[i] for v in c.values], dtype=object))
            raise TypeError("getItem on non-array column")
        return Expr(f, f"{self._name}[{i}]", self.refs)

    __getitem__ = getItem

    def withField(self, fieldName: str, col: "Expr"):
        """Struct with field ``fieldName`` added or replaced (Spark ``Column.withField``)."""
        val = col if isinstance(col, Expr) else lit(col)

        def f(df):
            from .dataframe import Row
            c, v = self.eval(df), _host_values(val.eval(df), len(df))
            out = np.empty(len(c), dtype=object)
            for i, (s_, x) in enumerate(zip(c.values, v)):
                if s_ is None:
                    out[i] = None
                    continue
                names = list(s_.__fields__) if hasattr(s_, "__fields__") else list(s_.keys())
                vals = list(s_) if hasattr(s_, "__fields__") else [s_[k] for k in names]
                if fieldName in names:
                    vals[names.index(fieldName)] = x
                else:
                    names.append(fieldName)
                    vals.append(x)
                out[i] = Row._make(names, vals)
            return C.ArrayColumn(out)
        return Expr(f, f"update_fields({self._name}, WithField({fieldName}))", self.refs + val.refs)

    def dropFields(self, *fieldNames: str):
        """Struct without the named fields (Spark ``Column.dropFields``)."""
        def f(df):
            from .dataframe import Row
            c = self.eval(df)
            out = np.empty(len(c), dtype=object)
            for i, s_ in enumerate(c.values):
                if s_ is None:
                    out[i] = None
                    continue
                names = list(s_.__fields__) if hasattr(s_, "__fields__") else list(s_.keys())
                vals = list(s_) if hasattr(s_, "__fields__") else [s_[k] for k in names]
                keep = [(n, v) for n, v in zip(names, vals) if n not in fieldNames]
                if not keep:
                    raise ValueError("cannot drop all fields of a struct")
                out[i] = Row._make([n for n, _ in keep], [v for _, v in keep])
            return C.ArrayColumn(out)
        return Expr(f, f"update_fields({self._name}, dropField())", self.refs)

    def getField(self, name: str):
        """Field of a struct column (``Row`` / dict values), e.g. ``window.start``."""
        def f(df):
            return struct_field(self.eval(df), name)
        return Expr(f, f"{self._name}.{name}", self.refs)


def struct_field(c: C.Column, name: str) -> C.Column:
    """Values of field ``name`` of a host column of structs (Rows or dicts); null structs -> null."""
    from .dataframe import _nullable_column
    if not isinstance(c, C.HostColumn):
        raise TypeError(f"field access '{name}' needs a struct column, got {c.dtype.simpleString()}")
    out = []
    for v in c.values:
        if v is None:
            out.append(None)
        elif isinstance(v, dict):
            out.append(v.get(name))
        elif hasattr(v, "__fields__") and name in v.__fields__:
            out.append(v[v.__fields__.index(name)])
        else:
            raise KeyError(f"no struct field '{name}'")
    return _nullable_column(out)


def _div(a, b):
    return torch.div(a.to(torch.float64), b.to(torch.float64))


def _pow(a, b):
    return torch.pow(a.to(torch.float64), b.to(torch.float64))


def _promote(a: torch.Tensor, b: torch.Tensor):
    if a.dtype == b.dtype:
        return a, b
    dt = torch.promote_types(a.dtype, b.dtype)
    if dt in (torch.float32, torch.float16, torch.bfloat16) and (a.dtype == torch.float64 or b.dtype == torch.float64 or
                                                                  not a.is_floating_point() or not b.is_floating_point()):
        dt = torch.float64
    return a.to(dt), b.to(dt)


def _binary(a: C.Column, b: C.Column, op, torch_op, bool_out, n):
    if isinstance(a, C.NumericColumn) and isinstance(b, C.NumericColumn):
        x, y = a.data, b.data.to(a.data.device)
        if y.dim() == 0:
            y = y.expand_as(x)
        if x.dim() == 0:
            x = x.expand_as(y)
        if op in ("AND", "OR"):
            r = torch_op(x.bool(), y.bool())
        else:
            x, y = _promote(x, y)
            r = torch_op(x, y)
        valid = _and_valid(a.valid, b.valid)
        if op == "/":
            valid = _and_valid(valid, y != 0)
        dt = T.BooleanType() if bool_out else T.from_torch_dtype(r.dtype)
        return C.NumericColumn(r, valid, dt)
    # host (string) comparisons
    av = _host_values(a, n)
    bv = _host_values(b, n)
    py = {"=": lambda p, q: p == q, "!=": lambda p, q: p != q, "<": lambda p, q: p < q,
          "<=": lambda p, q: p <= q, ">": lambda p, q: p > q, ">=": lambda p, q: p >= q,
          "+": lambda p, q: p + q}[op]
    out = [None if (p is None or q is None) else py(p, q) for p, q in zip(av, bv)]
    if bool_out:
        valid = torch.tensor([o is not None for o in out], dtype=torch.bool)
        return C.NumericColumn(torch.tensor([bool(o) for o in out], dtype=torch.bool),
                               None if bool(valid.all()) else valid, T.BooleanType())
    return C.StringColumn(np.array(out, dtype=object))


def _host_values(c: C.Column, n: int):
    if isinstance(c, C.NumericColumn):
        if c.data.dim() == 0:
            return [c.data.item()] * n
        return c.to_pylist()
    if isinstance(c, _Scalar):
        return [c.value] * n
    return list(c.values)


def _and_valid(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return a & b.to(a.device)


class _Scalar(C.Column):
    """Broadcast literal (host)."""

    def __init__(self, value, n):
        self.value, self._n = value, n
        self.dtype = T.StringType()
        self.values = np.array([value] * n, dtype=object)

    def __len__(self):
        return self._n


def lit(value: Any) -> Expr:
    if isinstance(value, Expr):
        return value

    def f(df):
        n = len(df)
        if value is None:
            return C.NumericColumn(torch.zeros(n, dtype=torch.float64, device=df.device),
                                   torch.zeros(n, dtype=torch.bool, device=df.device), T.DoubleType())
        if isinstance(value, bool):
            return C.NumericColumn(torch.full((n,), value, dtype=torch.bool, device=df.device), None, T.BooleanType())
        if isinstance(value, int):
            return C.NumericColumn(torch.full((n,), value, dtype=torch.int64 if (value > 2**31 - 1 or value < -2**31) else torch.int32,
                                              device=df.device))
        if isinstance(value, float):
            return C.NumericColumn(torch.full((n,), value, dtype=torch.float64, device=df.device))
        return C.StringColumn(np.array([value] * n, dtype=object))
    name = repr(value) if isinstance(value, str) else str(value)
    if value is None:
        name = "NULL"
    e = Expr(f, name)
    e._literal = value
    return e


def col(name: str) -> Expr:
    def f(df):
        return df._col(name)
    e = Expr(f, name, (name,))
    e._colname = name
    return e


def qualified_col(qual: str, name: str) -> Expr:
    """SQL ``t.name``: the column ``name`` of relation ``t`` (a join picks the side by it;
    a single-relation frame resolves the bare name)."""
    def f(df):
        g = getattr(type(df), "_col_qualified", None)
        return g(df, qual, name) if g is not None else df._col(name)
    e = Expr(f, name, (name,))
    e._colname = name
    e._qual = qual
    return e


def bound_col(name: str, src, frame=None) -> Expr:
    """``df[name]`` / ``df.name``: a column reference that also remembers WHICH column object
    it came from (Spark's attribute id) and which frame it was taken from (Spark's dataset
    id), so a join condition such as ``a.id == b.id`` can tell the two sides apart even
    when ``b`` is derived from ``a`` and shares its column objects (self joins).  Frames
    without side information resolve it by name like :func:`col`."""
    import weakref
    ref = weakref.ref(src)
    fref = weakref.ref(frame) if frame is not None else (lambda: None)

    def f(df):
        g = getattr(type(df), "_col_bound", None)
        return g(df, name, ref(), fref()) if g is not None else df._col(name)
    e = Expr(f, name, (name,))
    e._colname = name
    e._src = ref
    e._frame = fref
    return e


column = col


def when(cond: Expr, value) -> Expr:
    return _make_when([(cond, value)])


def _make_when(cases):
    e = _when_expr(cases, None)
    e._cases = cases
    return e


def _when_expr(cases, default):
    def f(df):
        n = len(df)
        out = lit(default).eval(df)
        for cond, val in reversed(cases):
            cm = cond.eval(df)
            m = cm.data.bool() & (cm.valid if cm.valid is not None else True)
            v = lit(val).eval(df) if not isinstance(val, Expr) else val.eval(df)
            if isinstance(v, C.NumericColumn) and isinstance(out, C.NumericColumn):
                x, y = _promote(v.data, out.data.to(v.data.device))
                data = torch.where(m.to(x.device), x, y)
                vv = v.valid if v.valid is not None else torch.ones(n, dtype=torch.bool, device=x.device)
                ov = out.valid if out.valid is not None else torch.ones(n, dtype=torch.bool, device=x.device)
                valid = torch.where(m.to(x.device), vv, ov)
                out = C.NumericColumn(data, None if bool(valid.all()) else valid)
            else:
                a, b = _host_values(v, n), _host_values(out, n)
                mm = m.cpu().numpy()
                out = C.StringColumn(np.array([p if k else q for p, q, k in zip(a, b, mm)], dtype=object))
        return out
    return Expr(f, "CASE WHEN ... END", tuple(r for c, _ in cases for r in c.refs))


def _unary(name, fn):
    def mk(e):
        e = col(e) if isinstance(e, str) else e

        def f(df):
            c = e.eval(df)
            return C.NumericColumn(fn(c.data.to(torch.float64)), c.valid, T.DoubleType())
        return Expr(f, f"{name}({e.name})", e.refs)
    return mk


sqrt = _unary("SQRT", torch.sqrt)
log = _unary("LOG", torch.log)
exp = _unary("EXP", torch.exp)
log1p = _unary("LOG1P", torch.log1p)


def abs(e):  # noqa: A001
    e = col(e) if isinstance(e, str) else e

    def f(df):
        c = e.eval(df)
        return C.NumericColumn(torch.abs(c.data), c.valid, c.dtype)
    return Expr(f, f"ABS({e.name})", e.refs)


def isnan(e):
    e = col(e) if isinstance(e, str) else e

    def f(df):
        c = e.eval(df)
        d = c.data
        return C.NumericColumn(torch.isnan(d) if d.is_floating_point() else torch.zeros_like(d, dtype=torch.bool),
                               None, T.BooleanType())
    return Expr(f, f"isnan({e.name})", e.refs)


def coalesce(*es):
    es = [col(e) if isinstance(e, str) else e for e in es]

    def f(df):
        out = es[-1].eval(df)
        for e in reversed(es[:-1]):
            c = e.eval(df)
            m = ~(c.null_mask())
            x, y = _promote(c.data, out.data.to(c.data.device))
            valid = m | (out.valid if out.valid is not None else torch.ones_like(m))
            out = C.NumericColumn(torch.where(m, x, y), None if bool(valid.all()) else valid)
        return out
    return Expr(f, "coalesce(" + ",".join(e.name for e in es) + ")", tuple(r for e in es for r in e.refs))


# ------------------------------------------------------------------ aggregate exprs
class Agg:
    """Aggregate expression for groupBy().agg() / DataFrame.agg() / SQL."""

    def __init__(self, fn: str, arg: Expr | None, name: str | None = None, distinct=False):
        self.fn, self.arg, self.distinct = fn, arg, distinct
        self._name = name or (f"{fn}({arg.name if arg is not None else '1'})" if fn != "count" or arg is not None
                              else "count(1)")

    @property
    def name(self):
        return self._name

    def alias(self, name):
        out = Agg(self.fn, self.arg, name, self.distinct)
        for extra in ("arg2", "param"):            # second column / parameter of corr, percentile, ...
            if hasattr(self, extra):
                setattr(out, extra, getattr(self, extra))
        return out

    def over(self, window):
        """Aggregate over a window frame (``sum("x").over(Window.partitionBy(...))``)."""
        from ..sql.window import WindowExpr
        return WindowExpr(self, window, f"{self._name} OVER (...)")


def _agg(fn):
    def mk(e="*"):
        if isinstance(e, str):
            e = None if e == "*" else col(e)
        return Agg(fn, e)
    return mk


sum = _agg("sum")  # noqa: A001
avg = mean = _agg("avg")
min = _agg("min")  # noqa: A001
max = _agg("max")  # noqa: A001
count = _agg("count")
stddev = _agg("stddev")
variance = _agg("variance")


def countDistinct(e):
    e = col(e) if isinstance(e, str) else e
    return Agg("count", e, f"count(DISTINCT {e.name})", distinct=True)


__all__ = ["Expr", "Agg", "col", "column", "lit", "when", "sqrt", "log", "exp", "log1p", "abs", "isnan",
           "coalesce", "sum", "avg", "mean", "min", "max", "count", "stddev", "variance", "countDistinct"]
_ = math
