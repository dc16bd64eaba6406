"""``pyspark.sql.functions`` surface for the columnar engine.

Reached from the reference through the PySpark Script widget (arbitrary pyspark code,
orangecontrib/spark/widgets/data/pyspark_script_console.py:331) and SQL.  Numeric
functions run as torch ops on the column's device; string / date / array functions run
on the host over the rank's slice (strings live on the host in this engine);
``rand``/``randn``/``monotonically_increasing_id`` are keyed on the global row index,
so results do not depend on the number of GPUs.
"""
from __future__ import annotations

import builtins
import hashlib
import math
import re

import numpy as np
import torch

from ..frame import column as C
from ..frame import expr as E
from ..frame import types as T
from ..frame.expr import (Agg, Expr, abs, avg, coalesce, col, column, count, countDistinct, exp, isnan,  # noqa: F401
                          lit, log, log1p, max, mean, min, sqrt, stddev, sum, variance, when)

# ----------------------------------------------------------------------------- helpers


def _e(x) -> Expr:
    return col(x) if isinstance(x, str) else (x if isinstance(x, Expr) else lit(x))


def _refs(*es):
    return tuple(r for e in es for r in e.refs)


def _host(c: C.Column, n: int) -> list:
    return E._host_values(c, n)


def _str_out(vals) -> C.Column:
    arr = np.empty(len(vals), dtype=object)
    arr[:] = list(vals)
    return C.StringColumn(arr)


def _num_out(vals, dtype=torch.float64, device="cpu") -> C.NumericColumn:
    valid = None
    if any(v is None for v in vals):
        valid = torch.tensor([v is not None for v in vals], device=device)
    data = torch.tensor([0 if v is None else v for v in vals], dtype=dtype, device=device)
    return C.NumericColumn(data, valid)


def _host_map(name, fn, *args, kind="str"):
    """Row-wise host function of evaluated argument columns (None propagates)."""
    es = [_e(a) for a in args]

    def f(df):
        n = len(df)
        cols = [_host(e.eval(df), n) for e in es]
        out = [None if any(v is None for v in row) else fn(*row) for row in zip(*cols)] if cols else []
        if kind == "str":
            return _str_out(out)
        if kind == "array":
            arr = np.empty(n, dtype=object)
            arr[:] = out
            return C.ArrayColumn(arr)
        dt = torch.int64 if kind == "int" else (torch.bool if kind == "bool" else torch.float64)
        return _num_out(out, dt, df.device)
    return Expr(f, f"{name}({', '.join(e.name for e in es)})", _refs(*es))


def _num_map(name, fn, *args):
    es = [_e(a) for a in args]

    def f(df):
        cols = [e.eval(df) for e in es]
        valid = None
        for c in cols:
            if isinstance(c, C.NumericColumn) and c.valid is not None:
                valid = c.valid if valid is None else valid & c.valid
        data = fn(*[c.data.to(torch.float64) for c in cols])
        return C.NumericColumn(data, valid, T.DoubleType() if data.is_floating_point() else None)
    return Expr(f, f"{name}({', '.join(e.name for e in es)})", _refs(*es))


# ----------------------------------------------------------------------------- strings
def upper(c): return _host_map("upper", lambda s: str(s).upper(), c)
def lower(c): return _host_map("lower", lambda s: str(s).lower(), c)
def trim(c): return _host_map("trim", lambda s: str(s).strip(), c)
def ltrim(c): return _host_map("ltrim", lambda s: str(s).lstrip(), c)
def rtrim(c): return _host_map("rtrim", lambda s: str(s).rstrip(), c)
def initcap(c): return _host_map("initcap", lambda s: " ".join(w.capitalize() for w in str(s).split(" ")), c)
def reverse(c): return _host_map("reverse", lambda s: str(s)[::-1], c)
def length(c): return _host_map("length", lambda s: len(str(s)), c, kind="int")
def repeat(c, n): return _host_map("repeat", lambda s: str(s) * n, c)


def substring(c, pos: int, length_: int):
    """1-based start like Spark (pos 0 behaves like 1; negative counts from the end)."""
    def sub(s):
        s = str(s)
        start = pos - 1 if pos > 0 else (len(s) + pos if pos < 0 else 0)
        b = builtins.max(start, 0)
        return s[b:b + length_]
    return _host_map("substring", sub, c)


def concat(*cols):
    return _host_map("concat", lambda *v: "".join(str(x) for x in v), *cols)


def concat_ws(sep: str, *cols):
    es = [_e(a) for a in cols]

    def f(df):
        n = len(df)
        vals = [_host(e.eval(df), n) for e in es]
        return _str_out([sep.join(str(x) for x in row if x is not None) for row in zip(*vals)])
    return Expr(f, f"concat_ws({sep}, {', '.join(e.name for e in es)})", _refs(*es))


def regexp_replace(c, pattern: str, replacement: str):
    rx = re.compile(pattern)
    repl = re.sub(r"\$(\d+)", r"\\\1", replacement)          # Java $1 -> Python \1
    return _host_map("regexp_replace", lambda s: rx.sub(repl, str(s)), c)


def regexp_extract(c, pattern: str, idx: int):
    rx = re.compile(pattern)

    def ext(s):
        m = rx.search(str(s))
        return (m.group(idx) or "") if m else ""
    return _host_map("regexp_extract", ext, c)


def split(c, pattern: str, limit: int = -1):
    rx = re.compile(pattern)
    return _host_map("split", lambda s: rx.split(str(s), maxsplit=0 if limit <= 0 else limit - 1), c, kind="array")


def instr(c, substr: str):
    return _host_map("instr", lambda s: str(s).find(substr) + 1, c, kind="int")


def lpad(c, n: int, pad: str):
    return _host_map("lpad", lambda s: (pad * n + str(s))[-n:] if len(str(s)) < n else str(s)[:n], c)


def rpad(c, n: int, pad: str):
    return _host_map("rpad", lambda s: (str(s) + pad * n)[:n], c)


def format_number(c, d: int):
    return _host_map("format_number", lambda x: f"{float(x):,.{d}f}", c)


def md5(c): return _host_map("md5", lambda s: hashlib.md5(str(s).encode()).hexdigest(), c)
def sha1(c): return _host_map("sha1", lambda s: hashlib.sha1(str(s).encode()).hexdigest(), c)


def sha2(c, numBits: int):
    algo = {0: "sha256", 224: "sha224", 256: "sha256", 384: "sha384", 512: "sha512"}[numBits]
    return _host_map("sha2", lambda s: hashlib.new(algo, str(s).encode()).hexdigest(), c)


def hash(*cols):  # noqa: A001
    """Signed 32-bit CRC of the values' string forms (deterministic; bit parity with
    Spark's typed murmur3 ``hash`` is unpinned)."""
    def h(*v):
        import zlib
        return zlib.crc32("\x1f".join(str(x) for x in v).encode()) - (1 << 31)
    return _host_map("hash", h, *cols, kind="int")


# ----------------------------------------------------------------------------- math
def pow(a, b): return _num_map("POWER", torch.pow, a, b)  # noqa: A001
def floor(c): return _num_map("FLOOR", torch.floor, c)
def ceil(c): return _num_map("CEIL", torch.ceil, c)
def signum(c): return _num_map("SIGNUM", torch.sign, c)
def sin(c): return _num_map("SIN", torch.sin, c)
def cos(c): return _num_map("COS", torch.cos, c)
def tan(c): return _num_map("TAN", torch.tan, c)
def asin(c): return _num_map("ASIN", torch.asin, c)
def acos(c): return _num_map("ACOS", torch.acos, c)
def atan(c): return _num_map("ATAN", torch.atan, c)
def atan2(a, b): return _num_map("ATAN2", torch.atan2, a, b)
def log10(c): return _num_map("LOG10", torch.log10, c)
def log2(c): return _num_map("LOG2", torch.log2, c)
def hypot(a, b): return _num_map("HYPOT", torch.hypot, a, b)
def cbrt(c): return _num_map("CBRT", lambda x: torch.sign(x) * torch.abs(x) ** (1.0 / 3.0), c)
def degrees(c): return _num_map("DEGREES", torch.rad2deg, c)
def radians(c): return _num_map("RADIANS", torch.deg2rad, c)


def round(c, scale: int = 0):  # noqa: A001
    """HALF_UP rounding like Spark's round (bround = HALF_EVEN)."""
    f = 10.0 ** scale
    return _num_map(f"round({scale})", lambda x: torch.sign(x) * torch.floor(torch.abs(x) * f + 0.5) / f, c)


def bround(c, scale: int = 0):
    f = 10.0 ** scale
    return _num_map(f"bround({scale})", lambda x: torch.round(x * f) / f, c)


def greatest(*cols):
    return _num_map("greatest", lambda *xs: torch.stack(xs).amax(0), *cols)


def least(*cols):
    return _num_map("least", lambda *xs: torch.stack(xs).amin(0), *cols)


def nanvl(a, b):
    return _num_map("nanvl", lambda x, y: torch.where(torch.isnan(x), y, x), a, b)


def isnull(c):
    e = _e(c)
    return Expr(lambda df: C.NumericColumn(e.eval(df).null_mask(), None, T.BooleanType()), f"({e.name} IS NULL)",
                e.refs)


def isnotnull(c):
    e = _e(c)
    return Expr(lambda df: C.NumericColumn(~e.eval(df).null_mask(), None, T.BooleanType()),
                f"({e.name} IS NOT NULL)", e.refs)


# ----------------------------------------------------------------------------- random / ids
def rand(seed: int = 0):
    from ..ops import sampling

    def f(df):
        return C.NumericColumn(sampling.uniform(df._global_rows(), seed, stream=17).to(torch.float64))
    return Expr(f, f"rand({seed})")


def randn(seed: int = 0):
    from ..ops import sampling

    def f(df):
        rows = df._global_rows()
        u1 = sampling.uniform(rows, seed, stream=18).to(torch.float64).clamp_min(1e-300)
        u2 = sampling.uniform(rows, seed, stream=19).to(torch.float64)
        return C.NumericColumn(torch.sqrt(-2 * torch.log(u1)) * torch.cos(2 * math.pi * u2))
    return Expr(f, f"randn({seed})")


def monotonically_increasing_id():
    return Expr(lambda df: C.NumericColumn(df._global_rows()), "monotonically_increasing_id()")


def spark_partition_id():
    return Expr(lambda df: C.NumericColumn(torch.full((len(df),), df.comm.rank, dtype=torch.int32,
                                                      device=df.device)), "SPARK_PARTITION_ID()")


# ----------------------------------------------------------------------------- dates
def _dates(vals):
    import pandas as pd
    return pd.to_datetime(pd.Series(vals, dtype=object), errors="coerce")


def _date_map(name, fn, c, kind="int"):
    e = _e(c)

    def f(df):
        n = len(df)
        s = _dates(_host(e.eval(df), n))
        out = fn(s)
        vals = [None if (v is None or (isinstance(v, float) and math.isnan(v))) else v for v in out.tolist()]
        if kind == "str":
            return _str_out(vals)
        return _num_out(vals, torch.int64 if kind == "int" else torch.float64, df.device)
    return Expr(f, f"{name}({e.name})", e.refs)


def year(c): return _date_map("year", lambda s: s.dt.year.astype("float"), c)
def month(c): return _date_map("month", lambda s: s.dt.month.astype("float"), c)
def dayofmonth(c): return _date_map("dayofmonth", lambda s: s.dt.day.astype("float"), c)
def dayofweek(c): return _date_map("dayofweek", lambda s: ((s.dt.dayofweek + 1) % 7 + 1).astype("float"), c)
def dayofyear(c): return _date_map("dayofyear", lambda s: s.dt.dayofyear.astype("float"), c)
def hour(c): return _date_map("hour", lambda s: s.dt.hour.astype("float"), c)
def minute(c): return _date_map("minute", lambda s: s.dt.minute.astype("float"), c)
def second(c): return _date_map("second", lambda s: s.dt.second.astype("float"), c)


def to_date(c, format=None):  # noqa: A002
    return _date_map("to_date", lambda s: s.dt.strftime("%Y-%m-%d").where(s.notna(), None), c, kind="str")


def date_format(c, format: str):  # noqa: A002
    py = (format.replace("yyyy", "%Y").replace("MM", "%m").replace("dd", "%d").replace("HH", "%H")
          .replace("mm", "%M").replace("ss", "%S"))
    return _date_map("date_format", lambda s: s.dt.strftime(py).where(s.notna(), None), c, kind="str")


def current_date():
    import datetime
    d = datetime.date.today().isoformat()
    return Expr(lambda df: _str_out([d] * len(df)), "current_date()")


def date_add(c, days: int):
    import pandas as pd
    return _date_map("date_add", lambda s: (s + pd.Timedelta(days=days)).dt.strftime("%Y-%m-%d")
                     .where(s.notna(), None), c, kind="str")


def date_sub(c, days: int):
    return date_add(c, -days)


def datediff(end, start):
    a, b = _e(end), _e(start)

    def f(df):
        n = len(df)
        x, y = _dates(_host(a.eval(df), n)), _dates(_host(b.eval(df), n))
        d = (x.dt.normalize() - y.dt.normalize()).dt.days
        return _num_out([None if math.isnan(v) else int(v) for v in d.astype("float").tolist()], torch.int64,
                        df.device)
    return Expr(f, f"datediff({a.name}, {b.name})", _refs(a, b))


# ----------------------------------------------------------------------------- arrays
def array(*cols):
    es = [_e(a) for a in cols]

    def f(df):
        n = len(df)
        vals = [_host(e.eval(df), n) for e in es]
        arr = np.empty(n, dtype=object)
        arr[:] = [list(r) for r in zip(*vals)]
        return C.ArrayColumn(arr)
    return Expr(f, f"array({', '.join(e.name for e in es)})", _refs(*es))


def size(c): return _host_map("size", lambda v: len(v), c, kind="int")
def array_contains(c, value): return _host_map("array_contains", lambda v: value in v, c, kind="bool")
def sort_array(c, asc: bool = True): return _host_map("sort_array", lambda v: sorted(v, reverse=not asc), c,
                                                      kind="array")
def array_distinct(c): return _host_map("array_distinct", lambda v: list(dict.fromkeys(v)), c, kind="array")


def element_at(c, i: int):
    return _host_map("element_at", lambda v: (v[i - 1] if i > 0 else v[i]) if len(v) >= builtins.abs(i) else None, c,
                     kind="str")


def explode(c):
    """Generator: one output row per array element (handled by DataFrame.select)."""
    e = _e(c)
    out = Expr(lambda df: e.eval(df), "col", e.refs)
    out._generator = "explode"
    return out


def posexplode(c):
    e = _e(c)
    out = Expr(lambda df: e.eval(df), "col", e.refs)
    out._generator = "posexplode"
    return out


# ----------------------------------------------------------------------------- aggregates
def first(c, ignorenulls: bool = False): return Agg("first", _e(c), f"first({_e(c).name})")
def last(c, ignorenulls: bool = False): return Agg("last", _e(c), f"last({_e(c).name})")
def collect_list(c): return Agg("collect_list", _e(c), f"collect_list({_e(c).name})")
def collect_set(c): return Agg("collect_set", _e(c), f"collect_set({_e(c).name})")
def stddev_samp(c): return stddev(c)
def var_samp(c): return variance(c)
def sumDistinct(c): return Agg("sum", _e(c), f"sum(DISTINCT {_e(c).name})", distinct=True)


sum_distinct = sumDistinct
count_distinct = countDistinct
std = stddev


# ----------------------------------------------------------------------------- misc
def expr(s: str) -> Expr:
    from .parser import parse_expression
    return parse_expression(s)


def asc(c): return _e(c).asc()
def desc(c): return _e(c).desc()


def broadcast(df):
    """Join hint; every join in this engine already broadcasts the smaller side."""
    return df


def udf(f=None, returnType=None):
    """Python UDF applied per row on the host.  ``returnType`` picks the column kind."""
    def wrap(fn):
        rt = T.parse_type(returnType) if returnType is not None else T.StringType()
        if isinstance(rt, T.BooleanType):
            kind = "bool"
        elif isinstance(rt, (T.IntegerType, T.LongType, T.ShortType, T.ByteType)):
            kind = "int"
        elif isinstance(rt, T.NumericType):
            kind = "float"
        elif isinstance(rt, T.ArrayType):
            kind = "array"
        else:
            kind = "str"

        def call(*cols):
            return _host_map(getattr(fn, "__name__", "udf"), fn, *cols, kind=kind)
        call.func, call.returnType = fn, rt
        return call
    if f is not None and callable(f):
        return wrap(f)
    if f is not None and returnType is None:
        returnType = f
    return wrap


# window functions (sql/window.py)
from .window import (Window, cume_dist, dense_rank, lag, lead, nth_value, ntile, percent_rank,  # noqa: E402,F401
                     rank, row_number)

__all__ = [n for n in dir() if not n.startswith("_") and n not in ("annotations", "hashlib", "math", "re", "np",
                                                                     "torch", "C", "E", "T")]
