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
from collections import OrderedDict
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
    ser = pd.Series(vals, dtype=object)
    try:                                    # rows may mix dates and timestamps
        return pd.to_datetime(ser, errors="coerce", format="mixed")
    except (TypeError, ValueError):
        return pd.to_datetime(ser, errors="coerce")


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
        for i, r in enumerate(zip(*vals) if vals else ((),) * n):
            arr[i] = list(r)
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


def grouping(c):
    """1 if ``c`` is aggregated away in this grouping set of a rollup / cube, else 0."""
    return Agg("grouping", _e(c), f"grouping({_e(c).name})")


def grouping_id(*cols):
    """Bit vector of :func:`grouping` over ``cols`` (default: all grouping keys), first
    column most significant."""
    a = Agg("grouping_id", None, f"grouping_id({', '.join(_e(x).name for x in cols)})")
    a.param = [_e(x).name for x in cols] or None
    return a
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


# ============================================================================ more of the
# pyspark.sql.functions surface (strings / dates / JSON / arrays / maps / math / nulls /
# statistical aggregates).  Host functions run over the rank's slice; the moment and
# co-moment aggregates run as device partial sums merged across ranks (frame/groupby.py).
import base64 as _b64  # noqa: E402
import binascii as _binascii  # noqa: E402
import json as _json  # noqa: E402
import zlib as _zlib  # noqa: E402


def _nn(v):
    return v is not None and not (isinstance(v, float) and math.isnan(v))


# ---- strings
def substring_index(c, delim: str, count: int):
    def f(s):
        parts = str(s).split(delim)
        if count > 0:
            return delim.join(parts[:count])
        if count < 0:
            return delim.join(parts[count:])
        return ""
    return _host_map("substring_index", f, c)


def format_string(format: str, *cols):  # noqa: A002
    py = re.sub(r"%(\d+)\$", r"%", format)                   # Java positional args unsupported -> sequential
    return _host_map("format_string", lambda *v: py % tuple(v), *cols)


def translate(c, matching: str, replace: str):
    table = {ord(m): (replace[i] if i < len(replace) else None) for i, m in enumerate(matching)}
    return _host_map("translate", lambda s: str(s).translate(table), c)


def levenshtein(left, right):
    def lev(a, b):
        a, b = str(a), str(b)
        prev = list(range(len(b) + 1))
        for i, ca in enumerate(a, 1):
            cur = [i]
            for j, cb in enumerate(b, 1):
                cur.append(builtins.min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb)))
            prev = cur
        return prev[-1]
    return _host_map("levenshtein", lev, left, right, kind="int")


def soundex(c):
    codes = {**dict.fromkeys("BFPV", "1"), **dict.fromkeys("CGJKQSXZ", "2"), **dict.fromkeys("DT", "3"),
             "L": "4", **dict.fromkeys("MN", "5"), "R": "6"}

    def sx(s):
        s = "".join(ch for ch in str(s).upper() if ch.isalpha())
        if not s:
            return ""
        out, last = s[0], codes.get(s[0], "")
        for ch in s[1:]:
            d = codes.get(ch, "")
            if d and d != last:
                out += d
            if ch not in "HW":
                last = d
        return (out + "000")[:4]
    return _host_map("soundex", sx, c)


def ascii(c):  # noqa: A001
    return _host_map("ascii", lambda s: ord(str(s)[0]) if str(s) else 0, c, kind="int")


def base64(c):
    return _host_map("base64", lambda s: _b64.b64encode(s if isinstance(s, bytes) else str(s).encode()).decode(), c)


def unbase64(c):
    return _host_map("unbase64", lambda s: _b64.b64decode(str(s)).decode("utf-8", "replace"), c)


def hex(c):  # noqa: A001
    def h(v):
        if isinstance(v, (int, float)) and not isinstance(v, bool) and float(v).is_integer():
            return format(int(v) & 0xFFFFFFFFFFFFFFFF, "X") if int(v) < 0 else format(int(v), "X")
        return _binascii.hexlify(str(v).encode()).decode().upper()
    return _host_map("hex", h, c)


def unhex(c):
    return _host_map("unhex", lambda s: _binascii.unhexlify(str(s)).decode("utf-8", "replace"), c)


def conv(c, fromBase: int, toBase: int):
    digits = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ"

    def cv(s):
        n = int(str(s).strip(), fromBase)
        if n == 0:
            return "0"
        neg, n, out = n < 0, builtins.abs(n), ""
        while n:
            n, r = divmod(n, builtins.abs(toBase))
            out = digits[r] + out
        return ("-" if neg else "") + out
    return _host_map("conv", cv, c)


def bin(c):  # noqa: A001
    return _host_map("bin", lambda v: format(int(v) & 0xFFFFFFFFFFFFFFFF if int(v) < 0 else int(v), "b"), c)


def crc32(c):
    return _host_map("crc32", lambda s: _zlib.crc32(s if isinstance(s, bytes) else str(s).encode()), c, kind="int")


def xxhash64(*cols):
    """64-bit xxHash of the values' UTF-8 text (seed 42 like Spark; parity with Spark's binary
    encoding of non-string types is not pinned)."""
    import xxhash as _xx

    def h(*v):
        x = _xx.xxh64(seed=42)
        for a in v:
            x.update(str(a).encode())
        u = x.intdigest()
        return u - (1 << 64) if u >= (1 << 63) else u
    return _host_map("xxhash64", h, *cols, kind="int")


def locate(substr: str, c, pos: int = 1):
    return _host_map("locate", lambda s: str(s).find(substr, builtins.max(pos - 1, 0)) + 1, c, kind="int")


# ---- nulls
def nvl(c1, c2):
    return coalesce(_e(c1), _e(c2))


ifnull = nvl


def nullif(c1, c2):
    a, b = _e(c1), _e(c2)

    def f(df):
        n = len(df)
        x, y = _host(a.eval(df), n), _host(b.eval(df), n)
        out = [None if (u is not None and v is not None and u == v) else u for u, v in zip(x, y)]
        if all(v is None or isinstance(v, (int, float)) for v in out):
            return _num_out(out, torch.float64, df.device)
        return _str_out(out)
    return Expr(f, f"nullif({a.name}, {b.name})", _refs(a, b))


# ---- math
def expm1(c): return _num_map("EXPM1", torch.expm1, c)
def factorial(c): return _host_map("factorial", lambda v: math.factorial(int(v)) if 0 <= int(v) <= 20 else None,
                                   c, kind="int")
def shiftleft(c, numBits: int): return _host_map("shiftleft", lambda v: int(v) << numBits, c, kind="int")
def shiftright(c, numBits: int): return _host_map("shiftright", lambda v: int(v) >> numBits, c, kind="int")
def bitwise_not(c): return _host_map("bitwise_not", lambda v: ~int(v), c, kind="int")


bitwiseNOT = bitwise_not
shiftLeft, shiftRight = shiftleft, shiftright


# ---- dates / timestamps
def _java_fmt(fmt: str) -> str:
    return (fmt.replace("yyyy", "%Y").replace("yy", "%y").replace("MM", "%m").replace("dd", "%d")
            .replace("HH", "%H").replace("mm", "%M").replace("ss", "%S"))


def to_timestamp(c, format=None):  # noqa: A002
    e = _e(c)

    def f(df):
        import pandas as pd
        vals = pd.Series(_host(e.eval(df), len(df)), dtype=object)
        s = pd.to_datetime(vals, format=_java_fmt(format) if format else None, errors="coerce")
        return _str_out([None if pd.isna(v) else v.strftime("%Y-%m-%d %H:%M:%S") for v in s])
    return Expr(f, f"to_timestamp({e.name})", e.refs)


def unix_timestamp(c=None, format: str = "yyyy-MM-dd HH:mm:ss"):  # noqa: A002
    if c is None:
        import time as _t
        now = int(_t.time())
        return Expr(lambda df: _num_out([now] * len(df), torch.int64, df.device), "unix_timestamp()")
    e = _e(c)

    def f(df):
        import pandas as pd
        s = pd.to_datetime(pd.Series(_host(e.eval(df), len(df)), dtype=object), format=_java_fmt(format),
                           errors="coerce")
        return _num_out([None if pd.isna(v) else int(v.timestamp()) for v in s], torch.int64, df.device)
    return Expr(f, f"unix_timestamp({e.name})", e.refs)


def from_unixtime(c, format: str = "yyyy-MM-dd HH:mm:ss"):  # noqa: A002
    import datetime as _dt
    py = _java_fmt(format)
    return _host_map("from_unixtime", lambda v: _dt.datetime.utcfromtimestamp(int(v)).strftime(py), c)


def date_trunc(format: str, c):  # noqa: A002
    unit = format.lower()
    freq = {"year": "YS", "yyyy": "YS", "yy": "YS", "month": "MS", "mon": "MS", "mm": "MS", "day": "D", "dd": "D",
            "hour": "h", "minute": "min", "second": "s", "week": "W-MON", "quarter": "QS"}.get(unit, "D")

    def trunc_(s):
        if freq in ("YS", "MS", "QS"):
            p = {"YS": "Y", "MS": "M", "QS": "Q"}[freq]
            return s.dt.to_period(p).dt.start_time
        if freq == "W-MON":
            return (s - __import__("pandas").to_timedelta(s.dt.dayofweek, unit="D")).dt.normalize()
        return s.dt.floor(freq)
    return _date_map("date_trunc", lambda s: trunc_(s).dt.strftime("%Y-%m-%d %H:%M:%S").where(s.notna(), None), c,
                     kind="str")


def trunc(c, format: str):  # noqa: A002
    return _date_map("trunc", lambda s: date_trunc_series(s, format).dt.strftime("%Y-%m-%d").where(s.notna(), None),
                     c, kind="str")


def date_trunc_series(s, format):  # noqa: A002
    p = {"year": "Y", "yyyy": "Y", "yy": "Y", "month": "M", "mon": "M", "mm": "M", "quarter": "Q"}.get(
        format.lower(), "M")
    return s.dt.to_period(p).dt.start_time


def weekofyear(c): return _date_map("weekofyear", lambda s: s.dt.isocalendar().week.astype("float"), c)
def quarter(c): return _date_map("quarter", lambda s: s.dt.quarter.astype("float"), c)


def last_day(c):
    return _date_map("last_day", lambda s: (s + __import__("pandas").offsets.MonthEnd(0)).dt.strftime("%Y-%m-%d")
                     .where(s.notna(), None), c, kind="str")


def next_day(c, dayOfWeek: str):
    import pandas as pd
    names = ["mo", "tu", "we", "th", "fr", "sa", "su"]
    target = names.index(dayOfWeek.lower()[:2])
    return _date_map("next_day", lambda s: (s + pd.to_timedelta(((target - s.dt.dayofweek - 1) % 7) + 1, unit="D"))
                     .dt.strftime("%Y-%m-%d").where(s.notna(), None), c, kind="str")


def add_months(c, months: int):
    import pandas as pd
    return _date_map("add_months", lambda s: (s + pd.DateOffset(months=months)).dt.strftime("%Y-%m-%d")
                     .where(s.notna(), None), c, kind="str")


def months_between(date1, date2, roundOff: bool = True):
    a, b = _e(date1), _e(date2)

    def f(df):
        n = len(df)
        x, y = _dates(_host(a.eval(df), n)), _dates(_host(b.eval(df), n))
        out = []
        for u, v in zip(x, y):
            if u is None or v is None or str(u) == "NaT" or str(v) == "NaT":
                out.append(None)
                continue
            m = (u.year - v.year) * 12 + (u.month - v.month)
            if not (u.day == v.day or (u.is_month_end and v.is_month_end)):
                m += (u.day - v.day) / 31.0 + ((u.hour * 3600 + u.minute * 60 + u.second) -
                                             (v.hour * 3600 + v.minute * 60 + v.second)) / (31.0 * 86400)
            out.append(round(m, 8) if roundOff else m)
        return _num_out(out, torch.float64, df.device)
    return Expr(f, f"months_between({a.name}, {b.name})", _refs(a, b))


def current_timestamp():
    import datetime
    t = datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S")
    return Expr(lambda df: _str_out([t] * len(df)), "current_timestamp()")


now = current_timestamp


def input_file_name():
    """Files are not tracked per row by this engine's readers: always the empty string."""
    return Expr(lambda df: _str_out([""] * len(df)), "input_file_name()")


# ---- JSON
def to_json(c, options=None):
    def tj(v):
        if hasattr(v, "asDict"):
            v = v.asDict(recursive=True)
        if hasattr(v, "toArray"):
            v = np.asarray(v.toArray()).tolist()
        return _json.dumps(v, separators=(",", ":"), default=str)
    return _host_map("to_json", tj, c)


def from_json(c, schema, options=None):
    """JSON text -> struct (a Row of the schema's fields) or, without field info, a dict."""
    from ..frame.dataframe import Row
    try:
        st = _ddl_schema(schema)
        names = [f.name for f in st.fields]
    except Exception:  # noqa: BLE001 - schema forms the type parser does not know: keep dicts
        names = None

    def fj(s):
        try:
            d = _json.loads(str(s))
        except ValueError:
            return None
        if names and isinstance(d, dict):
            return Row._make(names, [d.get(n) for n in names])
        return d
    return _host_map("from_json", fj, c, kind="array")


def get_json_object(c, path: str):
    """JSONPath subset: ``$.a.b``, ``$.a[0]``, ``$['a']``."""
    toks = re.findall(r"\.([A-Za-z_][\w]*)|\[(\d+)\]|\['([^']+)'\]", path)

    def g(s):
        try:
            v = _json.loads(str(s))
        except ValueError:
            return None
        for name, idx, qname in toks:
            if name or qname:
                if not isinstance(v, dict) or (name or qname) not in v:
                    return None
                v = v[name or qname]
            else:
                if not isinstance(v, list) or int(idx) >= len(v):
                    return None
                v = v[int(idx)]
        return v if isinstance(v, str) else _json.dumps(v, separators=(",", ":"))
    return _host_map("get_json_object", g, c)


# ---- structs and maps
def struct(*cols):
    from ..frame.dataframe import Row
    es = [_e(a) for a in (cols[0] if len(cols) == 1 and isinstance(cols[0], (list, tuple)) else cols)]

    def f(df):
        n = len(df)
        vals = [_host(e.eval(df), n) for e in es]
        names = [e.name for e in es]
        arr = np.empty(n, dtype=object)
        arr[:] = [Row._make(names, list(r)) for r in zip(*vals)]
        return C.ArrayColumn(arr)
    return Expr(f, f"struct({', '.join(e.name for e in es)})", _refs(*es))


def create_map(*cols):
    es = [_e(a) for a in (cols[0] if len(cols) == 1 and isinstance(cols[0], (list, tuple)) else cols)]

    def f(df):
        n = len(df)
        vals = [_host(e.eval(df), n) for e in es]
        arr = np.empty(n, dtype=object)
        arr[:] = [{r[i]: r[i + 1] for i in range(0, len(r) - 1, 2)} for r in zip(*vals)]
        return C.ArrayColumn(arr)
    return Expr(f, f"map({', '.join(e.name for e in es)})", _refs(*es))


def map_keys(c): return _host_map("map_keys", lambda m: list(m.keys()), c, kind="array")
def map_values(c): return _host_map("map_values", lambda m: list(m.values()), c, kind="array")


# ---- arrays
def array_join(c, delimiter: str, null_replacement=None):
    return _host_map("array_join", lambda v: delimiter.join(
        str(x) if x is not None else null_replacement for x in v if x is not None or null_replacement is not None), c)


def array_position(c, value):
    return _host_map("array_position", lambda v: (list(v).index(value) + 1) if value in v else 0, c, kind="int")


def array_remove(c, element):
    return _host_map("array_remove", lambda v: [x for x in v if x != element], c, kind="array")


def arrays_zip(*cols):
    return _host_map("arrays_zip", lambda *vs: [list(t) for t in __import__("itertools").zip_longest(*vs)], *cols,
                     kind="array")


def flatten(c):
    return _host_map("flatten", lambda v: [x for sub in v if sub is not None for x in sub], c, kind="array")


def slice(x, start: int, length: int):  # noqa: A001
    def sl(v):
        v = list(v)
        b = start - 1 if start > 0 else len(v) + start
        return v[builtins.max(b, 0):builtins.max(b, 0) + length]
    return _host_map("slice", sl, x, kind="array")


def sequence(start, stop, step=None):
    es = [_e(start), _e(stop)] + ([_e(step)] if step is not None else [])

    def seq(a, b, s=None):
        a, b = int(a), int(b)
        s = int(s) if s is not None else (1 if b >= a else -1)
        return list(range(a, b + (1 if s > 0 else -1), s))
    return _host_map("sequence", seq, *es, kind="array")


def array_union(a, b):
    return _host_map("array_union", lambda x, y: list(dict.fromkeys(list(x) + list(y))), a, b, kind="array")


def array_intersect(a, b):
    return _host_map("array_intersect", lambda x, y: [v for v in dict.fromkeys(x) if v in set(y)], a, b,
                     kind="array")


def array_except(a, b):
    return _host_map("array_except", lambda x, y: [v for v in dict.fromkeys(x) if v not in set(y)], a, b,
                     kind="array")


def array_max(c):
    return _host_map("array_max", lambda v: builtins.max((x for x in v if x is not None), default=None), c,
                     kind="float")


def array_min(c):
    return _host_map("array_min", lambda v: builtins.min((x for x in v if x is not None), default=None), c,
                     kind="float")


def array_sort(c):
    return _host_map("array_sort", lambda v: sorted((x for x in v if x is not None)) + [x for x in v if x is None],
                     c, kind="array")


def explode_outer(c):
    """explode that keeps rows whose array is empty or null (one null element)."""
    e = _e(c)
    out = Expr(lambda df: e.eval(df), "col", e.refs)
    out._generator = "explode_outer"
    return out


def posexplode_outer(c):
    e = _e(c)
    out = Expr(lambda df: e.eval(df), "col", e.refs)
    out._generator = "posexplode_outer"
    return out


# ---- sorting helpers
def asc_nulls_first(c): return _e(c).asc_nulls_first()
def asc_nulls_last(c): return _e(c).asc_nulls_last()
def desc_nulls_first(c): return _e(c).desc_nulls_first()
def desc_nulls_last(c): return _e(c).desc_nulls_last()


# ---- statistical aggregates (device partial moments, merged across ranks)
def stddev_pop(c): return Agg("stddev_pop", _e(c), f"stddev_pop({_e(c).name})")
def var_pop(c): return Agg("var_pop", _e(c), f"var_pop({_e(c).name})")
def skewness(c): return Agg("skewness", _e(c), f"skewness({_e(c).name})")
def kurtosis(c): return Agg("kurtosis", _e(c), f"kurtosis({_e(c).name})")


def _agg2(fn, a, b):
    x, y = _e(a), _e(b)
    out = Agg(fn, x, f"{fn}({x.name}, {y.name})")
    out.arg2 = y
    return out


def corr(col1, col2): return _agg2("corr", col1, col2)
def covar_pop(col1, col2): return _agg2("covar_pop", col1, col2)
def covar_samp(col1, col2): return _agg2("covar_samp", col1, col2)


def approx_count_distinct(c, rsd: float = 0.05):
    """Exact distinct count (device dedupe) -- within any ``rsd``."""
    return Agg("count", _e(c), f"approx_count_distinct({_e(c).name})", distinct=True)


approxCountDistinct = approx_count_distinct


def percentile_approx(c, percentage, accuracy: int = 10000):
    """Exact percentile(s): the smallest value v with at least ``p`` of the group <= v (Spark's
    definition of its approximation target)."""
    out = Agg("percentile", _e(c), f"percentile_approx({_e(c).name}, {percentage}, {accuracy})")
    out.param = percentage
    return out


approx_percentile = percentile_approx


def percentile(c, percentage, frequency=1):
    """Exact percentile(s) with linear interpolation between the closest ranks (Spark
    ``percentile``; ``frequency`` other than 1 is not supported)."""
    if not (isinstance(frequency, int) and frequency == 1):
        raise ValueError("percentile: only frequency=1 is supported")
    out = Agg("percentile_exact", _e(c), f"percentile({_e(c).name}, {percentage})")
    out.param = percentage
    return out


def ceiling(c):
    return ceil(c)


def btrim(c, trim=None):
    """Strip ``trim`` characters (default spaces) from both ends."""
    return _host_map("btrim", (lambda s: str(s).strip(" ")) if trim is None else (lambda s: str(s).strip(trim)), c)


def typeof(c):
    e = _e(c)

    def f(df):
        col = e.eval(df)
        return C.StringColumn(np.array([col.dtype.simpleString()] * len(col), dtype=object))
    return Expr(f, f"typeof({e.name})", e.refs)


def assert_true(c, errMsg=None):
    """NULL when every value is true, else raise (Spark ``assert_true``)."""
    e = _e(c)

    def f(df):
        col = e.eval(df)
        ok = col.data.bool() if isinstance(col, C.NumericColumn) else torch.tensor(
            [bool(v) for v in col.to_pylist()])
        if isinstance(col, C.NumericColumn) and col.valid is not None:
            ok = ok & col.valid
        if not bool(ok.all()):
            raise RuntimeError(errMsg if errMsg is not None else f"'{e.name}' is not true!")
        return C.NumericColumn(torch.zeros(len(col), dtype=torch.float64, device=df.device),
                               torch.zeros(len(col), dtype=torch.bool, device=df.device))
    return Expr(f, f"assert_true({e.name})", e.refs)


def inline_outer(c):
    """inline that keeps rows whose array is empty or null (one all-null row)."""
    out = explode_outer(c)
    out._inline = True
    return out


def stack(n, *cols):
    """Generator: splits the k values into ``n`` rows of k/n columns (``col0``, ``col1``, ...)."""
    n = int(n.eval_literal() if hasattr(n, "eval_literal") else n)
    es = [_e(x) for x in cols]
    width = -(-len(es) // n)
    from ..frame.dataframe import Row
    names = [f"col{i}" for i in range(width)]

    def f(df):
        m = len(df)
        vals = [_host(e.eval(df), m) for e in es]
        out = np.empty(m, dtype=object)
        for r in range(m):
            out[r] = [Row._make(names, [vals[j * width + i][r] if j * width + i < len(es) else None
                                        for i in range(width)]) for j in range(n)]
        return C.ArrayColumn(out)
    g = Expr(f, f"stack({n}, {', '.join(e.name for e in es)})", _refs(*es))
    g._generator = "explode"
    g._inline = True
    return g


def sentences(string, language=None, country=None):
    """Split text into sentences of words (array<array<string>>); punctuation dropped."""
    def sp(s):
        parts = [p for p in re.split(r"(?<=[.!?])\s+", str(s).strip()) if p]
        return [[w for w in re.findall(r"[\w']+", p)] for p in parts]
    return _host_map("sentences", sp, string, kind="array")


def to_number(c, format):  # noqa: A002
    """Parse strings formatted like ``format`` (digits, ',', '.', '$', sign) to doubles; an
    unparsable value raises (use ``try_to_number`` for NULL)."""
    return _to_number(c, format, strict=True)


def try_to_number(c, format):  # noqa: A002
    return _to_number(c, format, strict=False)


def _to_number(c, fmt, strict):
    fmt = fmt.eval_literal() if hasattr(fmt, "eval_literal") else fmt

    def conv(s):
        t = str(s).strip().replace(",", "").replace("$", "")
        neg = t.endswith("-") or (t.startswith("<") and t.endswith(">"))
        t = t.strip("<>-") if neg else t
        try:
            v = float(t)
        except ValueError:
            if strict:
                raise ValueError(f"the input '{s}' does not match the format '{fmt}'")
            return None
        return -v if neg else v
    return _host_map("to_number", conv, c, kind="float")


def to_char(c, format):  # noqa: A002
    """Format numbers with a Spark number format ('999,999.00', '$99.9', '0000'): digit
    count after the decimal point and grouping commas are honoured."""
    fmt = format.eval_literal() if hasattr(format, "eval_literal") else format
    dec = len(fmt.split(".")[1]) if "." in fmt else 0
    comma = "," in fmt
    dollar = fmt.startswith("$")
    width = len([ch for ch in fmt.split(".")[0] if ch in "09"])
    zero_pad = fmt.lstrip("$").startswith("0")

    def fm(x):
        s = f"{float(x):{',' if comma else ''}.{dec}f}"
        if zero_pad and not comma:
            ip, _, fp = s.partition(".")
            s = ip.zfill(width) + ("." + fp if fp else "")
        return ("$" if dollar else "") + s
    return _host_map("to_char", fm, c)


to_varchar = to_char


def pandas_udf(f=None, returnType=None, functionType=None):
    """Vectorised UDF: ``f(pandas.Series, ...) -> pandas.Series`` applied to the rank's whole
    slice at once (scalar pandas UDF)."""
    def wrap(fn):
        rt = T.parse_type(returnType) if returnType is not None else T.DoubleType()

        def call(*cols):
            es = [_e(a) for a in cols]

            def ev(df):
                import pandas as pd
                n = len(df)
                series = [pd.Series(_host(e.eval(df), n)) for e in es]
                res = pd.Series(fn(*series)).tolist()
                if isinstance(rt, T.NumericType):
                    return _num_out([None if not _nn(v) else v for v in res],
                                    torch.int64 if isinstance(rt, (T.IntegerType, T.LongType)) else torch.float64,
                                    df.device)
                return _str_out(res)
            return Expr(ev, f"{getattr(fn, '__name__', 'pandas_udf')}({', '.join(e.name for e in es)})",
                        _refs(*es))
        call.func, call.returnType = fn, rt
        return call
    if f is not None and callable(f):
        return wrap(f)
    if f is not None and returnType is None:
        returnType = f
    return wrap


# ============================================================================ round-out batch
# hyperbolic / trig / rounding
def sinh(c): return _num_map("SINH", torch.sinh, c)
def cosh(c): return _num_map("COSH", torch.cosh, c)
def tanh(c): return _num_map("TANH", torch.tanh, c)
def asinh(c): return _num_map("ASINH", torch.asinh, c)
def acosh(c): return _num_map("ACOSH", torch.acosh, c)
def atanh(c): return _num_map("ATANH", torch.atanh, c)
def cot(c): return _num_map("COT", lambda x: 1.0 / torch.tan(x), c)
def sec(c): return _num_map("SEC", lambda x: 1.0 / torch.cos(x), c)
def csc(c): return _num_map("CSC", lambda x: 1.0 / torch.sin(x), c)
def rint(c): return _num_map("rint", torch.round, c)       # torch.round is half-to-even, like Math.rint
def ln(c): return log(c)
def power(a, b): return pow(a, b)
def sign(c): return signum(c)
def positive(c): return _e(c)
def negative(c): return _num_map("negative", torch.neg, c)
def e(): return lit(math.e)
def pi(): return lit(math.pi)


def pmod(a, b):
    """Positive modulus (result has the divisor's sign convention of Spark: always >= 0 for b > 0)."""
    return _num_map("pmod", lambda x, y: torch.remainder(x, y) + 0.0, a, b)     # no -0.0


def mod(a, b):
    return _num_map("mod", lambda x, y: torch.fmod(x, y), a, b)


def try_divide(a, b):
    """a / b, null where b == 0 (instead of an error)."""
    ea, eb = _e(a), _e(b)

    def f(df):
        x, y = ea.eval(df), eb.eval(df)
        xd, yd = x.data.to(torch.float64), y.data.to(torch.float64).to(x.data.device)
        ok = yd != 0
        for c in (x, y):
            if getattr(c, "valid", None) is not None:
                ok = ok & c.valid.to(ok.device)
        return C.NumericColumn(torch.where(ok, xd / torch.where(ok, yd, torch.ones_like(yd)), torch.zeros_like(xd)),
                               ok, T.DoubleType())
    return Expr(f, f"try_divide({ea.name}, {eb.name})", _refs(ea, eb))


def try_add(a, b): return _e(a) + _e(b)


def width_bucket(v, min_, max_, numBucket):
    """Bucket 1..numBucket of v in [min, max); 0 below, numBucket+1 at/above max."""
    def wb(x, lo, hi, nb):
        if x < lo:
            return 0
        if x >= hi:
            return int(nb) + 1
        return int((x - lo) / (hi - lo) * nb) + 1
    return _host_map("width_bucket", wb, v, min_, max_, numBucket, kind="int")


# strings
def left(c, n): return _host_map("left", lambda s, k: str(s)[:builtins.max(int(k), 0)], c, n)
def right(c, n): return _host_map("right", lambda s, k: str(s)[-int(k):] if int(k) > 0 else "", c, n)
def char_length(c): return length(c)
def character_length(c): return length(c)
def ucase(c): return upper(c)
def lcase(c): return lower(c)
def bit_length(c): return _host_map("bit_length", lambda s: 8 * len(str(s).encode()), c, kind="int")
def octet_length(c): return _host_map("octet_length", lambda s: len(str(s).encode()), c, kind="int")
def startswith(c, p): return _host_map("startswith", lambda s, q: str(s).startswith(str(q)), c, p, kind="bool")
def endswith(c, p): return _host_map("endswith", lambda s, q: str(s).endswith(str(q)), c, p, kind="bool")
def contains(c, p): return _host_map("contains", lambda s, q: str(q) in str(s), c, p, kind="bool")


def _sql_like(pattern: str, flags=0):
    rx = "".join(".*" if ch == "%" else "." if ch == "_" else re.escape(ch) for ch in pattern)
    return re.compile(rx, flags | re.S)


def like(c, pattern):
    rx = _sql_like(pattern if isinstance(pattern, str) else pattern.eval_literal())
    return _host_map("like", lambda s: rx.fullmatch(str(s)) is not None, c, kind="bool")


def ilike(c, pattern):
    rx = _sql_like(pattern if isinstance(pattern, str) else pattern.eval_literal(), re.I)
    return _host_map("ilike", lambda s: rx.fullmatch(str(s)) is not None, c, kind="bool")


def rlike(c, pattern):
    rx = re.compile(pattern if isinstance(pattern, str) else pattern.eval_literal())
    return _host_map("rlike", lambda s: rx.search(str(s)) is not None, c, kind="bool")


regexp_like = rlike
regexp = rlike


def regexp_extract_all(c, pattern, idx=1):
    rx = re.compile(pattern if isinstance(pattern, str) else pattern.eval_literal())
    return _host_map("regexp_extract_all", lambda s: [m.group(idx) if rx.groups else m.group(0)
                                                      for m in rx.finditer(str(s))], c, kind="array")


def split_part(c, delimiter, partNum):
    def sp(s, d, k):
        parts = str(s).split(str(d))
        k = int(k)
        if k == 0:
            raise ValueError("split_part index must not be 0")
        return parts[k - 1] if 0 < k <= len(parts) else (parts[k] if -len(parts) <= k < 0 else "")
    return _host_map("split_part", sp, c, delimiter, partNum)


def overlay(src, replace, pos, len=-1):  # noqa: A002
    def ov(s, r, p, n):
        s, r, p, n = str(s), str(r), int(p), int(n)
        n = builtins.len(r) if n < 0 else n
        return s[:p - 1] + r + s[p - 1 + n:]
    return _host_map("overlay", ov, src, replace, pos, len)


def encode(c, charset):
    return _host_map("encode", lambda s: str(s).encode(charset.replace("-", "").lower()
                                                        .replace("utf8", "utf-8")), c, kind="str")


def decode(c, charset):
    return _host_map("decode", lambda b: (b if isinstance(b, (bytes, bytearray)) else str(b).encode())
                     .decode(charset.replace("-", "").lower().replace("utf8", "utf-8")), c)


# nulls / misc
def nvl2(c, v_if_not_null, v_if_null):
    return when(_e(c).isNotNull(), _e(v_if_not_null)).otherwise(_e(v_if_null))


def equal_null(a, b):
    ea, eb = _e(a), _e(b)

    def f(df):
        n = len(df)
        x, y = _host(ea.eval(df), n), _host(eb.eval(df), n)
        return _num_out([(u is None and v is None) or (u is not None and v is not None and u == v)
                         for u, v in zip(x, y)], torch.bool, df.device)
    return Expr(f, f"equal_null({ea.name}, {eb.name})", _refs(ea, eb))


def raise_error(msg):
    def f(df):
        if len(df):
            raise RuntimeError(str(msg))
        return _num_out([], torch.float64, df.device)
    return Expr(f, "raise_error()", ())


def curdate(): return current_date()


def timestamp_seconds(c):
    import datetime as _dt
    return _host_map("timestamp_seconds", lambda v: _dt.datetime.utcfromtimestamp(float(v))
                     .strftime("%Y-%m-%d %H:%M:%S"), c)


def make_date(y, m, d):
    import datetime as _dt
    return _host_map("make_date", lambda a, b, c_: _dt.date(int(a), int(b), int(c_)).isoformat(), y, m, d)


def from_utc_timestamp(c, tz):
    import pandas as pd

    def cv(v, z):
        t = pd.Timestamp(str(v))
        t = t.tz_localize("UTC") if t.tzinfo is None else t
        return t.tz_convert(str(z)).tz_localize(None).strftime("%Y-%m-%d %H:%M:%S")
    return _host_map("from_utc_timestamp", cv, c, tz)


def to_utc_timestamp(c, tz):
    import pandas as pd

    def cv(v, z):
        t = pd.Timestamp(str(v))
        t = t.tz_localize(str(z)) if t.tzinfo is None else t
        return t.tz_convert("UTC").tz_localize(None).strftime("%Y-%m-%d %H:%M:%S")
    return _host_map("to_utc_timestamp", cv, c, tz)


def window(timeColumn, windowDuration: str, slideDuration=None, startTime=None):
    """Time window struct(start, end).  Tumbling (no slide, or slide == duration): the one
    window holding each timestamp.  Sliding (slide < duration): a generator -- each row is
    repeated once per window [start, start + duration) that holds it, windows starting at
    startTime + k * slide, in ascending start order (Spark's sliding-window expansion)."""
    import pandas as pd
    dur = pd.Timedelta(windowDuration).total_seconds()
    off = pd.Timedelta(startTime).total_seconds() if startTime else 0.0
    slide = pd.Timedelta(slideDuration).total_seconds() if slideDuration else dur
    if not 0 < slide <= dur:
        raise ValueError(f"slideDuration must be positive and <= windowDuration, got {slideDuration}")
    from ..frame.dataframe import Row
    fmt = lambda x: pd.Timestamp(x, unit="s").strftime("%Y-%m-%d %H:%M:%S")  # noqa: E731

    if slide == dur:
        def w(v):
            t = pd.Timestamp(str(v)).timestamp()
            s0 = math.floor((t - off) / dur) * dur + off
            return Row._make(["start", "end"], [fmt(s0), fmt(s0 + dur)])
        return _host_map("window", w, timeColumn, kind="array").alias("window")

    def ws(v):
        t = pd.Timestamp(str(v)).timestamp()
        last = math.floor((t - off) / slide) * slide + off          # latest start <= t
        starts = []
        s0 = last
        while s0 + dur > t:
            starts.append(s0)
            s0 -= slide
        return [Row._make(["start", "end"], [fmt(a), fmt(a + dur)]) for a in reversed(starts)]
    return explode(_host_map("window", ws, timeColumn, kind="array")).alias("window")


def inline(c):
    """Generator over an array of structs: one row per struct (DataFrame.select expands
    it to the struct's fields)."""
    out = explode(c)
    out._inline = True
    return out


def json_tuple(c, *fields):
    import json as _json

    def jt(s):
        try:
            d = _json.loads(str(s))
        except ValueError:
            return [None] * len(fields)
        return [None if d.get(k) is None else (v if isinstance(v := d.get(k), str) else _json.dumps(v))
                for k in fields]
    return _host_map("json_tuple", jt, c, kind="array")


def schema_of_json(js):
    import json as _json
    s = js if isinstance(js, str) else js.eval_literal()

    def ty(v):
        if isinstance(v, bool):
            return "BOOLEAN"
        if isinstance(v, int):
            return "BIGINT"
        if isinstance(v, float):
            return "DOUBLE"
        if isinstance(v, list):
            return f"ARRAY<{ty(v[0]) if v else 'STRING'}>"
        if isinstance(v, dict):
            return "STRUCT<" + ", ".join(f"{k}: {ty(x)}" for k, x in sorted(v.items())) + ">"
        return "STRING"
    return lit(ty(_json.loads(s)))


# arrays / maps
def array_repeat(c, count): return _host_map("array_repeat", lambda v, k: [v] * int(k), c, count, kind="array")
def array_append(c, v): return _host_map("array_append", lambda a, x: list(a) + [x], c, v, kind="array")
def array_prepend(c, v): return _host_map("array_prepend", lambda a, x: [x] + list(a), c, v, kind="array")
def array_compact(c): return _host_map("array_compact", lambda a: [x for x in a if x is not None], c, kind="array")
def array_size(c): return size(c)
def cardinality(c): return size(c)


def array_insert(c, pos, value):
    def ins(a, p, x):
        a, p = list(a), int(p)
        if p == 0:
            raise ValueError("array_insert position must not be 0")
        i = p - 1 if p > 0 else len(a) + p + 1
        if i > len(a):
            a += [None] * (i - len(a))
        a.insert(builtins.max(i, 0), x)
        return a
    return _host_map("array_insert", ins, c, pos, value, kind="array")


def arrays_overlap(a, b):
    def ov(x, y):
        sx, sy = {v for v in x if v is not None}, {v for v in y if v is not None}
        if sx & sy:
            return True
        return None if (len(x) and len(y) and (None in x or None in y)) else False
    return _host_map("arrays_overlap", ov, a, b, kind="bool")


def shuffle(c, seed=None):
    import random as _random
    rng = _random.Random(seed)
    return _host_map("shuffle", lambda a: rng.sample(list(a), len(a)), c, kind="array")


def try_element_at(c, i):
    def ta(a, k):
        k = int(k)
        if isinstance(a, dict):
            return a.get(k)
        return (a[k - 1] if k > 0 else a[k]) if k != 0 and len(a) >= builtins.abs(k) else None
    return _host_map("try_element_at", ta, c, i, kind="str")


def map_concat(*cols):
    def mc(*ms):
        out = {}
        for m in ms:
            out.update(m)
        return out
    return _host_map("map_concat", mc, *cols, kind="array")


def map_entries(c):
    from ..frame.dataframe import Row
    return _host_map("map_entries", lambda m: [Row._make(["key", "value"], [k, v]) for k, v in m.items()], c,
                     kind="array")


def map_from_arrays(k, v): return _host_map("map_from_arrays", lambda a, b: dict(zip(a, b)), k, v, kind="array")


def map_from_entries(c):
    return _host_map("map_from_entries", lambda a: {(r[0]): r[1] for r in a}, c, kind="array")


# ---- higher-order functions: the lambda is evaluated ONCE per rank over the flattened
# elements (a local frame of all array elements), so its body runs as vectorised column
# code (device ops for numeric bodies), not per element in Python.
def _lambda_params(f):
    import inspect
    return [p for p in inspect.signature(f).parameters]


def _run_lambda(df, f, params: dict, owner: np.ndarray, outer_refs):
    """Evaluate ``f(*cols)`` over a local frame whose columns are the flattened lambda
    parameters; columns of ``df`` the body references are repeated per element."""
    import pandas as pd
    from ..frame.dataframe import DataFrame
    n_el = len(owner)
    def series(v):
        nn = [x for x in v if x is not None]
        if any(isinstance(x, (list, dict, str, bytes)) for x in nn) or not nn:
            return pd.Series(v, dtype=object)
        if len(nn) == len(v):
            return pd.Series(v)
        # numeric with nulls: nullable column (null-aware coalesce / isNull in the body)
        if all(isinstance(x, (int, np.integer)) and not isinstance(x, bool) for x in nn):
            return pd.Series(pd.array(v, dtype="Int64"))
        return pd.Series(pd.array(v, dtype="Float64"))
    data = {f"__lp{i}": series(v) for i, v in enumerate(params.values())}
    local = df.session.local_view()
    body = f(*[col(f"__lp{i}") for i in range(len(params))])
    body = _e(body)
    extra = [r for r in body.refs if not r.startswith("__lp") and r in df.columns]
    if n_el == 0:
        return []
    frame = local.createDataFrame(pd.DataFrame(data)) if data else None
    if extra:
        idx = torch.from_numpy(owner.astype(np.int64))
        cols = OrderedDict(frame._cols)
        for r in extra:
            cols[r] = df._col(r).take(idx.to(_dev_of(df._col(r), df.device)))
        frame = DataFrame(local, cols, n_el)
    return _host(body.eval(frame), n_el)


def _dev_of(c, default):
    d = getattr(getattr(c, "data", None), "device", None)
    return d if d is not None else ("cpu" if isinstance(c, C.HostColumn) else default)


def _hof(name, c, f, combine, kind="array", map_input=False):
    ec = _e(c)

    def ev(df):
        n = len(df)
        vals = _host(ec.eval(df), n)
        nargs = len(_lambda_params(f))
        owner, flat_a, flat_b = [], [], []
        for r, v in enumerate(vals):
            if v is None:
                continue
            items = list(v.items()) if map_input else list(enumerate(v))
            for i, x in items:
                owner.append(r)
                if map_input:
                    flat_a.append(i)
                    flat_b.append(x)
                else:
                    flat_a.append(x)
                    flat_b.append(i)
        owner = np.asarray(owner, dtype=np.int64)
        params = {"a": flat_a} if nargs == 1 else {"a": flat_a, "b": flat_b}
        res = _run_lambda(df, f, params, owner, ())
        per = [[] for _ in range(n)]
        for o, a_, b_, y in zip(owner.tolist(), flat_a, flat_b, res):
            per[o].append((a_, b_, y))
        out = [None if vals[r] is None else combine(per[r]) for r in range(n)]
        if kind == "array":
            arr = np.empty(n, dtype=object)
            for i, x in enumerate(out):
                arr[i] = x
            return C.ArrayColumn(arr)
        return _num_out(out, torch.bool, df.device)
    return Expr(ev, f"{name}({ec.name}, lambdafunction)", ec.refs)


def transform(c, f):
    """``transform(arr, x -> f(x))`` / ``(x, i) -> f(x, i)``."""
    return _hof("transform", c, f, lambda items: [y for _, _, y in items])


def filter(c, f):  # noqa: A001
    return _hof("filter", c, f, lambda items: [a for a, _, y in items if y])


def exists(c, f):
    return _hof("exists", c, f, lambda items: builtins.any(bool(y) for _, _, y in items if y is not None),
                kind="bool")


def forall(c, f):
    return _hof("forall", c, f, lambda items: builtins.all(bool(y) for _, _, y in items if y is not None),
                kind="bool")


def transform_values(c, f):
    return _hof("transform_values", c, f, lambda items: {k: y for k, _, y in items}, map_input=True)


def transform_keys(c, f):
    return _hof("transform_keys", c, f, lambda items: {y: v for _, v, y in items}, map_input=True)


def map_filter(c, f):
    return _hof("map_filter", c, f, lambda items: {k: v for k, v, y in items if y}, map_input=True)


def zip_with(left_, right_, f):
    el, er = _e(left_), _e(right_)

    def ev(df):
        n = len(df)
        a, b = _host(el.eval(df), n), _host(er.eval(df), n)
        owner, fa, fb = [], [], []
        for r, (x, y) in enumerate(zip(a, b)):
            if x is None or y is None:
                continue
            m = builtins.max(len(x), len(y))
            for i in range(m):
                owner.append(r)
                fa.append(x[i] if i < len(x) else None)
                fb.append(y[i] if i < len(y) else None)
        owner = np.asarray(owner, dtype=np.int64)
        res = _run_lambda(df, f, {"a": fa, "b": fb}, owner, ())
        per = [[] for _ in range(n)]
        for o, y in zip(owner.tolist(), res):
            per[o].append(y)
        arr = np.empty(n, dtype=object)
        for r in range(n):
            arr[r] = None if a[r] is None or b[r] is None else per[r]
        return C.ArrayColumn(arr)
    return Expr(ev, f"zip_with({el.name}, {er.name}, lambdafunction)", _refs(el, er))


def aggregate(c, initialValue, merge, finish=None):
    """Left fold of each array: vectorised across rows one element position at a time
    (``max(len)`` evaluations of ``merge`` over the rows that still have elements)."""
    ec, ei = _e(c), _e(initialValue)

    def ev(df):
        n = len(df)
        vals = _host(ec.eval(df), n)
        acc = list(_host(ei.eval(df), n))
        lens = [0 if v is None else len(v) for v in vals]
        for j in range(builtins.max(lens, default=0)):
            rows = [r for r in range(n) if lens[r] > j]
            res = _run_lambda(df, merge, {"acc": [acc[r] for r in rows], "x": [vals[r][j] for r in rows]},
                              np.asarray(rows, dtype=np.int64), ())
            for r, y in zip(rows, res):
                acc[r] = y
        if finish is not None and n:
            acc = _run_lambda(df, finish, {"acc": acc}, np.arange(n, dtype=np.int64), ())
        out = [None if vals[r] is None else acc[r] for r in range(n)]
        if builtins.all(isinstance(v, (int, float, bool)) or v is None for v in out):
            return _num_out(out, torch.float64 if builtins.any(isinstance(v, float) for v in out) else torch.int64,
                            df.device)
        return _str_out(out)
    return Expr(ev, f"aggregate({ec.name}, ...)", _refs(ec, ei))


reduce = aggregate


# ---- aggregates
def median(c):
    """Exact median (Spark ``median`` = ``percentile(c, 0.5)``, linear interpolation)."""
    out = Agg("median", _e(c), f"median({_e(c).name})")
    return out


def mode(c):
    return Agg("mode", _e(c), f"mode({_e(c).name})")


def product(c):
    return Agg("product", _e(c), f"product({_e(c).name})")


def count_if(c):
    return Agg("count", when(_e(c), lit(1)), f"count_if({_e(c).name})")


def bool_and(c): return Agg("bool_and", _e(c), f"bool_and({_e(c).name})")
def bool_or(c): return Agg("bool_or", _e(c), f"bool_or({_e(c).name})")


every = bool_and
some = bool_or


def any_value(c, ignoreNulls=False):
    return Agg("first", _e(c), f"any_value({_e(c).name})")


def max_by(c, ord_):
    out = Agg("max_by", array(_e(ord_), _e(c)), f"max_by({_e(c).name}, {_e(ord_).name})")
    return out


def min_by(c, ord_):
    return Agg("min_by", array(_e(ord_), _e(c)), f"min_by({_e(c).name}, {_e(ord_).name})")


def first_value(c, ignoreNulls=False): return first(c, ignoreNulls)
def last_value(c, ignoreNulls=False): return last(c, ignoreNulls)


# ---------------------------------------------------------------- Spark 3.4 / 3.5 additions
def array_agg(c): return Agg("collect_list", _e(c), f"array_agg({_e(c).name})")
def bit_and(c): return Agg("bit_and", _e(c), f"bit_and({_e(c).name})")
def bit_or(c): return Agg("bit_or", _e(c), f"bit_or({_e(c).name})")
def bit_xor(c): return Agg("bit_xor", _e(c), f"bit_xor({_e(c).name})")


def bit_count(c):
    """Set bits of the value sign-extended to 64 bits (Spark BitwiseCount evaluates
    java.lang.Long.bitCount for every integral input type)."""
    return _host_map("bit_count", lambda v: builtins.bin(int(v) & 0xFFFFFFFFFFFFFFFF).count("1"), c, kind="int")


date_diff = datediff
day = dayofmonth


def weekday(c): return _date_map("weekday", lambda s: s.dt.dayofweek.astype("float"), c)   # Monday = 0


def date_from_unix_date(c):
    import datetime as _dt
    return _host_map("date_from_unix_date",
                     lambda v: (_dt.date(1970, 1, 1) + _dt.timedelta(days=int(v))).isoformat(), c)


def make_timestamp(years, months, days, hours, mins, secs):
    import datetime as _dt

    def mk(y, mo, d, h, mi, s):
        s = float(s)
        t = _dt.datetime(int(y), int(mo), int(d), int(h), int(mi), int(s), int(builtins.round((s % 1) * 1e6)))
        return t.strftime("%Y-%m-%d %H:%M:%S") + (f".{t.microsecond:06d}".rstrip("0") if t.microsecond else "")
    return _host_map("make_timestamp", mk, years, months, days, hours, mins, secs)


def get(c, index):
    """0-based array element, null when out of range (Spark 3.4 ``get``)."""
    idx = index if isinstance(index, (E.Expr, str)) else E.lit(int(index))
    return _host_map("get", lambda v, i: v[int(i)] if 0 <= int(i) < len(v) else None, c, idx, kind="str")


def json_array_length(c):
    def f(s):
        try:
            v = _json.loads(str(s))
        except ValueError:
            return None
        return len(v) if isinstance(v, list) else None
    return _host_map("json_array_length", f, c, kind="int")


def json_object_keys(c):
    def f(s):
        try:
            v = _json.loads(str(s))
        except ValueError:
            return None
        return list(v.keys()) if isinstance(v, dict) else None
    return _host_map("json_object_keys", f, c, kind="array")


def map_contains_key(c, key):
    k = key if isinstance(key, E.Expr) else E.lit(key)
    return _host_map("map_contains_key", lambda m, kk: kk in m, c, k, kind="bool")


def named_struct(*cols):
    """named_struct(lit(name1), col1, lit(name2), col2, ...)."""
    if len(cols) % 2:
        raise ValueError("named_struct expects name, value pairs")
    names = [n.eval_literal() if hasattr(n, "eval_literal") else str(n) for n in cols[::2]]
    return struct(*[_e(v).alias(k) for k, v in zip(names, cols[1::2])])


def negate(c): return -_e(c)


def position(substr, c, start=None):
    """1-based position of ``substr`` in ``c`` at or after ``start`` (0 when absent)."""
    st = start if start is not None else E.lit(1)
    return _host_map("position", lambda sub, s, p: str(s).find(str(sub), builtins.max(int(p) - 1, 0)) + 1,
                     substr if isinstance(substr, E.Expr) else E.lit(substr), c,
                     st if isinstance(st, E.Expr) else E.lit(int(st)), kind="int")


def regexp_count(c, regexp):
    return _host_map("regexp_count", lambda s, p: len(re.findall(str(p), str(s))), c,
                     regexp if isinstance(regexp, E.Expr) else E.lit(regexp), kind="int")


def regexp_substr(c, regexp):
    def f(s, p):
        m = re.search(str(p), str(s))
        return m.group(0) if m else None
    return _host_map("regexp_substr", f, c, regexp if isinstance(regexp, E.Expr) else E.lit(regexp))


def replace(src, search, replace=None):  # noqa: A002
    rep = E.lit("") if replace is None else (replace if isinstance(replace, E.Expr) else E.lit(replace))
    return _host_map("replace", lambda s, a, b: str(s).replace(str(a), str(b)), src,
                     search if isinstance(search, E.Expr) else E.lit(search), rep)


def substr(c, pos, length_=None):
    """substr(str, pos[, len]) with column or literal arguments (1-based, like substring)."""
    p = pos if isinstance(pos, E.Expr) else E.lit(int(pos))
    n = E.lit(1 << 30) if length_ is None else (length_ if isinstance(length_, E.Expr) else E.lit(int(length_)))

    def f(s, a, b):
        s, a, b = str(s), int(a), int(b)
        start = a - 1 if a > 0 else (len(s) + a if a < 0 else 0)
        lo = builtins.max(start, 0)
        return s[lo:builtins.max(lo, start + b)] if b > 0 else ""
    return _host_map("substr", f, c, p, n)


def try_subtract(a, b): return _e(a) - _e(b)
def try_multiply(a, b): return _e(a) * _e(b)


def url_encode(c):
    """application/x-www-form-urlencoded as java.net.URLEncoder (UTF-8): letters, digits
    and ``.-*_`` stay, space -> ``+``, everything else (``~`` included) is %XX."""
    from urllib.parse import quote_plus
    return _host_map("url_encode", lambda s: quote_plus(str(s), safe="*").replace("~", "%7E"), c)


def url_decode(c):
    from urllib.parse import unquote_plus
    return _host_map("url_decode", lambda s: unquote_plus(str(s)), c)


def uuid():
    import uuid as _uuid
    return Expr(lambda df: _str_out([str(_uuid.uuid4()) for _ in range(len(df))]), "uuid()")


def _csv_cast(v, dt):
    if v == "":
        return None
    name = dt.simpleString() if hasattr(dt, "simpleString") else str(dt)
    try:
        if name in ("int", "bigint", "smallint", "tinyint"):
            return int(v)
        if name in ("double", "float") or name.startswith("decimal"):
            return float(v)
        if name == "boolean":
            return {"true": True, "false": False}.get(v.strip().lower())
    except ValueError:
        return None                      # PERMISSIVE mode: a malformed field becomes null
    return v


def _ddl_schema(schema) -> T.StructType:
    """StructType, DDL string ("a INT, b STRING") or STRUCT<...> string -> StructType."""
    if isinstance(schema, T.StructType):
        return schema
    text = (schema.eval_literal() if hasattr(schema, "eval_literal") else str(schema)).strip()
    if text.lower().startswith("struct<") and text.endswith(">"):
        text = text[7:-1]
    return T.parse_schema(text)


def from_csv(c, schema, options=None):
    """CSV text -> struct of the DDL schema's fields (Spark ``from_csv``; options ``sep``)."""
    import csv as _csv
    from ..frame.dataframe import Row
    st = _ddl_schema(schema)
    sep = (options or {}).get("sep", (options or {}).get("delimiter", ","))
    names, types = [f.name for f in st.fields], [f.dataType for f in st.fields]

    def fc(s):
        vals = next(_csv.reader([str(s)], delimiter=sep), [])
        vals = (vals + [""] * len(names))[:len(names)]
        return Row._make(names, [_csv_cast(v, t) for v, t in zip(vals, types)])
    return _host_map("from_csv", fc, c, kind="array")


def schema_of_csv(csv, options=None):
    """DDL of a CSV sample (Spark ``schema_of_csv``: columns _c0, _c1, ... with inferred types)."""
    import csv as _csv
    text = csv.eval_literal() if hasattr(csv, "eval_literal") else str(csv)
    sep = (options or {}).get("sep", ",")
    vals = next(_csv.reader([text], delimiter=sep), [])

    def typ(v):
        for t, f in (("INT", int), ("DOUBLE", float)):
            try:
                f(v)
                return t
            except ValueError:
                pass
        return "BOOLEAN" if v.lower() in ("true", "false") else "STRING"
    ddl = "STRUCT<" + ", ".join(f"_c{i}: {typ(v)}" for i, v in enumerate(vals)) + ">"
    return E.lit(ddl)


def years(c):
    """Partition transform years(ts) (writeTo().partitionedBy); evaluates to the year."""
    return year(c)


def map_zip_with(col1, col2, f):
    """Merge two maps key-wise with ``f(k, v1, v2)`` over the union of their keys (a key
    missing from one side passes null for that side)."""
    e1, e2 = _e(col1), _e(col2)

    def ev(df):
        n = len(df)
        a, b = _host(e1.eval(df), n), _host(e2.eval(df), n)
        owner, ks, v1, v2 = [], [], [], []
        for r, (x, y) in enumerate(zip(a, b)):
            if x is None or y is None:
                continue
            for k in list(x.keys()) + [k for k in y.keys() if k not in x]:
                owner.append(r)
                ks.append(k)
                v1.append(x.get(k))
                v2.append(y.get(k))
        owner = np.asarray(owner, dtype=np.int64)
        res = _run_lambda(df, f, {"k": ks, "v1": v1, "v2": v2}, owner, ()) if len(owner) else []
        per = [dict() for _ in range(n)]
        for o, k, y in zip(owner.tolist(), ks, res):
            per[o][k] = y
        arr = np.empty(n, dtype=object)
        for r in range(n):
            arr[r] = None if a[r] is None or b[r] is None else per[r]
        return C.ArrayColumn(arr)
    return Expr(ev, f"map_zip_with({e1.name}, {e2.name}, lambdafunction)", _refs(e1, e2))


def histogram_numeric(c, nBins):
    """Approximate histogram as an array of (x, y) = (bin centre, count) structs."""
    n = nBins.eval_literal() if hasattr(nBins, "eval_literal") else int(nBins)
    a = Agg("histogram_numeric", _e(c), f"histogram_numeric({_e(c).name}, {n})")
    a.param = int(n)
    return a


# ---------------------------------------------------------------- aliases and small built-ins
try_sum = sum
try_avg = avg
sha = sha1
to_timestamp_ltz = to_timestamp
to_timestamp_ntz = to_timestamp
try_to_timestamp = to_timestamp
localtimestamp = current_timestamp
dateadd = date_add


def printf(format, *cols):  # noqa: A002
    fmt = format.eval_literal() if hasattr(format, "eval_literal") else format
    return format_string(fmt, *cols)


def _epoch(name, scale, c):
    import pandas as pd

    def f(v):
        t = pd.Timestamp(str(v))
        t = t.tz_convert("UTC").tz_localize(None) if t.tzinfo is not None else t
        return int(t.value // scale)
    return _host_map(name, f, c, kind="int")


def unix_date(c): return _epoch("unix_date", 86_400 * 10 ** 9, c)
def unix_seconds(c): return _epoch("unix_seconds", 10 ** 9, c)
def unix_millis(c): return _epoch("unix_millis", 10 ** 6, c)
def unix_micros(c): return _epoch("unix_micros", 10 ** 3, c)


def to_unix_timestamp(c, format=None):  # noqa: A002
    return unix_timestamp(c) if format is None else \
        unix_timestamp(c, format.eval_literal() if hasattr(format, "eval_literal") else format)


def _from_epoch(name, per_second, c):
    import datetime as _dt

    def f(v):
        t = _dt.datetime(1970, 1, 1) + _dt.timedelta(microseconds=int(v) * (10 ** 6 // per_second))
        return t.strftime("%Y-%m-%d %H:%M:%S") + (f".{t.microsecond:06d}".rstrip("0") if t.microsecond else "")
    return _host_map(name, f, c)


def timestamp_millis(c): return _from_epoch("timestamp_millis", 1000, c)
def timestamp_micros(c): return _from_epoch("timestamp_micros", 10 ** 6, c)


def date_part(field, source):
    """date_part('YEAR' | 'MONTH' | 'DAY' | 'HOUR' | 'MINUTE' | 'SECOND' | 'QUARTER' | 'WEEK' |
    'DAYOFWEEK' | 'DOY', source)."""
    f = (field.eval_literal() if hasattr(field, "eval_literal") else str(field)).strip().upper()
    table = {"YEAR": year, "YEARS": year, "Y": year, "MONTH": month, "MON": month, "MONTHS": month,
             "DAY": dayofmonth, "D": dayofmonth, "DAYS": dayofmonth, "HOUR": hour, "H": hour, "HOURS": hour,
             "MINUTE": minute, "MIN": minute, "MINUTES": minute, "SECOND": second, "S": second, "SEC": second,
             "SECONDS": second, "QUARTER": quarter, "QTR": quarter, "WEEK": weekofyear, "W": weekofyear,
             "WEEKS": weekofyear, "DAYOFWEEK": dayofweek, "DOW": dayofweek, "DOY": dayofyear}
    if f not in table:
        raise ValueError(f"date_part: unsupported field {f!r}")
    return table[f](source)


datepart = date_part
extract = date_part


def convert_timezone(sourceTz, targetTz, sourceTs=None):
    """convert_timezone([sourceTz, ]targetTz, sourceTs): wall clock in sourceTz -> targetTz."""
    import pandas as pd
    if sourceTs is None:
        sourceTz, targetTz, sourceTs = E.lit("UTC"), sourceTz, targetTz

    def cv(v, a, b):
        t = pd.Timestamp(str(v))
        t = t.tz_localize(str(a)) if t.tzinfo is None else t
        return t.tz_convert(str(b)).tz_localize(None).strftime("%Y-%m-%d %H:%M:%S")
    return _host_map("convert_timezone", cv, sourceTs, sourceTz, targetTz)


def _const(name, value):
    return Expr(lambda df: _str_out([value] * len(df)), f"{name}()")


def current_timezone(): return _const("current_timezone", "UTC")
def current_user(): return _const("current_user", __import__("getpass").getuser())
def user(): return current_user()
def current_catalog(): return _const("current_catalog", "spark_catalog")
def current_database(): return _const("current_database", "default")
def current_schema(): return current_database()
def version(): return _const("version", "3.5.0 orange3-spark-amd")


def mask(c, upperChar=None, lowerChar=None, digitChar=None, otherChar=None):
    """Spark mask(): upper -> 'X', lower -> 'x', digits -> 'n', others kept (or otherChar)."""
    lit_of = lambda v, d: d if v is None else (v.eval_literal() if hasattr(v, "eval_literal") else v)  # noqa: E731
    up, lo, dg, ot = lit_of(upperChar, "X"), lit_of(lowerChar, "x"), lit_of(digitChar, "n"), lit_of(otherChar, None)

    def m(s):
        out = []
        for ch in str(s):
            if ch.isupper():
                out.append(ch if up is None else up)
            elif ch.islower():
                out.append(ch if lo is None else lo)
            elif ch.isdigit():
                out.append(ch if dg is None else dg)
            else:
                out.append(ch if ot is None else ot)
        return "".join(out)
    return _host_map("mask", m, c)


def find_in_set(str, str_array):  # noqa: A002
    """1-based index of ``str`` in the comma-separated ``str_array`` (0 if absent or if str has a comma)."""
    def f(s, arr):
        s = builtins.str(s)
        if "," in s:
            return 0
        parts = builtins.str(arr).split(",")
        return parts.index(s) + 1 if s in parts else 0
    return _host_map("find_in_set", f, str, str_array, kind="int")


def elt(*inputs):
    """elt(n, in1, in2, ...): the n-th input (1-based), null when out of range."""
    es = [_e(a) for a in inputs]

    def f(df):
        n = len(df)
        cols = [_host(e.eval(df), n) for e in es]
        out = []
        for r in range(n):
            k = cols[0][r]
            out.append(cols[int(k)][r] if k is not None and 1 <= int(k) < len(cols) else None)
        return _str_out([None if v is None else builtins.str(v) for v in out])
    return Expr(f, f"elt({', '.join(e.name for e in es)})", _refs(*es))


def chr(c):  # noqa: A001
    """Character of code point n mod 256 (Spark chr / char); '' for negative n."""
    return _host_map("chr", lambda v: "" if int(v) < 0 else builtins.chr(int(v) % 256), c)


char = chr


def shiftrightunsigned(c, numBits: int):
    """``>>>`` at the column's width (Spark ShiftRightUnsigned: Java ``>>>`` on an int for
    byte/short/int columns, on a long for bigint), the shift taken mod the width."""
    e = _e(c)

    def f(df):
        col = e.eval(df)
        narrow = isinstance(col, C.NumericColumn) and col.data.dtype in (torch.int8, torch.int16, torch.int32)
        bits, mask = (32, 0xFFFFFFFF) if narrow else (64, 0xFFFFFFFFFFFFFFFF)
        k = int(numBits) % bits
        vals = _host(col, len(df))
        return _num_out([None if v is None else (int(v) & mask) >> k for v in vals], torch.int64, df.device)
    return Expr(f, f"shiftrightunsigned({e.name}, {int(numBits)})", _refs(e))


def to_binary(c, format=None):  # noqa: A002
    """to_binary(str[, 'hex' | 'utf-8' | 'base64']) -> bytes."""
    fmt = "hex" if format is None else (format.eval_literal() if hasattr(format, "eval_literal") else format).lower()

    def f(s):
        s = builtins.str(s)
        try:
            if fmt == "hex":
                return _binascii.unhexlify(s if len(s) % 2 == 0 else "0" + s)
            if fmt == "base64":
                return _b64.b64decode(s)
            return s.encode("utf-8")
        except (ValueError, _binascii.Error):
            return None
    return _host_map("to_binary", f, c, kind="array")
