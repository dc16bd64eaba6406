"""pandas <-> Orange Table conversion and SQL pretty-printing.

Reference behaviour (orangecontrib/spark/utils/data_utils.py):
  * ``construct_domain`` (:35-52): a numeric column is Continuous if it has >= 13 unique
    values, is a float dtype, or max > #unique; otherwise Discrete with sorted string
    values; non-numeric columns become String metas; no class variable.
  * ``pandas_to_orange`` (:21-24): X = attribute columns, metas = string columns, Y = None.
  * ``orange_to_pandas`` (:27-32) is broken there (``csv.writer(delimiter='')`` raises,
    quirk Q1); here it is a direct columnar conversion of X / Y / metas.
  * ``format_sql`` (:17-18) used sqlparse (absent here): an in-house keyword upper-caser
    and clause re-indenter with the same intent.
  * ``save_csv_IO`` (:55-74) wrote an Orange table into an in-memory CSV with an empty
    delimiter (TypeError) and handed it over un-rewound; ``load_csvIO`` (:77-114) built its
    rows lazily and returned nothing (quirk Q2).  Both are fixed here: comma-separated,
    header row of variable names, buffer rewound / rows materialised.
"""
from __future__ import annotations

import csv
import io
import re
from collections import OrderedDict

import numpy as np
import pandas as pd

from . import orange_compat as O


def construct_domain(df: pd.DataFrame):
    attributes: "OrderedDict[str, object]" = OrderedDict()
    metas: "OrderedDict[str, object]" = OrderedDict()
    for name, dtype in df.dtypes.items():
        col = df[name]
        if np.issubdtype(dtype, np.number) and not np.issubdtype(dtype, np.bool_):
            nun = len(col.unique())
            if nun >= 13 or np.issubdtype(dtype, np.inexact) or (col.max() > nun):
                attributes[name] = O.ContinuousVariable(str(name))
            else:
                vals = sorted(col.astype(str).unique().tolist())
                attributes[name] = O.DiscreteVariable(str(name), values=vals)
        else:
            metas[name] = O.StringVariable(str(name))
    domain = O.Domain(list(attributes.values()), metas=list(metas.values()))
    return domain, list(attributes.keys()), list(metas.keys())


def pandas_to_orange(df: pd.DataFrame):
    domain, attributes, metas = construct_domain(df)
    X = np.empty((len(df), len(attributes)), dtype=np.float64)
    for j, (name, var) in enumerate(zip(attributes, domain.attributes)):
        if isinstance(var, O.DiscreteVariable):
            lookup = {v: i for i, v in enumerate(var.values)}
            X[:, j] = [lookup[str(v)] for v in df[name].astype(str)]
        else:
            X[:, j] = df[name].to_numpy(dtype=np.float64)
    M = df[metas].to_numpy(dtype=object) if metas else None
    return O.Table.from_numpy(domain=domain, X=X, Y=None, metas=M, W=None)


def orange_to_pandas(table) -> pd.DataFrame:
    dom = table.domain
    data = OrderedDict()

    def put(var, column):
        if getattr(var, "is_discrete", False) or isinstance(var, O.DiscreteVariable):
            vals = list(var.values)
            data[var.name] = [None if (c is None or (isinstance(c, float) and np.isnan(c))) else vals[int(c)]
                              for c in column]
        elif getattr(var, "is_string", False) or isinstance(var, O.StringVariable):
            data[var.name] = [None if c is None else str(c) for c in column]
        else:
            data[var.name] = np.asarray(column, dtype=np.float64)
    X = np.asarray(table.X)
    for j, v in enumerate(dom.attributes):
        put(v, X[:, j])
    Y = np.asarray(table.Y)
    if Y.ndim == 1:
        Y = Y[:, None]
    for j, v in enumerate(dom.class_vars):
        put(v, Y[:, j])
    M = np.asarray(table.metas, dtype=object)
    for j, v in enumerate(dom.metas):
        put(v, M[:, j])
    return pd.DataFrame(data)


def save_csv_IO(data) -> io.StringIO:
    """Orange Table or pandas DataFrame -> rewound in-memory CSV (header = column names)."""
    pdf = data if isinstance(data, pd.DataFrame) else orange_to_pandas(data)
    buf = io.StringIO()
    w = csv.writer(buf, delimiter=",", lineterminator="\n")
    w.writerow([str(c) for c in pdf.columns])
    for row in pdf.itertuples(index=False):
        w.writerow(["" if v is None or (isinstance(v, float) and np.isnan(v)) else v for v in row])
    buf.seek(0)
    return buf


def load_csvIO(buf, delimiter: str = ","):
    """In-memory CSV -> (header, rows); numeric cells parsed as float, empty cells None."""
    if hasattr(buf, "seek"):
        buf.seek(0)
    rows = list(csv.reader(buf, delimiter=delimiter))
    if not rows:
        return [], []

    def cell(v):
        if v == "":
            return None
        try:
            return float(v)
        except ValueError:
            return v
    return rows[0], [[cell(v) for v in r] for r in rows[1:]]


_KEYWORDS = ["select", "from", "where", "group by", "order by", "having", "limit", "join", "left join",
             "right join", "inner join", "outer join", "full outer join", "on", "and", "or", "not", "as", "in",
             "is", "null", "distinct", "count", "sum", "avg", "min", "max", "union", "all", "case", "when",
             "then", "else", "end", "asc", "desc", "like", "between", "show", "databases", "tables", "create",
             "table", "insert", "into", "values", "cast", "by", "with", "intersect", "except", "minus", "exists",
             "using", "natural", "cross join", "left semi join", "left anti join", "lateral view", "pivot", "filter",
             "over", "partition by", "rows", "range", "preceding", "following", "unbounded", "current row",
             "tablesample", "explain", "cache", "uncache", "view", "overwrite", "nulls first", "nulls last"]
_CLAUSES = ["select", "from", "where", "group by", "order by", "having", "limit", "union", "intersect", "except",
            "minus", "left join", "right join", "inner join", "full outer join", "cross join", "left semi join",
            "left anti join", "lateral view", "join"]


def format_sql(sql: str) -> str:
    """Upper-case keywords and put each top-level clause on its own line."""
    toks = re.split(r"('(?:[^']|'')*'|\"[^\"]*\")", sql.strip())
    out = []
    for t in toks:
        if t.startswith(("'", '"')):
            out.append(t)
            continue
        t = re.sub(r"\s+", " ", t)
        for kw in sorted(_KEYWORDS, key=len, reverse=True):
            t = re.sub(rf"\b{kw}\b", kw.upper(), t, flags=re.I)
        for cl in sorted(_CLAUSES, key=len, reverse=True):
            t = re.sub(rf"\s+\b({cl.upper()})\b", r"\n\1", t)
        t = re.sub(r"\b(LEFT|RIGHT|INNER|OUTER|CROSS|SEMI|ANTI)\n(JOIN)\b", r"\1 \2", t)   # keep "LEFT JOIN" whole
        t = re.sub(r",\s*(?![^()]*\))", ",\n       ", t) if "SELECT" in t else t
        out.append(t)
    return "".join(out).strip()
