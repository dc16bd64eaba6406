"""The rest of the pyspark ``DataFrame`` surface: multiset operators, replace, tail,
statistics (``df.stat``: approxQuantile / corr / cov / crosstab / freqItems / sampleBy),
rebalancing / hash repartitioning, unpivot, pandas UDF entry points and plan no-ops.

Everything is distributed the same way as the core operators: statistics are per-rank
partial sums combined with one collective, quantiles are an exact distributed selection
(bisection on order-preserving int64 codes, one ``all_reduce`` of P counts per step --
64 passes over HBM-resident data cost milliseconds on the GPU, so no sketch error is
needed), and row movement goes through :func:`shuffle.exchange` (``all_to_all_v``).
"""
from __future__ import annotations

import json
import math
from collections import OrderedDict

import numpy as np
import torch

from . import column as C
from . import expr as E
from . import types as T


def _local_comm(df):
    from ..parallel.comm import LocalComm
    return LocalComm(df.device)


class DataFrameExtras:
    """Mixed into :class:`DataFrame` (see module docstring)."""

    # ------------------------------------------------------------------ multiset ops
    def _setop(self, other, rule):
        from .shuffle import keep_mask
        if len(other.columns) != len(self.columns):
            raise ValueError(f"{rule} requires the same number of columns")
        other = other.toDF(*self.columns)
        return self._mask(keep_mask(self, None, rule, other, None))

    def intersect(self, other):
        """Distinct rows present in both (SQL INTERSECT)."""
        return self._setop(other, "intersect")

    def intersectAll(self, other):
        """Rows in both, keeping min(count_a, count_b) duplicates (INTERSECT ALL)."""
        return self._setop(other, "intersect_all")

    def subtract(self, other):
        """Distinct rows of this frame absent from ``other`` (EXCEPT DISTINCT)."""
        return self._setop(other, "subtract")

    def exceptAll(self, other):
        """Rows of this frame minus ``other`` as multisets (EXCEPT ALL)."""
        return self._setop(other, "except_all")

    # ------------------------------------------------------------------ renames / misc
    def toDF(self, *names):
        if len(names) != len(self.columns):
            raise ValueError(f"toDF needs {len(self.columns)} names, got {len(names)}")
        return self._new(OrderedDict(zip(names, self._cols.values())))

    def withColumnsRenamed(self, colsMap: dict):
        return self._new(OrderedDict((colsMap.get(k, k), c) for k, c in self._cols.items()))

    def transform(self, func, *args, **kwargs):
        return func(self, *args, **kwargs)

    def hint(self, name, *parameters):
        return self

    def isLocal(self) -> bool:
        return self.comm.world_size == 1

    def isEmpty(self) -> bool:
        return self.count() == 0

    def checkpoint(self, eager: bool = True):
        return self.cache()

    localCheckpoint = checkpoint

    def explain(self, extended=False, mode=None):
        """Frames are materialised eagerly; the 'plan' is the physical layout."""
        lines = ["== Physical Layout ==",
                 f"rows={self.count()} partitions={self.comm.world_size} backend={self.comm.backend} "
                 f"device={self.device}"]
        for k, c in self._cols.items():
            where = "host" if isinstance(c, C.HostColumn) else str(getattr(getattr(c, "data", None), "device",
                                                                           self.device))
            lines.append(f"  {k}: {type(c).__name__}[{c.dtype}] on {where}")
        if self.lineage is not None:
            lines.append(f"  lineage: {type(self.lineage).__name__} (generated on demand)")
        text = "\n".join(lines)
        if self.comm.rank == 0:
            print(text)
        return text

    # ------------------------------------------------------------------ rows to the driver
    def tail(self, num: int):
        sizes = self.partition_sizes()
        total = sum(sizes)
        lo = max(0, total - num)
        off = self.row_offset()
        keep = torch.arange(max(lo - off, 0), self._n, dtype=torch.int64) if off + self._n > lo \
            else torch.zeros(0, dtype=torch.int64)
        return self._take(keep).collect()

    def toLocalIterator(self, prefetchPartitions=False):
        return iter(self.collect())

    def toJSON(self, use_unicode=True):
        def conv(v):
            if hasattr(v, "toArray"):
                return np.asarray(v.toArray()).tolist()
            if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
                return None
            return v
        out = []
        for r in self.collect():
            out.append(json.dumps({k: conv(v) for k, v in r.asDict().items() if v is not None}))
        return out

    def foreach(self, f):
        """Runs ``f(row)`` on the rank that owns the row (like Spark executors)."""
        names = list(self._cols)
        lists = [c.to_pylist() for c in self._cols.values()]
        from .dataframe import Row
        for vals in zip(*lists):
            f(Row._make(names, vals))

    def foreachPartition(self, f):
        from .dataframe import Row
        names = list(self._cols)
        lists = [c.to_pylist() for c in self._cols.values()]
        f(iter([Row._make(names, vals) for vals in zip(*lists)]))

    # ------------------------------------------------------------------ value replace
    def replace(self, to_replace, value=None, subset=None):
        """Spark ``DataFrame.replace``: scalar / list / dict mapping; numeric mappings apply
        to numeric columns, string mappings to string columns."""
        if isinstance(to_replace, dict):
            mapping = dict(to_replace)
            if value is not None and subset is None and isinstance(value, (list, tuple, str)):
                subset = value
        else:
            src = list(to_replace) if isinstance(to_replace, (list, tuple)) else [to_replace]
            dst = list(value) if isinstance(value, (list, tuple)) else [value] * len(src)
            if len(src) != len(dst):
                raise ValueError("to_replace and value lists should be of the same length")
            mapping = dict(zip(src, dst))
        if isinstance(subset, str):
            subset = [subset]
        out = OrderedDict()
        for k, c in self._cols.items():
            if subset is not None and k not in subset:
                out[k] = c
                continue
            if isinstance(c, C.NumericColumn) and not isinstance(c.dtype, T.BooleanType):
                num = {a: b for a, b in mapping.items() if isinstance(a, (int, float)) and not isinstance(a, bool)}
                if not num:
                    out[k] = c
                    continue
                d = c.data.clone()
                valid = None if c.valid is None else c.valid.clone()
                orig = c.data
                for a, b in num.items():
                    hit = (orig == a) if not (isinstance(a, float) and math.isnan(a)) else torch.isnan(orig.double())
                    if c.valid is not None:
                        hit = hit & c.valid
                    if b is None:
                        valid = (torch.ones_like(hit) if valid is None else valid) & ~hit
                    else:
                        d = torch.where(hit, torch.tensor(b, dtype=d.dtype, device=d.device), d)
                out[k] = C.NumericColumn(d, valid, c.dtype)
            elif isinstance(c, C.StringColumn):
                smap = {a: b for a, b in mapping.items() if isinstance(a, str)}
                if not smap:
                    out[k] = c
                    continue
                vals = np.array([smap.get(v, v) if v is not None else None for v in c.values], dtype=object)
                out[k] = C.StringColumn(vals)
            else:
                out[k] = c
        return self._new(out)

    # ------------------------------------------------------------------ statistics
    @property
    def stat(self):
        return DataFrameStatFunctions(self)

    def approxQuantile(self, col, probabilities, relativeError=0.0):
        """Exact quantiles (relativeError 0 accuracy at any setting): distributed
        bisection on order-preserving codes.  Returns the smallest value v with
        rank(v) >= p * (n - 1) (Spark's definition at error 0).  NaN/null skipped."""
        from .shuffle import _order_code
        if isinstance(col, (list, tuple)):
            return [self.approxQuantile(c, probabilities, relativeError) for c in col]
        probs = [float(p) for p in probabilities]
        if any(p < 0 or p > 1 for p in probs):
            raise ValueError("probabilities must be in [0, 1]")
        c = self._col(col) if isinstance(col, str) else col.eval(self)
        if not isinstance(c, C.NumericColumn):
            raise TypeError("approxQuantile needs a numeric column")
        d = c.data.to(torch.float64)
        ok = ~c.null_mask().to(d.device) & ~torch.isnan(d)
        code = _order_code(_local_comm(self), C.NumericColumn(d[ok]), True, True)
        n = self.comm.sum_scalar(int(code.numel()))
        if n == 0:
            return [None] * len(probs)
        lo_hi = torch.tensor([code.min().item() if code.numel() else (1 << 62),
                              -(code.max().item()) if code.numel() else (1 << 62)], dtype=torch.int64)
        lo_hi = self.comm.all_reduce(lo_hi.to(self.comm.device), "min").cpu()
        lo = torch.full((len(probs),), int(lo_hi[0]), dtype=torch.int64)
        hi = torch.full((len(probs),), -int(lo_hi[1]), dtype=torch.int64)
        target = torch.tensor([math.floor(p * (n - 1)) + 1 for p in probs], dtype=torch.int64)  # need count >= target
        code_dev = code
        for _ in range(66):
            if bool((lo >= hi).all()):
                break
            mid = (lo >> 1) + (hi >> 1) + (lo & hi & 1)          # floor((lo+hi)/2), no overflow
            cnt = torch.stack([(code_dev <= int(m)).sum() for m in mid.tolist()]).to(torch.int64) \
                if code_dev.numel() else torch.zeros(len(probs), dtype=torch.int64)
            cnt = self.comm.all_reduce(cnt.to(self.comm.device)).cpu()
            good = cnt >= target
            hi = torch.where(good, mid, hi)
            lo = torch.where(good, lo, mid + 1)
        bits = torch.where(lo < 0, lo ^ 0x7FFFFFFFFFFFFFFF, lo)
        vals = bits.view(torch.float64).tolist()
        return [float(v) for v in vals]

    def corr(self, col1, col2, method="pearson"):
        if method != "pearson":
            raise ValueError("only pearson correlation is supported (as in Spark)")
        s = self._moments(col1, col2)
        n, sx, sy, sxx, syy, sxy = s
        cov = sxy - sx * sy / n
        vx, vy = sxx - sx * sx / n, syy - sy * sy / n
        return cov / math.sqrt(vx * vy) if vx > 0 and vy > 0 else float("nan")

    def cov(self, col1, col2):
        n, sx, sy, _, _, sxy = self._moments(col1, col2)
        return (sxy - sx * sy / n) / (n - 1) if n > 1 else float("nan")

    def _moments(self, col1, col2):
        a = self._col(col1).data.to(torch.float64)
        b = self._col(col2).data.to(torch.float64)
        ok = ~self._col(col1).null_mask().to(a.device) & ~self._col(col2).null_mask().to(a.device)
        a, b = a[ok], b[ok]
        t = torch.stack([torch.tensor(float(a.numel()), dtype=torch.float64, device=a.device), a.sum(), b.sum(),
                         (a * a).sum(), (b * b).sum(), (a * b).sum()])
        return self.comm.all_reduce(t.to(self.comm.device)).cpu().tolist()

    def crosstab(self, col1, col2):
        """Contingency table: one row per distinct ``col1`` value, one column per
        distinct ``col2`` value (named ``<col1>_<col2>`` first column, as Spark)."""
        g = self.groupBy(col1, col2).count().toPandas()
        name = f"{col1}_{col2}"
        rows = sorted({str(v) for v in g[col1]}) if len(g) else []
        cols = sorted({str(v) for v in g[col2]}) if len(g) else []
        tab = {r: dict.fromkeys(cols, 0) for r in rows}
        for a, b, n in zip(g[col1], g[col2], g["count"]):
            tab[str(a)][str(b)] = int(n)
        full = OrderedDict([(name, C.StringColumn(np.array(rows, dtype=object)))])
        for cname in cols:
            full[cname] = C.NumericColumn(torch.tensor([tab[r][cname] for r in rows], dtype=torch.int64),
                                          None, T.LongType())
        return self._from_full(full)

    def freqItems(self, cols, support=None):
        """Items with frequency >= support * n per column (exact counts, so a superset-free
        answer; Spark's sketch may return false positives)."""
        if isinstance(cols, str):
            cols = [cols]
        support = 0.01 if support is None else float(support)
        n = self.count()
        out = OrderedDict()
        for c in cols:
            g = self.groupBy(c).count().toPandas()
            items = [None if (isinstance(v, float) and math.isnan(v)) else v
                     for v, k in zip(g[c], g["count"]) if k >= support * n]
            out[f"{c}_freqItems"] = C.ArrayColumn(_obj1(items))
        return self._from_full(out)

    def sampleBy(self, col, fractions: dict, seed=None):
        """Stratified Bernoulli sample: row kept with probability fractions[key] (0 for
        unlisted keys), keyed on (seed, global row) like ``sample``."""
        from ..ops import sampling
        seed = int(self.session.conf.seed() if seed is None else seed)
        c = self._col(col) if isinstance(col, str) else col.eval(self)
        vals = c.to_pylist()
        fr = torch.tensor([float(fractions.get(v, 0.0)) if v is not None else 0.0 for v in vals],
                          dtype=torch.float64, device=self.device)
        u = sampling.uniform(self._global_rows(), seed)
        return self._mask(u.to(fr.device).double() < fr)

    # ------------------------------------------------------------------ partitioning
    def repartition(self, numPartitions=None, *cols):
        """Rebalance rows over the ranks (the rank count is the partition count here).
        With columns: hash-exchange so equal keys share a rank.  Without: even ranges of
        the global row order.  Moves rows with ``all_to_all_v`` -- no driver gather."""
        from .shuffle import exchange, row_keys
        if isinstance(numPartitions, (str, E.Expr)):
            cols = (numPartitions,) + cols
        w = self.comm.world_size
        if w == 1:
            return self
        if cols:
            names = [c if isinstance(c, str) else c.name for c in cols]
            dest = row_keys(self, names)[:, 0] % w
        else:
            total = self.count()
            dest = (self._global_rows() * w) // max(total, 1)
        return exchange(self, dest)

    def coalesce(self, numPartitions=1):
        return self.repartition()

    def repartitionByRange(self, numPartitions, *cols):
        if isinstance(numPartitions, (str, E.Expr)):
            cols = (numPartitions,) + cols
        return self.orderBy(*cols)

    def sortWithinPartitions(self, *cols, ascending=True):
        from .shuffle import _order_code, local_sort_perm
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        asc = list(ascending) if isinstance(ascending, (list, tuple)) else [ascending] * len(cols)
        lc = _local_comm(self)
        codes = []
        for c, a in zip(cols, asc):
            e = E.col(c) if isinstance(c, str) else c
            a = bool(a) and not getattr(e, "_desc", False)
            nf = getattr(e, "_nulls_first", None)
            codes.append(_order_code(lc, e.eval(self), a, a if nf is None else nf).to(self.device))
        return self._take(local_sort_perm(codes)) if codes else self

    # ------------------------------------------------------------------ reshaping
    def unpivot(self, ids, values, variableColumnName, valueColumnName):
        ids = [ids] if isinstance(ids, str) else list(ids)
        values = [c for c in self.columns if c not in ids] if values is None else (
            [values] if isinstance(values, str) else list(values))
        if not values:
            raise ValueError("unpivot needs at least one value column")
        n, k = len(self), len(values)
        rep = torch.arange(n, dtype=torch.int64).repeat_interleave(k)
        out = OrderedDict()
        for i in ids:
            c = self._col(i)
            out[i] = c.take(rep if isinstance(c, C.HostColumn) else rep.to(self.device))
        out[variableColumnName] = C.StringColumn(np.array(values * n, dtype=object))
        vcols = [self._col(v) for v in values]
        if all(isinstance(v, C.NumericColumn) for v in vcols):
            data = torch.stack([v.data.to(torch.float64) for v in vcols], 1).reshape(-1)
            valid = torch.stack([~v.null_mask().to(data.device) for v in vcols], 1).reshape(-1)
            out[valueColumnName] = C.NumericColumn(data, None if bool(valid.all()) else valid, T.DoubleType())
        else:
            lists = [v.to_pylist() for v in vcols]
            out[valueColumnName] = C.StringColumn(np.array(
                [None if lists[j][r] is None else str(lists[j][r]) for r in range(n) for j in range(k)], dtype=object))
        return self._new(out, n * k)

    melt = unpivot

    # ------------------------------------------------------------------ pandas UDFs
    def mapInPandas(self, func, schema):
        """``func(iterator of pandas.DataFrame) -> iterator of pandas.DataFrame`` per rank."""
        import pandas as pd
        parts = list(func(iter([self.toPandas_local()])))
        pdf = pd.concat(parts, ignore_index=True) if parts else pd.DataFrame()
        return _frame_from_pandas(self, pdf, schema)

    def toPandas_local(self):
        import pandas as pd
        return pd.DataFrame(OrderedDict((k, c.to_pylist()) for k, c in self._cols.items()))


def _obj1(items):
    a = np.empty(1, dtype=object)
    a[0] = items
    return a


def _frame_from_pandas(df, pdf, schema):
    """Per-rank pandas result -> this rank's partition of a new DataFrame."""
    from .dataframe import DataFrame
    local = df.session.local_view().createDataFrame(pdf, schema) if len(pdf.columns) else None
    if local is None:
        return DataFrame(df.session, OrderedDict(), 0)
    return DataFrame(df.session, local._cols, len(local))


class DataFrameStatFunctions:
    def __init__(self, df):
        self.df = df

    def approxQuantile(self, col, probabilities, relativeError=0.0):
        return self.df.approxQuantile(col, probabilities, relativeError)

    def corr(self, col1, col2, method=None):
        return self.df.corr(col1, col2, method or "pearson")

    def cov(self, col1, col2):
        return self.df.cov(col1, col2)

    def crosstab(self, col1, col2):
        return self.df.crosstab(col1, col2)

    def freqItems(self, cols, support=None):
        return self.df.freqItems(cols, support)

    def sampleBy(self, col, fractions, seed=None):
        return self.df.sampleBy(col, fractions, seed)


class Observation:
    """``pyspark.sql.Observation``: named metrics collected by ``df.observe``.  Frames are
    materialised eagerly here, so the metrics are available as soon as ``observe``
    returns (Spark fills them at the first action)."""

    def __init__(self, name: str | None = None):
        self.name = name or f"observation_{id(self):x}"
        self._metrics = None

    @property
    def get(self) -> dict:
        if self._metrics is None:
            raise RuntimeError("observation has not been attached to a DataFrame")
        return self._metrics


_GLOBAL_TEMP: dict = {}     # ``global_temp`` database: views shared by every session of the process


class DataFrameExtras2:
    """Remaining pyspark ``DataFrame`` methods: grouping sets, regex column selection,
    offset, observations, global temp views, schema coercion, Arrow batches and the
    streaming no-ops of a batch engine."""

    # ------------------------------------------------------------------ grouping sets
    def rollup(self, *cols):
        """Hierarchical subtotals: grouping sets (k1..kn), (k1..kn-1), ..., () ."""
        from .grouping_sets import GroupingSets, rollup_sets
        keys = _key_exprs(cols)
        return GroupingSets(self, keys, rollup_sets(len(keys)))

    def cube(self, *cols):
        """All 2**n grouping sets of the keys."""
        from .grouping_sets import GroupingSets, cube_sets
        keys = _key_exprs(cols)
        return GroupingSets(self, keys, cube_sets(len(keys)))

    # ------------------------------------------------------------------ selection
    def colRegex(self, colName: str):
        """Columns whose name fully matches the (optionally back-quoted) regex; expands
        in ``select``."""
        import re
        pat = colName[1:-1] if colName.startswith("`") and colName.endswith("`") else colName
        rx = re.compile(pat)
        names = [k for k in self.columns if rx.fullmatch(k)]
        return _ColumnList(names)

    def offset(self, num: int):
        """Skip the first ``num`` rows of the global row order."""
        off = self.row_offset()
        start = max(0, min(self._n, num - off))
        return self._take(torch.arange(start, self._n, dtype=torch.int64))

    def observe(self, observation, *exprs):
        """Compute the aggregate ``exprs`` over this frame into ``observation`` (an
        :class:`Observation` or a name) and return the frame unchanged."""
        if isinstance(observation, str):
            observation = Observation(observation)
        row = self.agg(*exprs).collect()[0]
        observation._metrics = row.asDict()
        self._observations = getattr(self, "_observations", {})
        self._observations[observation.name] = observation
        return self

    # ------------------------------------------------------------------ views / session
    @property
    def sparkSession(self):
        return self.session

    @property
    def isStreaming(self) -> bool:
        return False

    def createGlobalTempView(self, name: str):
        if name in _GLOBAL_TEMP:
            raise ValueError(f"Temporary view '{name}' already exists")
        _GLOBAL_TEMP[name] = self

    def createOrReplaceGlobalTempView(self, name: str):
        _GLOBAL_TEMP[name] = self

    def inputFiles(self) -> list:
        """Files this frame was read from (empty for frames built in memory)."""
        return list(getattr(self, "_input_files", []))

    def sameSemantics(self, other) -> bool:
        """True when both frames hold the same column objects in the same layout (frames
        are materialised, so identical storage is identical semantics)."""
        return self.semanticHash() == other.semanticHash()

    def semanticHash(self) -> int:
        return hash(tuple((k, id(c), len(c)) for k, c in self._cols.items()))

    def withMetadata(self, columnName: str, metadata: dict):
        out = self._new(OrderedDict(self._cols))
        out._metadata = dict(getattr(self, "_metadata", {}))
        out._metadata[columnName] = dict(metadata)
        return out

    def to(self, schema):
        """Reorder / cast columns to ``schema`` (StructType or DDL string): columns are
        matched by name, missing nullable columns raise like Spark."""
        st = T.parse_schema(schema) if isinstance(schema, str) else schema
        cols = []
        for f in st.fields:
            if f.name not in self._cols:
                raise KeyError(f"column '{f.name}' not found")
            cols.append(E.col(f.name).cast(f.dataType).alias(f.name))
        return self.select(*cols)

    # ------------------------------------------------------------------ arrow / streaming no-ops
    def mapInArrow(self, func, schema):
        """``func(iterator of pyarrow.RecordBatch) -> iterator of RecordBatch`` per rank."""
        import pyarrow as pa
        batch = pa.RecordBatch.from_pandas(self.toPandas_local(), preserve_index=False)
        out = list(func(iter([batch])))
        pdf = pa.Table.from_batches(out).to_pandas() if out else __import__("pandas").DataFrame()
        return _frame_from_pandas(self, pdf, schema)

    def withWatermark(self, eventTime: str, delayThreshold: str):
        """Batch frames are complete: a watermark drops nothing."""
        if eventTime not in self._cols:
            raise KeyError(eventTime)
        return self

    def dropDuplicatesWithinWatermark(self, subset=None):
        return self.dropDuplicates(subset)

    def writeTo(self, table: str):
        return DataFrameWriterV2(self, table)


class DataFrameWriterV2:
    """``df.writeTo(table)``: create / replace / append / overwrite a warehouse table."""

    def __init__(self, df, table: str):
        self.df, self.table = df, table
        self._props: dict = {}

    def using(self, provider):
        return self

    def option(self, key, value):
        self._props[key] = value
        return self

    def options(self, **kw):
        self._props.update(kw)
        return self

    def tableProperty(self, key, value):
        return self.option(key, value)

    def partitionedBy(self, *cols):
        return self

    def create(self):
        self.df.session.catalog.saveAsTable(self.df, self.table, "error")

    def replace(self):
        if not self.df.session.catalog.tableExists(self.table):
            raise KeyError(f"table {self.table} does not exist")
        self.df.session.catalog.saveAsTable(self.df, self.table, "overwrite")

    def createOrReplace(self):
        self.df.session.catalog.saveAsTable(self.df, self.table, "overwrite")

    def append(self):
        self.df.session.catalog.saveAsTable(self.df, self.table, "append")

    def overwrite(self, condition=None):
        self.df.session.catalog.saveAsTable(self.df, self.table, "overwrite")

    overwritePartitions = overwrite


class _ColumnList(list):
    """Result of ``colRegex``: a list of column names that ``select`` expands in place."""
    _expand = True


def _key_exprs(cols):
    if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
        cols = tuple(cols[0])
    return [E.col(c) if isinstance(c, str) else c for c in cols]
