"""Row-sharded columnar DataFrame (replaces ``pyspark.sql.DataFrame``).

Every rank of the session holds a contiguous block of the global rows (its
*partition*); numeric/vector columns live in HBM.  Operations are eager; column
buffers are shared between DataFrames until modified.  Global operations (count,
collect/toPandas, sort, groupBy) use the session communicator (RCCL over xGMI on a
GPU node, gloo on CPU).

Reference call sites this type serves (orangecontrib/spark/...):
  * ``df.fillna(value, subset)``      widgets/data/spark_fill.py:63
  * ``df.sample(withReplacement, fraction, seed)``  widgets/data/spark_sample.py:70
  * ``df.cache()``                    widgets/data/spark_df_cache.py:39, base/spark_ml_transformer.py:134
  * ``df.withColumn('label', df[c].cast('double'))``  widgets/ml/spark_ml_dataset.py:578
  * ``df.columns``                    base/spark_ml_transformer.py:105, widgets/ml/spark_ml_dataset.py:422
  * ``df.toPandas()``                 widgets/data/spark_to_pandas.py:25, spark_to_orange.py:31
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Iterable

import numpy as np
import torch

from . import column as C
from . import expr as E
from . import types as T
from .extras import DataFrameExtras, DataFrameExtras2


class Row(tuple):
    """Immutable named row (``pyspark.sql.Row``-like)."""

    def __new__(cls, *args, **kwargs):
        if kwargs:
            names = list(kwargs.keys())
            r = tuple.__new__(cls, list(kwargs.values()))
            r.__fields__ = names
            return r
        r = tuple.__new__(cls, args)
        r.__fields__ = None
        return r

    @classmethod
    def _make(cls, names, values):
        r = tuple.__new__(cls, values)
        r.__fields__ = list(names)
        return r

    def asDict(self, recursive: bool = False):
        d = dict(zip(self.__fields__ or [], self))
        if recursive:
            def conv(v):
                if isinstance(v, Row):
                    return v.asDict(True)
                if isinstance(v, list):
                    return [conv(x) for x in v]
                if isinstance(v, dict):
                    return {k: conv(x) for k, x in v.items()}
                return v
            d = {k: conv(v) for k, v in d.items()}
        return d

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        try:
            return self[self.__fields__.index(item)]
        except (ValueError, AttributeError):
            raise AttributeError(item)

    def __getitem__(self, k):
        if isinstance(k, str):
            return tuple.__getitem__(self, self.__fields__.index(k))
        return tuple.__getitem__(self, k)

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self.__fields__, self)) + ")"
        return "Row" + tuple.__repr__(self)

    def __reduce__(self):
        return (Row._make, (self.__fields__, tuple(self)))


class StorageLevel:
    """Spark storage levels.  MEMORY_ONLY pins rows in HBM (rows beyond the budget of a
    synthetic table are recomputed from lineage); MEMORY_AND_DISK keeps the rows of dense
    vector columns beyond the HBM budget in pinned host memory and streams them through the
    GPU on every pass (frame/spill.py); DISK_ONLY keeps all of them on the host."""
    NONE = "NONE"
    MEMORY_ONLY = "MEMORY_ONLY"
    MEMORY_ONLY_2 = "MEMORY_ONLY_2"
    MEMORY_AND_DISK = "MEMORY_AND_DISK"
    MEMORY_AND_DISK_2 = "MEMORY_AND_DISK_2"
    MEMORY_AND_DISK_DESER = "MEMORY_AND_DISK_DESER"
    DISK_ONLY = "DISK_ONLY"
    DISK_ONLY_2 = "DISK_ONLY_2"
    OFF_HEAP = "OFF_HEAP"


class DataFrame(DataFrameExtras, DataFrameExtras2):
    def __init__(self, session, cols: "OrderedDict[str, C.Column]", nrows: int | None = None):
        self.session = session
        self._cols: OrderedDict = OrderedDict(cols)
        if nrows is None:
            nrows = len(next(iter(self._cols.values()))) if self._cols else 0
        self._n = int(nrows)
        for k, c in self._cols.items():
            if len(c) != self._n:
                raise ValueError(f"column {k!r} has {len(c)} rows, expected {self._n}")
        self._cached = False
        self._offset = None
        self.lineage = None  # optional SyntheticLineage (rows recomputable in-kernel)

    # ------------------------------------------------------------------ basics
    @property
    def comm(self):
        return self.session.comm

    @property
    def device(self):
        return self.session.device

    @property
    def rdd(self):
        """RDD of Rows: one partition per rank holding that rank's shard (rdd.py)."""
        from ..rdd import RDD
        df = self
        cache = {}

        def rows(p):
            if "rows" not in cache:
                names = list(df._cols)
                lists = [c.to_pylist() for c in df._cols.values()]
                cache["rows"] = [Row._make(names, vals) for vals in zip(*lists)]
            return cache["rows"]
        ctx = self.session.sparkContext
        return RDD(ctx, self.comm.world_size, rows, owner=lambda p: p)

    def __len__(self):
        return self._n

    @property
    def columns(self) -> list[str]:
        return list(self._cols.keys())

    @property
    def dtypes(self) -> list[tuple[str, str]]:
        return [(k, c.dtype.simpleString()) for k, c in self._cols.items()]

    @property
    def schema(self) -> T.StructType:
        st = T.StructType()
        for k, c in self._cols.items():
            md = {}
            if isinstance(c, (C.VectorColumn, C.SparseVectorColumn)):
                md = {"ml_attr": {"num_attrs": c.size}}
            st.add(k, c.dtype, True, md)
        return st

    def printSchema(self):
        print("root")
        for k, c in self._cols.items():
            print(f" |-- {k}: {c.dtype.simpleString()} (nullable = true)")

    def _col(self, name: str) -> C.Column:
        try:
            return self._cols[name]
        except KeyError:
            for k in self._cols:
                if k.lower() == name.lower():
                    return self._cols[k]
            qual, _, part = name.rpartition(".")
            if qual and qual.split(".")[-1] in self.__dict__.get("_aliases", ()):
                return self._col(part)           # "alias.col" after df.alias("alias")
            head, _, rest = name.partition(".")
            if rest and head in self._cols and isinstance(self._cols[head], C.HostColumn):
                c = self._cols[head]             # "struct.field[.field]" (e.g. window.start)
                for fld in rest.split("."):
                    c = E.struct_field(c, fld)
                return c
            raise KeyError(f"cannot resolve column '{name}' among {self.columns}")

    def column_data(self, name: str) -> C.Column:
        return self._col(name)

    def __getitem__(self, item):
        if isinstance(item, str):
            return E.bound_col(item, self._col(item), self)
        if isinstance(item, int):
            return E.col(self.columns[item])
        if isinstance(item, (list, tuple)):
            return self.select(*item)
        if isinstance(item, E.Expr):
            return self.filter(item)
        raise TypeError(item)

    def __getattr__(self, name):
        if name.startswith("_") or name in ("session", "lineage"):
            raise AttributeError(name)
        cols = self.__dict__.get("_cols", {})
        if name in cols:
            return E.bound_col(name, cols[name], self)
        raise AttributeError(name)

    def _col_bound(self, name: str, src, frame=None) -> C.Column:
        """Resolve ``other[name]`` on this frame: the column object itself when this frame holds
        it, the renamed copy a condition join made of it (``_prov``), else by name."""
        if src is not None:
            c = self._cols.get(name)
            if c is src:
                return c
            for ref, out in self.__dict__.get("_prov", ()):
                if ref() is src and out in self._cols:
                    return self._cols[out]
        return self._col(name)

    def _col_qualified(self, qual: str, name: str) -> C.Column:
        """SQL ``qual.name``: after a condition join the renamed copy of that side's column."""
        out = self.__dict__.get("_qual_map", {}).get((qual.split(".")[-1], name))
        if out in self._cols:
            return self._cols[out]
        head = qual.split(".")[0]
        if head in self._cols and isinstance(self._cols[head], C.HostColumn) and \
                head not in self.__dict__.get("_aliases", ()):
            return self._col(f"{qual}.{name}")          # SQL struct.field
        return self._col(name)

    def _new(self, cols, n=None) -> "DataFrame":
        return DataFrame(self.session, cols, self._n if n is None else n)

    def _resolve(self, c) -> tuple[str, C.Column]:
        if isinstance(c, str):
            if c == "*":
                raise ValueError("'*' handled by caller")
            col = self._col(c)
            if "." in c and c not in self._cols and c.split(".")[0] in self._cols:
                return c.rsplit(".", 1)[1], col  # struct field: Spark names the column by the field
            return c, col
        if isinstance(c, E.Expr):
            return c.name, c.eval(self)
        raise TypeError(f"unsupported column spec {c!r}")

    # ------------------------------------------------------------------ counts/offsets
    def count(self) -> int:
        return int(self.comm.sum_scalar(int(self._n)))

    def row_offset(self) -> int:
        """Global index of this partition's first row."""
        if self._offset is None:
            sizes = self.comm.all_gather_object(int(self._n))
            self._offset = int(sum(sizes[: self.comm.rank]))
        return self._offset

    def partition_sizes(self) -> list[int]:
        return self.comm.all_gather_object(int(self._n))

    # ------------------------------------------------------------------ projection
    def _with_windows(self, exprs):
        """Frame with the hidden window columns ``exprs`` need (sql/window.py), or None."""
        from ..sql.window import apply, window_refs
        keys = [k for k in window_refs(exprs) if k not in self._cols]
        return apply(self, keys) if keys else None

    def select(self, *cols) -> "DataFrame":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        win = self._with_windows([c for c in cols if isinstance(c, E.Expr)])
        if win is not None:
            return win.select(*[c if not (isinstance(c, str) and c == "*") else E.col(k)
                                for c in cols for k in ([c] if not (isinstance(c, str) and c == "*")
                                                        else list(self.columns))])
        if any(getattr(c, "_expand", False) for c in cols):           # colRegex results
            cols = tuple(x for c in cols for x in (c if getattr(c, "_expand", False) else [c]))
        gens = [c for c in cols if getattr(c, "_generator", None)]
        if len(gens) > 1:
            raise ValueError("Only one generator (explode) allowed per select clause")
        out = OrderedDict()
        for c in cols:
            if isinstance(c, str) and c == "*":
                out.update(self._cols)
                continue
            name, data = self._resolve(c)
            out[name] = data
        if gens:
            return self._explode(out, gens[0])
        return self._new(out)

    def _explode(self, out: "OrderedDict[str, C.Column]", g) -> "DataFrame":
        """Row expansion for explode/posexplode: one row per array element (rows with
        empty or null arrays disappear, as in Spark)."""
        name = g.name
        arr = out[name]
        outer = g._generator.endswith("_outer")          # explode_outer: empty / null -> one null row
        lists = [(list(v) if v is not None and len(v) else ([None] if outer else []))
                 for v in (arr.values if isinstance(arr, C.HostColumn) else arr.to_pylist())]
        lens = np.array([len(v) for v in lists], dtype=np.int64)
        idx = torch.from_numpy(np.repeat(np.arange(len(lists)), lens))
        flat = [x for v in lists for x in v]
        res = OrderedDict()
        for k, c in out.items():
            if k == name and getattr(g, "_inline", False):          # inline: struct fields -> columns
                fields = list(next((x for x in flat if x is not None), Row()).__fields__)
                for j, fname in enumerate(fields):
                    vals = [None if x is None else x[j] for x in flat]
                    obj = any(v is None or isinstance(v, (str, list, dict)) for v in vals)
                    res[fname] = C.from_numpy(np.array(vals, dtype=object) if obj else np.array(vals), self.device)
                continue
            if k == name:
                if g._generator.startswith("posexplode"):
                    res["pos"] = C.NumericColumn(torch.from_numpy(np.concatenate(
                        [np.arange(n_) for n_ in lens]) if len(lens) else np.zeros(0, dtype=np.int64)).to(self.device),
                        None, T.IntegerType())
                has_none = any(x is None for x in flat)
                first = next((x for x in flat if x is not None), None)
                if isinstance(first, (tuple, list, dict)):      # structs / arrays stay one value per row
                    vals = np.empty(len(flat), dtype=object)
                    for j, x in enumerate(flat):
                        vals[j] = x
                    res[k] = C.ArrayColumn(vals)
                    continue
                res[k] = C.from_numpy(np.array(flat, dtype=object) if flat and (has_none or isinstance(
                    next((x for x in flat if x is not None), ""), str)) else np.array(flat), self.device) \
                    if flat else C.StringColumn(np.array([], dtype=object))
            else:
                res[k] = c.take(idx.to(c.data.device) if isinstance(c, C.NumericColumn) else idx)
        return self._new(res, len(flat))

    def selectExpr(self, *exprs) -> "DataFrame":
        from ..sql.parser import parse_expression
        return self.select(*[parse_expression(e) for e in exprs])

    def withColumn(self, name: str, e) -> "DataFrame":
        if isinstance(e, E.Expr):
            win = self._with_windows([e])
            if win is not None:
                res = win.withColumn(name, e)
                return res.select(*[k for k in res.columns if not k.startswith("__win:")])
        data = e.eval(self) if isinstance(e, E.Expr) else E.lit(e).eval(self)
        out = OrderedDict(self._cols)
        out[name] = data
        return self._new(out)

    def withColumns(self, mapping: dict) -> "DataFrame":
        df = self
        for k, v in mapping.items():
            df = df.withColumn(k, v)
        return df

    def withColumnData(self, name: str, data: C.Column) -> "DataFrame":
        """Attach an already-computed column (used by ML transformers)."""
        if len(data) != self._n:
            raise ValueError("row count mismatch")
        out = OrderedDict(self._cols)
        out[name] = data
        df = self._new(out)
        df.lineage = self.lineage
        return df

    def withColumnRenamed(self, existing: str, new: str) -> "DataFrame":
        out = OrderedDict((new if k == existing else k, v) for k, v in self._cols.items())
        return self._new(out)

    def drop(self, *names) -> "DataFrame":
        drop_names = set()
        for n in names:
            src = getattr(n, "_src", None) if isinstance(n, E.Expr) else None
            if src is not None:                  # df.drop(other.id) after a condition join
                try:
                    obj = self._col_bound(n.name, src())
                except KeyError:
                    continue
                if self._cols.get(n.name) is obj:
                    drop_names.add(n.name)
                else:
                    drop_names.update(k for k, v in self._cols.items() if v is obj)
            else:
                drop_names.add(n.name if isinstance(n, E.Expr) else n)
        return self._new(OrderedDict((k, v) for k, v in self._cols.items() if k not in drop_names))

    def alias(self, name) -> "DataFrame":
        """Same columns (shared buffers) under a relation name: ``col("name.x")`` resolves
        here, and a condition join uses it to pick the side of a qualified reference."""
        out = self._new(self._cols)
        out.lineage, out._cached = self.lineage, self._cached
        out._aliases = frozenset([name])
        return out

    # ------------------------------------------------------------------ row selection
    def _take(self, idx: torch.Tensor) -> "DataFrame":
        idx = idx.to(torch.int64)
        out = OrderedDict()
        for k, c in self._cols.items():
            out[k] = c.take(idx.cpu() if isinstance(c, C.HostColumn) else idx.to(_col_device(c, self.device)))
        return self._new(out, int(idx.numel()))

    def _mask(self, mask: torch.Tensor) -> "DataFrame":
        out = OrderedDict()
        n = int(mask.sum().item())
        for k, c in self._cols.items():
            out[k] = c.mask_select(mask.cpu() if isinstance(c, C.HostColumn) else mask.to(_col_device(c, self.device)))
        return self._new(out, n)

    def filter(self, condition) -> "DataFrame":
        if isinstance(condition, str):
            from ..sql.parser import parse_expression
            condition = parse_expression(condition)
        c = condition.eval(self)
        m = c.data.bool()
        if c.valid is not None:
            m = m & c.valid
        return self._mask(m)

    where = filter

    def limit(self, num: int) -> "DataFrame":
        sizes = self.partition_sizes()
        off = sum(sizes[: self.comm.rank])
        keep = max(0, min(self._n, num - off))
        return self._take(torch.arange(keep, dtype=torch.int64))

    # ------------------------------------------------------------------ missing values
    def fillna(self, value, subset=None) -> "DataFrame":
        """Replace null/NaN (Spark ``DataFrame.fillna`` semantics: numeric value fills
        numeric columns, string value fills string columns, dict maps column->value)."""
        if isinstance(subset, str):
            subset = [subset]
        if isinstance(value, dict):
            items = value.items()
        else:
            items = [(k, value) for k in (subset or self.columns)]
        out = OrderedDict(self._cols)
        for k, v in items:
            if k not in out:
                if subset is not None or isinstance(value, dict):
                    raise KeyError(f"cannot resolve column '{k}'")
                continue
            c = out[k]
            if isinstance(c, C.NumericColumn) and isinstance(v, (int, float)) and not isinstance(v, bool):
                if isinstance(c.dtype, T.BooleanType):
                    continue
                m = c.null_mask()
                fill = torch.tensor(v, dtype=c.data.dtype, device=c.data.device) if c.data.is_floating_point() \
                    else torch.tensor(int(v), dtype=c.data.dtype, device=c.data.device)
                out[k] = C.NumericColumn(torch.where(m, fill, c.data), None, c.dtype)
            elif isinstance(c, C.NumericColumn) and isinstance(v, bool) and isinstance(c.dtype, T.BooleanType):
                m = c.null_mask()
                out[k] = C.NumericColumn(torch.where(m, torch.tensor(v, device=c.data.device), c.data), None, c.dtype)
            elif isinstance(c, C.StringColumn) and isinstance(v, str):
                vals = c.values.copy()
                for i, x in enumerate(vals):
                    if x is None:
                        vals[i] = v
                out[k] = C.StringColumn(vals)
        return self._new(out)

    def dropna(self, how: str = "any", thresh: int | None = None, subset=None) -> "DataFrame":
        names = [subset] if isinstance(subset, str) else (subset or self.columns)
        nulls = []
        for k in names:
            c = self._col(k)
            if isinstance(c, (C.NumericColumn, C.HostColumn)):
                nulls.append(c.null_mask().to(self.device))
        if not nulls:
            return self
        nn = torch.stack([~m for m in nulls]).sum(0)
        if thresh is not None:
            keep = nn >= thresh
        elif how == "all":
            keep = nn > 0
        else:
            keep = nn == len(nulls)
        return self._mask(keep)

    @property
    def na(self):
        return _NaFunctions(self)

    # ------------------------------------------------------------------ sampling
    def _global_rows(self) -> torch.Tensor:
        off = self.row_offset()
        return torch.arange(off, off + self._n, dtype=torch.int64, device=self.device)

    def sample(self, withReplacement=None, fraction=None, seed=None) -> "DataFrame":
        """Bernoulli (or Poisson when withReplacement) sampling keyed on (seed, global
        row), so the sample is independent of how rows are partitioned over GPUs."""
        if isinstance(withReplacement, float) and fraction is None:
            withReplacement, fraction = False, withReplacement
        if isinstance(fraction, int) and seed is None and isinstance(withReplacement, float):
            withReplacement, fraction, seed = False, withReplacement, fraction
        withReplacement = bool(withReplacement)
        fraction = float(0.5 if fraction is None else fraction)
        if fraction < 0:
            raise ValueError("fraction must be nonnegative")
        seed = int(self.session.conf.seed() if seed is None else seed)
        from ..ops import sampling
        rows = self._global_rows()
        if withReplacement:
            counts = sampling.poisson_counts(rows, seed, fraction)
            idx = torch.repeat_interleave(torch.arange(self._n, device=self.device), counts)
            return self._take(idx)
        if fraction > 1:
            raise ValueError("fraction must be <= 1 without replacement")
        return self._mask(sampling.bernoulli_mask(rows, seed, fraction))

    def randomSplit(self, weights, seed=None) -> list["DataFrame"]:
        w = np.asarray(weights, dtype=np.float64)
        if (w < 0).any() or w.sum() <= 0:
            raise ValueError("weights must be nonnegative with positive sum")
        cum = np.concatenate([[0.0], np.cumsum(w / w.sum())])
        seed = int(self.session.conf.seed() if seed is None else seed)
        from ..ops import sampling
        u = sampling.uniform(self._global_rows(), seed)
        outs = []
        for i in range(len(w)):
            hi = 1.0 + 1e-12 if i == len(w) - 1 else cum[i + 1]
            outs.append(self._mask((u >= cum[i]) & (u < hi)))
        return outs

    # ------------------------------------------------------------------ caching
    def cache(self) -> "DataFrame":
        """Materialise and pin the partition in HBM (everything is already eager; this
        also resolves any pending synthetic lineage into device memory within the
        session's cache budget)."""
        if self.lineage is not None:
            self.lineage.materialise(self)
        self._cached = True
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return self

    def persist(self, storageLevel=None) -> "DataFrame":
        """``MEMORY_AND_DISK`` / ``DISK_ONLY`` (and their variants): rows of dense vector
        columns beyond the HBM budget (``o3s.storage.hbmBudget`` bytes; default
        ``o3s.memory.fraction`` of the HBM this frame's vectors and the free memory span)
        move to pinned host memory and are streamed on every pass; other levels pin in HBM
        (:meth:`cache`)."""
        lvl = str(storageLevel if storageLevel is not None else StorageLevel.MEMORY_AND_DISK).upper()
        self.cache()
        if "DISK" in lvl or lvl == StorageLevel.OFF_HEAP:
            from . import spill
            budget = None
            if self.session.conf.get("o3s.storage.hbmBudget", None) in (None, "", "auto") \
                    and self.device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(self.device)
                mine = sum(c.data.numel() * c.data.element_size() for c in self._cols.values()
                           if isinstance(c, C.VectorColumn))
                budget = int((free + mine) * self.session.conf.memory_fraction())
            spill.spill_to_budget(self, budget, disk_only=lvl.startswith("DISK_ONLY"))
        self._level = lvl
        return self

    def unpersist(self, blocking=False) -> "DataFrame":
        self._cached = False
        self._level = None
        return self

    @property
    def is_cached(self) -> bool:
        return self._cached

    @property
    def storageLevel(self):
        lvl = getattr(self, "_level", None)
        if lvl is not None and self._cached:
            return lvl
        return StorageLevel.MEMORY_ONLY if self._cached else StorageLevel.NONE

    # ------------------------------------------------------------------ gathering
    def _gather_column(self, c: C.Column) -> C.Column:
        comm = self.comm
        if comm.world_size == 1:
            return c
        if isinstance(c, C.NumericColumn):
            data = comm.all_gather_v(c.data)
            valid = None
            anynull = comm.all_gather_object(c.valid is not None)
            if any(anynull):
                v = c.valid if c.valid is not None else torch.ones_like(c.data, dtype=torch.bool)
                valid = comm.all_gather_v(v.to(torch.uint8)).bool()
            return C.NumericColumn(data, valid, c.dtype)
        if isinstance(c, C.VectorColumn):
            return C.VectorColumn(comm.all_gather_v(c.data), c.size)
        parts = comm.all_gather_object(c)
        return C.Column.concat(parts)

    def _gathered(self) -> "OrderedDict[str, C.Column]":
        return OrderedDict((k, self._gather_column(c)) for k, c in self._cols.items())

    def collect(self) -> list[Row]:
        cols = self._gathered()
        names = list(cols.keys())
        if not names:
            return []
        lists = [c.to_pylist() for c in cols.values()]
        return [Row._make(names, vals) for vals in zip(*lists)]

    def take(self, num: int) -> list[Row]:
        return self.limit(num).collect()

    def head(self, n: int | None = None):
        if n is None:
            rows = self.take(1)
            return rows[0] if rows else None
        return self.take(n)

    def first(self):
        return self.head()

    def toPandas(self):
        import pandas as pd
        cols = self._gathered()
        data = OrderedDict()
        for k, c in cols.items():
            if isinstance(c, (C.VectorColumn, C.SparseVectorColumn)):
                data[k] = c.to_pylist()
            else:
                data[k] = c.to_numpy()
        return pd.DataFrame(data, columns=list(cols.keys()))

    def toArrow(self):
        import pyarrow as pa
        cols = self._gathered()
        arrays, names = [], []
        for k, c in cols.items():
            names.append(k)
            if isinstance(c, C.NumericColumn):
                a = c.data.detach().cpu()
                if a.dtype == torch.bfloat16:
                    a = a.float()
                mask = None if c.valid is None else ~c.valid.cpu().numpy()
                arrays.append(pa.array(a.numpy(), mask=mask))
            elif isinstance(c, (C.VectorColumn, C.SparseVectorColumn)):
                arrays.append(pa.array([list(r) for r in c.to_numpy()], type=pa.list_(pa.float64())))
            else:
                arrays.append(pa.array(c.to_pylist()))
        return pa.table(arrays, names=names)

    def show(self, n: int = 20, truncate: bool = True):
        rows = self.take(n)
        names = self.columns

        def fmt(v):
            s = "null" if v is None else str(v)
            return s[:17] + "..." if truncate and len(s) > 20 else s
        table = [[fmt(v) for v in r] for r in rows]
        widths = [max([len(h)] + [len(r[i]) for r in table]) for i, h in enumerate(names)]
        sep = "+" + "+".join("-" * w for w in widths) + "+"
        print(sep)
        print("|" + "|".join(h.rjust(w) for h, w in zip(names, widths)) + "|")
        print(sep)
        for r in table:
            print("|" + "|".join(v.rjust(w) for v, w in zip(r, widths)) + "|")
        print(sep)

    # ------------------------------------------------------------------ redistribution
    def _from_full(self, cols: "OrderedDict[str, C.Column]") -> "DataFrame":
        """Keep this rank's even slice of a replicated full-column set."""
        n = len(next(iter(cols.values()))) if cols else 0
        r, w = self.comm.rank, self.comm.world_size
        lo, hi = (n * r) // w, (n * (r + 1)) // w
        out = OrderedDict()
        for k, c in cols.items():
            c = c.slice(lo, hi)
            if isinstance(c, C.NumericColumn):
                c = C.NumericColumn(c.data.to(self.device), None if c.valid is None else c.valid.to(self.device), c.dtype)
            elif isinstance(c, C.VectorColumn):
                c = C.VectorColumn(c.data.to(self.device), c.size)
            out[k] = c
        return DataFrame(self.session, out, hi - lo)

    def orderBy(self, *cols, ascending=True) -> "DataFrame":
        """Distributed sample sort (frame/shuffle.py): range exchange on the leading key,
        stable local lexicographic sort.  ``col.desc()`` / ``asc_nulls_last()`` etc. honoured;
        Spark's null order (first when ascending, last when descending) by default."""
        from .shuffle import sort
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        asc = list(ascending) if isinstance(ascending, (list, tuple)) else [ascending] * len(cols)
        exprs, dirs, nulls = [], [], []
        for c, a in zip(cols, asc):
            e = E.col(c) if isinstance(c, str) else c
            a = bool(a) and not getattr(e, "_desc", False)
            nf = getattr(e, "_nulls_first", None)
            exprs.append(e)
            dirs.append(a)
            nulls.append(a if nf is None else nf)
        return sort(self, exprs, dirs, nulls)

    sort = orderBy

    def union(self, other: "DataFrame") -> "DataFrame":
        if len(other.columns) != len(self.columns):
            raise ValueError("union requires the same number of columns")
        out = OrderedDict()
        for (k, a), b in zip(self._cols.items(), other._cols.values()):
            out[k] = C.Column.concat([a, b])
        return self._new(out, self._n + len(other))

    unionAll = union

    def unionByName(self, other: "DataFrame") -> "DataFrame":
        return self.union(other.select(*self.columns))

    def distinct(self) -> "DataFrame":
        return self.dropDuplicates()

    def dropDuplicates(self, subset=None) -> "DataFrame":
        """First occurrence (global row order) of each distinct row / ``subset`` key:
        128-bit row keys hash-exchanged to owner ranks, survivors masked in place."""
        from .shuffle import keep_mask
        if isinstance(subset, str):
            subset = [subset]
        return self._mask(keep_mask(self, subset, "distinct"))

    drop_duplicates = dropDuplicates

    def join(self, other: "DataFrame", on=None, how: str = "inner") -> "DataFrame":
        from .join import join as _join
        return _join(self, other, on, how)

    def crossJoin(self, other: "DataFrame") -> "DataFrame":
        return self.join(other, None, "cross")

    # ------------------------------------------------------------------ aggregation
    def groupBy(self, *cols) -> "GroupedData":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        gens = [c for c in cols if getattr(c, "_generator", None)]
        if gens:                 # e.g. groupBy(window(ts, "10 minutes", "5 minutes")): expand rows first
            g = gens[0]
            return self.select("*", g).groupBy(*[E.col(g.name) if c is g else c for c in cols])
        return GroupedData(self, [E.col(c) if isinstance(c, str) else c for c in cols])

    groupby = groupBy

    def agg(self, *aggs) -> "DataFrame":
        return GroupedData(self, []).agg(*aggs)

    def describe(self, *cols) -> "DataFrame":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = cols[0]
        names = list(cols) or [k for k, c in self._cols.items()
                               if isinstance(c, (C.NumericColumn, C.StringColumn))]
        stats = ["count", "mean", "stddev", "min", "max"]
        res = OrderedDict(summary=np.array(stats, dtype=object))
        for k in names:
            c = self._col(k)
            vals = []
            if isinstance(c, C.NumericColumn):
                s = _numeric_stats(self.comm, c)
                vals = [s["count"], s["mean"], s["stddev"], s["min"], s["max"]]
            else:
                full = self._gather_column(c).to_pylist()
                nn = [v for v in full if v is not None]
                vals = [len(nn), None, None, min(nn) if nn else None, max(nn) if nn else None]
            res[k] = np.array([None if v is None else str(v) for v in vals], dtype=object)
        local = self.session.local_view()
        full = OrderedDict((k, C.StringColumn(v)) for k, v in res.items())
        return self._from_full(DataFrame(local, full)._cols)

    summary = describe

    # ------------------------------------------------------------------ io / catalog
    @property
    def write(self):
        from ..io import DataFrameWriter
        return DataFrameWriter(self)

    def createOrReplaceTempView(self, name: str) -> None:
        self.session.catalog.registerTempView(name, self)

    registerTempTable = createOrReplaceTempView
    createTempView = createOrReplaceTempView

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{k}: {t}" for k, t in self.dtypes) + "]"


def _col_device(c: C.Column, default):
    if isinstance(c, (C.NumericColumn, C.VectorColumn)):
        return c.data.device
    if isinstance(c, C.SparseVectorColumn):
        return c.indptr.device
    return default


def _hashable(v):
    if isinstance(v, list):
        return tuple(v)
    if hasattr(v, "toArray"):
        return tuple(np.asarray(v.toArray()).tolist())
    if isinstance(v, float) and math.isnan(v):
        return "NaN"
    return v


def _numeric_stats(comm, c: C.NumericColumn) -> dict:
    d = c.data.to(torch.float64)
    ok = ~c.null_mask()
    v = d[ok]
    n = float(v.numel())
    s = float(v.sum().item()) if n else 0.0
    ss = float((v * v).sum().item()) if n else 0.0
    mn = float(v.min().item()) if n else math.inf
    mx = float(v.max().item()) if n else -math.inf
    t = torch.tensor([n, s, ss], dtype=torch.float64, device=comm.device)
    comm.all_reduce(t)
    n, s, ss = t.tolist()
    mn = comm.all_gather_object(mn)
    mx = comm.all_gather_object(mx)
    mn, mx = min(mn), max(mx)
    mean = s / n if n else None
    var = (ss - n * mean * mean) / (n - 1) if n > 1 else None
    return {"count": int(n), "mean": mean, "stddev": math.sqrt(max(var, 0.0)) if var is not None else None,
            "min": mn if n else None, "max": mx if n else None, "sum": s}


class _NaFunctions:
    def __init__(self, df):
        self.df = df

    def fill(self, value, subset=None):
        return self.df.fillna(value, subset)

    def drop(self, how="any", thresh=None, subset=None):
        return self.df.dropna(how, thresh, subset)

    def replace(self, to_replace, value=None, subset=None):
        return self.df.replace(to_replace, value, subset)


class GroupedData:
    """groupBy(...).agg(...): per-partition partial aggregates, combined across ranks."""

    def __init__(self, df: DataFrame, keys: list):
        self.df, self.keys = df, keys

    def agg(self, *aggs) -> DataFrame:
        """Device-side partial aggregation per rank + merge by key (frame/groupby.py)."""
        from .groupby import aggregate
        if len(aggs) == 1 and isinstance(aggs[0], dict):
            aggs = tuple(getattr(E, fn if fn != "mean" else "avg")(c).alias(f"{fn}({c})") for c, fn in aggs[0].items())
        return self.df._from_full(aggregate(self.df, self.keys, list(aggs)))

    def count(self) -> DataFrame:
        return self.agg(E.count().alias("count"))

    def _simple(self, fn, cols):
        if not cols:
            cols = [k for k, c in self.df._cols.items() if isinstance(c, C.NumericColumn)
                    and k not in {e.name for e in self.keys}]
        return self.agg(*[getattr(E, fn)(c).alias(f"{fn}({c})") for c in cols])

    def sum(self, *cols):
        return self._simple("sum", cols)

    def avg(self, *cols):
        return self._simple("avg", cols)

    mean = avg

    def min(self, *cols):
        return self._simple("min", cols)

    def max(self, *cols):
        return self._simple("max", cols)

    def pivot(self, pivot_col, values=None) -> "PivotedData":
        return PivotedData(self.df, self.keys, E.col(pivot_col) if isinstance(pivot_col, str) else pivot_col, values)

    def applyInPandas(self, func, schema) -> DataFrame:
        """``func(pandas.DataFrame of one group) -> pandas.DataFrame``: rows are
        hash-exchanged by the grouping keys so every group lives on one rank, then each
        rank runs its groups (Spark's FlatMapGroupsInPandas)."""
        import pandas as pd
        from .extras import _frame_from_pandas
        names = [k.name for k in self.keys]
        local = self.df.repartition(*names).toPandas_local()
        with_key = _takes_key(func, 2)
        parts = [func(_group_key(k), g) if with_key else func(g)
                 for k, g in local.groupby(names, sort=False, dropna=False)] if len(local) else []
        return _frame_from_pandas(self.df, pd.concat(parts, ignore_index=True) if parts else pd.DataFrame(), schema)

    def cogroup(self, other: "GroupedData") -> "CoGroupedData":
        return CoGroupedData(self, other)


def _takes_key(func, n_frames: int) -> bool:
    """Spark passes the grouping key first when the function takes one more argument."""
    import inspect
    try:
        ps = [p for p in inspect.signature(func).parameters.values()
              if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
    except (TypeError, ValueError):
        return False
    return len(ps) == n_frames


def _group_key(k) -> tuple:
    """pandas group key -> Spark's key tuple (NaN -> None, numpy scalars -> python)."""
    k = k if isinstance(k, tuple) else (k,)
    out = []
    for v in k:
        if isinstance(v, float) and v != v:
            v = None
        out.append(v.item() if hasattr(v, "item") else v)
    return tuple(out)


class CoGroupedData:
    """``df1.groupBy(k).cogroup(df2.groupBy(k)).applyInPandas(f, schema)``: both sides are
    hash-exchanged by their keys (same keys -> same rank), then each rank calls
    ``f(left_group, right_group)`` -- or ``f(key, left_group, right_group)`` -- once per key
    present on either side, the missing side as an empty frame (Spark's
    FlatMapCoGroupsInPandas).  Key columns must have the same types on both sides."""

    def __init__(self, g1: GroupedData, g2: GroupedData):
        if len(g1.keys) != len(g2.keys):
            raise ValueError("cogroup needs the same number of grouping keys on both sides")
        self.g1, self.g2 = g1, g2

    def applyInPandas(self, func, schema) -> DataFrame:
        import pandas as pd
        from .extras import _frame_from_pandas
        sides = []
        for g in (self.g1, self.g2):
            names = [k.name for k in g.keys]
            local = g.df.repartition(*names).toPandas_local()
            groups = OrderedDict((_group_key(k), p) for k, p in local.groupby(names, sort=False, dropna=False)) \
                if len(local) else OrderedDict()
            sides.append((local.iloc[0:0], groups))
        (e1, g1), (e2, g2) = sides
        keys = list(g1) + [k for k in g2 if k not in g1]
        with_key = _takes_key(func, 3)
        parts = []
        for k in keys:
            a, b = g1.get(k, e1), g2.get(k, e2)
            parts.append(func(k, a, b) if with_key else func(a, b))
        return _frame_from_pandas(self.g1.df, pd.concat(parts, ignore_index=True) if parts else pd.DataFrame(),
                                  schema)


def _nullable_column(vals) -> C.Column:
    """Host column from python values with None = null: numbers stay numeric (long when
    all are integral, else double) with a validity mask; anything else goes through
    ``from_numpy``."""
    present = [v for v in vals if v is not None]
    if present and all(isinstance(v, (bool, int, float, np.number)) and not isinstance(v, (bool, np.bool_))
                       for v in present):
        integral = all(isinstance(v, (int, np.integer)) for v in present)
        dt = np.int64 if integral else np.float64
        data = np.array([0 if v is None else v for v in vals], dtype=dt)
        valid = np.array([v is not None for v in vals])
        return C.NumericColumn(torch.from_numpy(data), None if valid.all() else torch.from_numpy(valid),
                               T.LongType() if integral else T.DoubleType())
    return C.from_numpy(np.array(vals, dtype=object), "cpu")


class PivotedData(GroupedData):
    """``groupBy(keys).pivot(col[, values]).agg(...)``: one output column per (pivot value,
    aggregate).  One device aggregation over keys + pivot column, reshaped on the host
    (the aggregated table is small).  Pivot values default to the sorted distinct values."""

    def __init__(self, df, keys, pivot, values):
        super().__init__(df, keys)
        self.pivot_expr, self.values = pivot, values

    def agg(self, *aggs) -> DataFrame:
        from .groupby import aggregate
        if len(aggs) == 1 and isinstance(aggs[0], dict):
            aggs = tuple(getattr(E, fn if fn != "mean" else "avg")(c).alias(f"{fn}({c})") for c, fn in aggs[0].items())
        local = self.df.session.local_view()
        # the pivot key gets its own name: pivoting on a grouping column must not merge the two
        keyed = DataFrame(local, aggregate(self.df, self.keys + [self.pivot_expr.alias("__pivot__")],
                                           list(aggs))).collect()
        groups = DataFrame(local, aggregate(self.df, self.keys, [E.count().alias("__n")])).collect()
        nk = len(self.keys)
        values = self.values
        if values is None:
            seen = {_hashable(r[nk]): r[nk] for r in keyed}
            values = sorted(seen.values(), key=lambda v: (v is None, v if v is not None else 0))
        table = {(tuple(_hashable(x) for x in r[:nk]), _hashable(r[nk])): r[nk + 1:] for r in keyed}
        out = OrderedDict()
        for i, k in enumerate(self.keys):
            out[k.name] = _nullable_column([g[i] for g in groups])     # numeric keys stay numeric
        for v in values:
            for j, a in enumerate(aggs):
                name = str(v) if len(aggs) == 1 else f"{v}_{a.name}"
                col = []
                for g in groups:
                    hit = table.get((tuple(_hashable(x) for x in g[:nk]), _hashable(v)))
                    col.append(None if hit is None else hit[j])
                out[name] = _nullable_column(col)
        return self.df._from_full(out)
