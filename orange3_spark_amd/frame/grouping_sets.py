"""``DataFrame.rollup`` / ``DataFrame.cube`` (and SQL ``GROUP BY ROLLUP/CUBE/GROUPING SETS``).

Spark expands a grouping-sets aggregate into an ``Expand`` of every input row once per
grouping set (nulling the keys outside the set) followed by one hash aggregate keyed on
(keys, grouping id).  Here the input is never expanded: each grouping set is one
device-side partial aggregation over the HBM-resident shard (frame/groupby.py), whose
small per-group tables are merged across ranks, and the per-set results are stacked.
``k`` keys cost ``k+1`` (rollup) or ``2**k`` (cube) streaming passes over the key and
value columns instead of materialising ``2**k`` copies of the table.

``grouping(col)`` / ``grouping_id(*cols)`` aggregates are resolved per set (they are
constants of the set), with Spark's bit order: the first key is the most significant
bit of ``grouping_id``.
"""
from __future__ import annotations

import itertools
from collections import OrderedDict

import numpy as np
import torch

from . import column as C
from . import expr as E


def _null_column(template: C.Column, n: int) -> C.Column:
    if isinstance(template, C.NumericColumn):
        dev = template.data.device
        return C.NumericColumn(torch.zeros(n, dtype=template.data.dtype, device=dev),
                               torch.zeros(n, dtype=torch.bool, device=dev), template.dtype)
    if isinstance(template, C.HostColumn):
        return type(template)(np.full(n, None, dtype=object))
    raise TypeError(f"cannot null a {type(template).__name__} grouping key")


def _const_column(v: int, n: int, dev) -> C.Column:
    return C.NumericColumn(torch.full((n,), v, dtype=torch.int64, device=dev))


def rollup_sets(k: int) -> list[tuple[int, ...]]:
    return [tuple(range(i)) for i in range(k, -1, -1)]


def cube_sets(k: int) -> list[tuple[int, ...]]:
    out = []
    for r in range(k, -1, -1):
        out.extend(itertools.combinations(range(k), r))
    return out


class GroupingSets:
    """Result of ``df.rollup(...)`` / ``df.cube(...)``: same aggregate methods as
    :class:`GroupedData`."""

    def __init__(self, df, keys: list, sets: list[tuple[int, ...]]):
        self.df, self.keys, self.sets = df, keys, sets

    def agg(self, *aggs):
        from .groupby import aggregate
        if len(aggs) == 1 and isinstance(aggs[0], dict):
            aggs = tuple(getattr(E, fn if fn != "mean" else "avg")(c).alias(f"{fn}({c})")
                         for c, fn in aggs[0].items())
        key_names = [k.name for k in self.keys]
        real = [a for a in aggs if a.fn not in ("grouping", "grouping_id")]
        results = [aggregate(self.df, [self.keys[i] for i in s], real) for s in self.sets]
        templates = {}                  # a typed column per key, to build its null fill
        for s, res in zip(self.sets, results):
            for i in s:
                templates.setdefault(key_names[i], res[key_names[i]])
        for k, e in zip(key_names, self.keys):
            if k not in templates:      # key in no set: type it from the input column
                templates[k] = e.eval(self.df.limit(0))
        pieces = []
        for s, res in zip(self.sets, results):
            n = len(next(iter(res.values()))) if res else 0
            dev = self.df.device
            cols = OrderedDict()
            for i, k in enumerate(key_names):
                cols[k] = res[k] if i in s else _null_column(templates[k], n)
            for a in aggs:
                if a.fn == "grouping":
                    j = key_names.index(a.arg.name)
                    cols[a.name] = _const_column(0 if j in s else 1, n, dev)
                elif a.fn == "grouping_id":
                    names = list(getattr(a, "param", None) or key_names)
                    gid = 0
                    for nm in names:
                        gid = (gid << 1) | (0 if key_names.index(nm) in s else 1)
                    cols[a.name] = _const_column(gid, n, dev)
                else:
                    cols[a.name] = res[a.name]
            pieces.append(cols)
        out = OrderedDict((k, C.Column.concat([p[k] for p in pieces])) for k in pieces[0])
        return self.df._from_full(out)

    def count(self):
        return self.agg(E.count().alias("count"))

    def _simple(self, fn, cols):
        if not cols:
            names = {k.name for k in self.keys}
            cols = [k for k, c in self.df._cols.items() if isinstance(c, C.NumericColumn) and k not in names]
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
