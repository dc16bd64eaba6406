"""DataFrame joins (equi / cross).  The right side is gathered to every rank (broadcast
hash join, Spark's strategy for small dimension tables); left rows stay on their rank."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from . import column as C
from .dataframe import DataFrame, _hashable


def join(left: DataFrame, right: DataFrame, on, how: str = "inner") -> DataFrame:
    how = {"left_outer": "left", "leftouter": "left", "right_outer": "right", "rightouter": "right",
           "full": "outer", "fullouter": "outer", "full_outer": "outer", "semi": "left_semi",
           "leftsemi": "left_semi", "anti": "left_anti", "leftanti": "left_anti"}.get(how, how)
    rfull = DataFrame(right.session.local_view(), right._gathered())
    if on is None or how == "cross":
        nl, nr = len(left), len(rfull)
        li = torch.arange(nl).repeat_interleave(nr)
        ri = torch.arange(nr).repeat(nl)
        return _assemble(left, rfull, li, ri, [], None)
    if isinstance(on, str):
        on = [on]
    if how == "right":
        # right join == left join with sides swapped, computed on the gathered left
        lfull = DataFrame(left.session.local_view(), left._gathered())
        out = _hash_join(rfull, lfull, on, "left", swap=True)
        return left._from_full(out._cols)
    if how == "outer":
        lfull = DataFrame(left.session.local_view(), left._gathered())
        out = _hash_join(lfull, rfull, on, "outer")
        return left._from_full(out._cols)
    return _hash_join(left, rfull, on, how)


def _key_codes(left: DataFrame, right: DataFrame, on):
    """Exact per-row key codes (int64 on the left's device) for both sides, or None when
    a key column is not numeric / string: equal keys <-> equal codes; rows with a null
    key get -1 (left) / -2 (right) so they never match; NaN equals NaN (Spark)."""
    dev = left.device
    per_col = []
    for k in on:
        a, b = left._col(k), right._col(k)
        if isinstance(a, C.NumericColumn) and isinstance(b, C.NumericColumn):
            fl = a.data.is_floating_point() or b.data.is_floating_point()
            dt = torch.float64 if fl else torch.int64
            va, vb = a.data.to(dev, dt), b.data.to(dev, dt)
            both = torch.cat([va, vb])
            nan = torch.isnan(both) if fl else torch.zeros_like(both, dtype=torch.bool)
            if fl:
                both = torch.where(nan, torch.zeros_like(both), both)
            _, codes = torch.unique(both, return_inverse=True)
            codes = torch.where(nan, torch.full_like(codes, int(codes.max().item()) + 1 if codes.numel() else 0),
                                codes)
            null = torch.cat([a.null_mask().to(dev), b.null_mask().to(dev)]) if fl or a.valid is not None \
                or b.valid is not None else torch.zeros_like(codes, dtype=torch.bool)
            if fl:                                   # null_mask() counts NaN as null: NaN keys stay matchable
                null = null & ~nan
            per_col.append((codes, null))
        elif isinstance(a, C.HostColumn) and isinstance(b, C.HostColumn) and not isinstance(a, C.ArrayColumn) \
                and not isinstance(b, C.ArrayColumn):
            import pandas as pd
            vals = np.concatenate([np.asarray(a.values, dtype=object), np.asarray(b.values, dtype=object)])
            codes, _ = pd.factorize(pd.Series(vals, dtype=object), use_na_sentinel=True)
            codes = torch.from_numpy(codes.astype(np.int64)).to(dev)
            per_col.append((codes, codes < 0))
        else:
            return None
    nl = len(left)
    if len(per_col) == 1:
        code, null = per_col[0]
    else:
        stacked = torch.stack([c for c, _ in per_col], 1)
        _, code = torch.unique(stacked, dim=0, return_inverse=True)
        null = torch.stack([m for _, m in per_col], 1).any(1)
    code = code.to(torch.int64)
    lc = torch.where(null[:nl], torch.full_like(code[:nl], -1), code[:nl])
    rc = torch.where(null[nl:], torch.full_like(code[nl:], -2), code[nl:])
    return lc, rc


def _vector_join(lc: torch.Tensor, rc: torch.Tensor, how: str):
    """(li, ri) pairs of an equi-join from key codes: left rows in order, each left row's
    matches in right-row order (stable sort + searchsorted; no per-row Python)."""
    dev = lc.device
    nl, nr = lc.numel(), rc.numel()
    rs, rperm = torch.sort(rc, stable=True)
    lo = torch.searchsorted(rs, lc, right=False)
    hi = torch.searchsorted(rs, lc, right=True)
    cnt = hi - lo
    if how == "left_semi":
        return torch.nonzero(cnt > 0).squeeze(1), None
    if how == "left_anti":
        return torch.nonzero(cnt == 0).squeeze(1), None
    take = cnt if how == "inner" else torch.clamp_min(cnt, 1)
    li = torch.repeat_interleave(torch.arange(nl, device=dev), take)
    start = torch.cumsum(take, 0) - take
    off = torch.arange(li.numel(), device=dev) - start[li]
    has = cnt[li] > 0
    ri = torch.where(has, rperm[(lo[li] + off).clamp_max(max(nr - 1, 0))] if nr else torch.zeros_like(li),
                     torch.full_like(li, -1))
    if how == "outer":
        ls, _ = torch.sort(lc)
        rl = torch.searchsorted(ls, rc, right=False)
        rh = torch.searchsorted(ls, rc, right=True)
        unmatched = torch.nonzero(rh == rl).squeeze(1)
        li = torch.cat([li, torch.full_like(unmatched, -1)])
        ri = torch.cat([ri, unmatched])
    return li, ri


def _keys(df: DataFrame, on):
    lists = [df.column_data(k).to_pylist() for k in on]
    return [tuple(_hashable(v) for v in row) for row in zip(*lists)] if lists else []


def _hash_join(left: DataFrame, right: DataFrame, on, how, swap=False) -> DataFrame:
    codes = _key_codes(left, right, on)
    if codes is not None:
        li, ri = _vector_join(codes[0], codes[1], how)
        li = li.cpu() if li.is_cuda else li
        if how in ("left_semi", "left_anti"):
            return left._take(li)
        out = _assemble(left, right, li, ri.cpu(), on, how)
        return _restore_order(out, left, right, on) if swap else out
    rk = _keys(right, on)
    table = {}
    for j, k in enumerate(rk):
        if any(v is None for v in k):
            continue
        table.setdefault(k, []).append(j)
    lk = _keys(left, on)
    li, ri = [], []
    matched_r = np.zeros(len(rk), dtype=bool)
    for i, k in enumerate(lk):
        hits = table.get(k)
        if how == "left_semi":
            if hits:
                li.append(i)
            continue
        if how == "left_anti":
            if not hits:
                li.append(i)
            continue
        if hits:
            for j in hits:
                li.append(i)
                ri.append(j)
                matched_r[j] = True
        elif how in ("left", "outer"):
            li.append(i)
            ri.append(-1)
    if how in ("left_semi", "left_anti"):
        return left._take(torch.tensor(li, dtype=torch.int64))
    if how == "outer":
        for j in np.nonzero(~matched_r)[0]:
            li.append(-1)
            ri.append(int(j))
    out = _assemble(left, right, torch.tensor(li, dtype=torch.int64), torch.tensor(ri, dtype=torch.int64), on, how)
    return _restore_order(out, left, right, on) if swap else out


def _restore_order(out, left, right, on):
    """right join computed as a swapped left join: restore the column order
    (join keys, then the original left's columns, then the original right's)."""
    cols = OrderedDict()
    for k in on:
        cols[k] = out._cols[k]
    for k in right.columns:
        if k not in on:
            cols[k] = out._cols[k]
    for k in left.columns:
        if k not in on and k in out._cols:
            cols[k] = out._cols[k]
    return DataFrame(out.session, cols, len(out))


def _take_nullable(col: C.Column, idx: torch.Tensor) -> C.Column:
    miss = idx < 0
    safe = torch.where(miss, torch.zeros_like(idx), idx)
    if len(col) == 0:
        safe = torch.zeros(0, dtype=torch.int64)
    if isinstance(col, C.NumericColumn):
        if len(col) == 0:
            return C.NumericColumn(torch.zeros(idx.numel(), dtype=col.data.dtype, device=col.data.device),
                                   torch.zeros(idx.numel(), dtype=torch.bool, device=col.data.device), col.dtype)
        t = col.take(safe)
        if bool(miss.any()):
            v = t.valid if t.valid is not None else torch.ones_like(t.data, dtype=torch.bool)
            t = C.NumericColumn(t.data, v & ~miss.to(v.device), col.dtype)
        return t
    if isinstance(col, C.HostColumn):
        vals = col.values[safe.numpy()] if len(col) else np.empty(idx.numel(), dtype=object)
        vals = vals.copy()
        vals[miss.numpy()] = None
        return type(col)(vals) if not isinstance(col, C.ArrayColumn) else C.ArrayColumn(vals)
    return col.take(safe)


def _assemble(left, right, li, ri, on, how) -> DataFrame:
    cols = OrderedDict()
    for k, c in left._cols.items():
        if on and how == "outer" and k in on:
            lcol = _take_nullable(c, li)
            rcol = _take_nullable(right._col(k), ri)
            lv, rv = lcol.to_pylist(), rcol.to_pylist()
            merged = [a if a is not None else b for a, b in zip(lv, rv)]
            cols[k] = C.from_numpy(np.array(merged, dtype=object) if isinstance(c, C.HostColumn)
                                   else np.array(merged), left.device)
            continue
        cols[k] = _take_nullable(c, li) if how in ("left", "outer") else c.take(
            li.to(c.data.device) if isinstance(c, (C.NumericColumn, C.VectorColumn)) else li)
    for k, c in right._cols.items():
        if on and k in on:
            continue
        name = k if k not in cols else k + "_r"
        col = _take_nullable(c, ri)
        if isinstance(col, C.NumericColumn):
            col = C.NumericColumn(col.data.to(left.device), None if col.valid is None else col.valid.to(left.device),
                                  col.dtype)
        elif isinstance(col, C.VectorColumn):
            col = C.VectorColumn(col.data.to(left.device), col.size)
        cols[name] = col
    return DataFrame(left.session, cols, int(li.numel()))
