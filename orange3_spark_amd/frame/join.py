"""DataFrame joins (equi / cross / arbitrary condition).  The right side is gathered to every
rank (broadcast hash join, Spark's strategy for small dimension tables); left rows stay on
their rank.

Condition joins (``a.join(b, (a.id == b.uid) & (a.t < b.t), how)``) take the equality
conjuncts between the two sides as hash keys (vectorised sort + searchsorted) and evaluate
the rest of the condition on the candidate pairs; with no equality conjunct the candidates
are the cross product, walked in bounded blocks of left rows (Spark's nested-loop join).

Intentional difference from Spark: a right-side column whose name clashes with a left-side
column is kept under ``<name>_r`` (Spark keeps both under the same name and requires
qualified access).  Positional results are identical; ``other[c]`` / ``b.c`` references and
qualified names (``col("b.t")``) still resolve to the renamed column through the join's
provenance map, so only code that looks the duplicate up by its bare name sees the suffix."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from . import column as C
from . import expr as E
from .dataframe import DataFrame, _hashable


def join(left: DataFrame, right: DataFrame, on, how: str = "inner") -> DataFrame:
    how = {"left_outer": "left", "leftouter": "left", "right_outer": "right", "rightouter": "right",
           "full": "outer", "fullouter": "outer", "full_outer": "outer", "semi": "left_semi",
           "leftsemi": "left_semi", "anti": "left_anti", "leftanti": "left_anti"}.get(how, how)
    if isinstance(on, (list, tuple)) and on and all(isinstance(o, E.Expr) for o in on):
        cond = on[0]
        for o in on[1:]:
            cond = cond & o
        on = cond
    if isinstance(on, E.Expr):
        return condition_join(left, right, on, "inner" if how == "cross" else how)
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


# --------------------------------------------------------------------------- condition joins
_PAIR_BLOCK = 1 << 22          # candidate pairs evaluated per block (bounds the temporaries)


class _Sides:
    """Which side of a condition join a column reference names.  Identity first (``a.id``
    is the very column object ``a`` holds), then the relation alias of a qualified name
    (``col("a.id")``, SQL ``a.id``), then a name present on exactly one side; a name on
    both sides with nothing else to go by is ambiguous, as in Spark."""

    def __init__(self, left: DataFrame, right: DataFrame, ldata: DataFrame, rdata: DataFrame):
        self.orig = (left, right)
        self.data = (ldata, rdata)

    def _has(self, s: int, name: str) -> bool:
        try:
            self.orig[s]._col(name)
            return True
        except KeyError:
            return False

    def _key(self, s: int, name: str) -> str:
        """The column's actual key on side s (case / "alias." prefix resolved)."""
        f = self.orig[s]
        obj = f._col(name)
        if f._cols.get(name) is obj:
            return name
        return next(k for k, v in f._cols.items() if v is obj)

    def _key_of(self, s: int, src) -> str | None:
        f = self.orig[s]
        for k, v in f._cols.items():
            if v is src:
                return k
        return None

    def resolve(self, name: str, src=None, qual: str | None = None, frame=None) -> tuple[int, str]:
        if frame is not None:
            # the frame the reference was taken from (Spark's dataset id) decides the side,
            # also when both sides share the column object (df.join(df.withColumn(..)))
            for s in (0, 1):
                if self.orig[s] is frame:
                    k = self._key_of(s, src) if src is not None else None
                    if k is not None:
                        return s, k
                    if self._has(s, name):
                        return s, self._key(s, name)
        if src is not None:
            for s in (0, 1):
                f = self.orig[s]
                if f._cols.get(name) is src:
                    return s, name
                for k, v in f._cols.items():
                    if v is src:
                        return s, k
        if qual is None and "." in name and not any(self._has(s, name) for s in (0, 1)):
            qual, _, name = name.rpartition(".")
        if qual:
            q = qual.split(".")[-1]
            for s in (0, 1):
                f = self.orig[s]
                if q in f.__dict__.get("_aliases", ()):
                    out = f.__dict__.get("_qual_map", {}).get((q, name))
                    if out is not None:
                        return s, out
                    if self._has(s, name):
                        return s, self._key(s, name)
        hits = [s for s in (0, 1) if self._has(s, name)]
        if len(hits) == 1:
            return hits[0], self._key(hits[0], name)
        if not hits:
            raise KeyError(f"cannot resolve column '{name}' on either side of the join")
        raise ValueError(f"Reference '{name}' is ambiguous: both join sides have it "
                         "(use df['col'] of one side or an alias)")

    def side_of(self, e) -> tuple[int, str] | None:
        """(side, column) of a bare column reference, else None."""
        name = getattr(e, "_colname", None)
        if name is None:
            return None
        ref = getattr(e, "_src", None)
        fref = getattr(e, "_frame", None)
        return self.resolve(name, None if ref is None else ref(), getattr(e, "_qual", None),
                            None if fref is None else fref())

    def split_shared(self, e1, e2) -> tuple[str, str] | None:
        """``x.id == y.id`` whose operands both resolved to one side because the two frames
        share the column object: as Spark does for a trivially-true self-join equality,
        take the left operand from the left side and the right operand from the right
        side (None when the objects are not present on both sides)."""
        r1, r2 = getattr(e1, "_src", None), getattr(e2, "_src", None)
        if r1 is None or r2 is None:
            return None
        k1, k2 = self._key_of(0, r1()), self._key_of(1, r2())
        if k1 is not None and k2 is not None:
            return k1, k2
        k1, k2 = self._key_of(0, r2()), self._key_of(1, r1())
        if k1 is not None and k2 is not None:
            return k1, k2
        return None


class _PairFrame(DataFrame):
    """A condition evaluated over candidate pairs (li[k], ri[k]): each referenced column is
    taken from its side for exactly those pairs, once."""

    def __init__(self, sides: _Sides, li: torch.Tensor, ri: torch.Tensor):
        DataFrame.__init__(self, sides.data[0].session, OrderedDict(), int(li.numel()))
        self._sides, self._li, self._ri, self._taken = sides, li, ri, {}

    def _take_side(self, side: int, name: str) -> C.Column:
        key = (side, name)
        if key not in self._taken:
            self._taken[key] = self._sides.data[side]._col(name).take(self._li if side == 0 else self._ri)
        return self._taken[key]

    def _col(self, name):
        return self._take_side(*self._sides.resolve(name))

    def _col_bound(self, name, src, frame=None):
        return self._take_side(*self._sides.resolve(name, src, None, frame))

    def _col_qualified(self, qual, name):
        return self._take_side(*self._sides.resolve(name, None, qual))


def _conjuncts(e):
    t = getattr(e, "_tree", None)
    if t is not None and t[0] == "AND":
        return _conjuncts(t[1]) + _conjuncts(t[2])
    return [e]


def _split_condition(cond, sides: _Sides):
    """Equality conjuncts between a left and a right column -> hash keys; the rest stays a
    residual predicate (None when every conjunct was a key)."""
    keys, rest = [], []
    for c in _conjuncts(cond):
        t = getattr(c, "_tree", None)
        if t is not None and t[0] == "=":
            a, b = sides.side_of(t[1]), sides.side_of(t[2])
            if a is not None and b is not None and a[0] != b[0]:
                keys.append((a[1], b[1]) if a[0] == 0 else (b[1], a[1]))
                continue
            if a is not None and b is not None and a[1] == b[1]:
                # both operands on one side through a shared column object: never let the
                # always-true residual x == x turn the join into a cross product
                pair = sides.split_shared(t[1], t[2])
                if pair is None:
                    raise ValueError(f"join condition {c} compares column '{a[1]}' with itself; the sides "
                                     "share it -- alias the frames (df.alias('a')) and use qualified names")
                keys.append(pair)
                continue
        rest.append(c)
    residual = None
    for c in rest:
        residual = c if residual is None else residual & c
    return keys, residual


def _truth(c: C.Column, device) -> torch.Tensor:
    """SQL truth of a predicate column (null -> false), as a bool tensor on ``device``."""
    if isinstance(c, C.NumericColumn):
        m = c.data.bool()
        if c.valid is not None:
            m = m & c.valid
        return m.to(device)
    return torch.tensor([bool(v) if v is not None else False for v in c.to_pylist()], dtype=torch.bool,
                        device=device)


def _match_pairs(sides: _Sides, cond) -> tuple[torch.Tensor, torch.Tensor]:
    ldata, rdata = sides.data
    nl, nr = len(ldata), len(rdata)
    keys, residual = _split_condition(cond, sides)
    codes = None
    if keys:
        kl = DataFrame(ldata.session, OrderedDict((f"k{i}", ldata._col(a)) for i, (a, _) in enumerate(keys)), nl)
        kr = DataFrame(rdata.session, OrderedDict((f"k{i}", rdata._col(b)) for i, (_, b) in enumerate(keys)), nr)
        codes = _key_codes(kl, kr, [f"k{i}" for i in range(len(keys))])
    dev = ldata.device                  # pair indices and masks stay on the device until the end
    if codes is not None:
        li, ri = _vector_join(codes[0], codes[1], "inner")
        if residual is None or li.numel() == 0:
            return li.cpu(), ri.cpu()
        li, ri = li.to(dev), ri.to(dev)
        keep = [_truth(residual.eval(_PairFrame(sides, li[s:s + _PAIR_BLOCK], ri[s:s + _PAIR_BLOCK])), dev)
                for s in range(0, li.numel(), _PAIR_BLOCK)]
        m = torch.cat(keep)
        return li[m].cpu(), ri[m].cpu()
    # nested loop: blocks of left rows against every right row
    li_parts, ri_parts = [], []
    step = max(1, _PAIR_BLOCK // max(nr, 1))
    for s in range(0, nl if nr else 0, step):
        e = min(nl, s + step)
        bl = torch.arange(s, e, device=dev).repeat_interleave(nr)
        br = torch.arange(nr, device=dev).repeat(e - s)
        m = _truth(cond.eval(_PairFrame(sides, bl, br)), dev)
        li_parts.append(bl[m])
        ri_parts.append(br[m])
    if not li_parts:
        return torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64)
    return torch.cat(li_parts).cpu(), torch.cat(ri_parts).cpu()


def condition_join(left: DataFrame, right: DataFrame, cond, how: str = "inner") -> DataFrame:
    """``left.join(right, <Column condition>, how)``: every column of both sides is kept (a
    right-side name that clashes gets ``_r``); ``other[c]`` references made before the join
    still find their column in the result (``joined.select(b.id)``, ``joined.drop(b.id)``)."""
    if how not in ("inner", "left", "right", "outer", "left_semi", "left_anti"):
        raise ValueError(f"Unsupported join type '{how}'")
    full = how in ("right", "outer")
    ldata = DataFrame(left.session.local_view(), left._gathered()) if full else left
    rdata = DataFrame(right.session.local_view(), right._gathered())
    sides = _Sides(left, right, ldata, rdata)
    li, ri = _match_pairs(sides, cond)
    nl, nr = len(ldata), len(rdata)
    if how in ("left_semi", "left_anti"):
        hit = torch.zeros(nl, dtype=torch.bool)
        hit[li] = True
        return left._take(torch.nonzero(hit if how == "left_semi" else ~hit).squeeze(1))
    if how in ("left", "outer"):
        hit = torch.zeros(nl, dtype=torch.bool)
        hit[li] = True
        miss = torch.nonzero(~hit).squeeze(1)
        li = torch.cat([li, miss])
        ri = torch.cat([ri, torch.full_like(miss, -1)])
        order = torch.sort(li, stable=True).indices          # left row order, matches in right order
        li, ri = li[order], ri[order]
    if how in ("right", "outer"):
        hit = torch.zeros(nr, dtype=torch.bool)
        hit[ri[ri >= 0]] = True
        miss = torch.nonzero(~hit).squeeze(1)
        li = torch.cat([li, torch.full_like(miss, -1)])
        ri = torch.cat([ri, miss])
    import weakref
    cols, prov, qmap = OrderedDict(), [], {}
    for s, (orig, data, idx) in enumerate(((left, ldata, li), (right, rdata, ri))):
        nullable = bool((idx < 0).any())
        for k, c in data._cols.items():
            name = k
            while name in cols:
                name += "_r"
            t = _take_nullable(c, idx) if nullable else c.take(idx)
            if isinstance(t, C.NumericColumn):
                t = C.NumericColumn(t.data.to(left.device), None if t.valid is None else t.valid.to(left.device),
                                    t.dtype)
            elif isinstance(t, C.VectorColumn):
                t = C.VectorColumn(t.data.to(left.device), t.size)
            cols[name] = t
            src = orig._cols.get(k)
            if src is not None:
                prov.append((weakref.ref(src), name))
            for a in orig.__dict__.get("_aliases", ()):
                qmap[(a, k)] = name
    out = DataFrame(left.session, cols, int(li.numel()))
    if full:
        out = left._from_full(out._cols)
    out._prov = prov
    out._aliases = frozenset(left.__dict__.get("_aliases", ())) | frozenset(right.__dict__.get("_aliases", ()))
    out._qual_map = qmap
    return out
