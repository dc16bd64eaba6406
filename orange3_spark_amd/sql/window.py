"""Window functions (``pyspark.sql.Window`` / ``Column.over``).

Spark evaluates a window by shuffling rows on the PARTITION BY keys, sorting each
partition by the ORDER BY keys and scanning it.  Here (frame/shuffle.py machinery):

1. rows are hash-exchanged on the partition keys (``all_to_all_v``; everything goes to
   rank 0 without PARTITION BY, as Spark moves it to a single partition);
2. one stable local sort by (partition key hash, order codes) on the device;
3. every window function is a segmented scan / gather on device tensors: segment ids
   from key changes, positions from ``arange - segment start``, peer groups from order
   key changes; ranks / ntile / percent_rank / cume_dist are index arithmetic,
   lag / lead are shifted gathers masked at segment edges, aggregates use segment
   prefix sums (running / ROWS BETWEEN frames: differences of inclusive prefix sums;
   RANGE frames with ties: the value at the last peer; RANGE frames with value offsets:
   edges from a vectorised per-partition binary search) or segment reductions
   (unordered windows); frame min/max use a sparse table (log-step doubling, any frame).

Several window expressions in one ``select`` share the exchange + sort when they use
the same window spec.
"""
from __future__ import annotations

import itertools
import math
import weakref
from collections import OrderedDict

import numpy as np
import torch

from ..frame import column as C
from ..frame import expr as E
from ..frame import types as T

_IDS = itertools.count()
_REGISTRY: "weakref.WeakValueDictionary[str, WindowExpr]" = weakref.WeakValueDictionary()
_PREFIX = "__win:"

# aggregates evaluated per frame by the group-by finaliser (host): no prefix-sum form
_HOST_FRAME_AGGS = ("collect_set", "median", "mode", "product", "bool_and", "bool_or", "percentile",
                    "percentile_exact", "max_by", "min_by", "bit_and", "bit_or", "bit_xor",
                    "histogram_numeric")

unboundedPreceding = -(1 << 62)
unboundedFollowing = 1 << 62
currentRow = 0


HOST_FRAME_WARN_ROWS = 50_000_000


def _warn_frame_volume(lo_n, hi_n, fn):
    """Host-evaluated frame aggregates cost O(sum of frame sizes) for frames that differ row
    to row (sliding ROWS frames); warn when that volume is large."""
    vol = float(np.maximum(hi_n - lo_n + 1, 0).sum())
    if vol > HOST_FRAME_WARN_ROWS:
        import logging
        logging.getLogger(__name__).warning(
            "window %s over %.3g frame rows is evaluated on the host (O(rows x frame)); "
            "bound the frame or aggregate with groupBy", fn, vol)


class WindowSpec:
    def __init__(self, partition=(), order=(), frame=None):
        self._partition, self._order, self._frame = tuple(partition), tuple(order), frame

    @staticmethod
    def _cols(cols):
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        return tuple(E.col(c) if isinstance(c, str) else c for c in cols)

    def partitionBy(self, *cols):
        return WindowSpec(self._cols(cols), self._order, self._frame)

    def orderBy(self, *cols):
        return WindowSpec(self._partition, self._cols(cols), self._frame)

    def rowsBetween(self, start: int, end: int):
        return WindowSpec(self._partition, self._order, ("rows", int(start), int(end)))

    def rangeBetween(self, start, end):
        """RANGE frame: ``unboundedPreceding`` / ``currentRow`` (the row's peers) /
        ``unboundedFollowing``, or numeric value offsets -- a row is in the frame when its
        ORDER BY value lies within ``[v + start, v + end]`` (Spark ``RangeFrame``; needs
        exactly one numeric ORDER BY expression)."""
        def norm(x):
            x = float(x) if not isinstance(x, int) else x
            return int(x) if float(x).is_integer() else x
        return WindowSpec(self._partition, self._order, ("range", norm(start), norm(end)))

    def _key(self):
        return (tuple(e.name for e in self._partition),
                tuple((e.name, bool(getattr(e, "_desc", False)), getattr(e, "_nulls_first", None))
                      for e in self._order), self._frame)


class Window:
    unboundedPreceding = unboundedPreceding
    unboundedFollowing = unboundedFollowing
    currentRow = currentRow

    @staticmethod
    def partitionBy(*cols):
        return WindowSpec().partitionBy(*cols)

    @staticmethod
    def orderBy(*cols):
        return WindowSpec().orderBy(*cols)

    @staticmethod
    def rowsBetween(start, end):
        return WindowSpec().rowsBetween(start, end)

    @staticmethod
    def rangeBetween(start, end):
        return WindowSpec().rangeBetween(start, end)


class WindowFunction:
    """A function that is only meaningful over a window (row_number, lag, ...)."""

    def __init__(self, fn, args=(), name=None):
        self.fn, self.args = fn, tuple(args)
        self._name = name or f"{fn}()"

    @property
    def name(self):
        return self._name

    def over(self, window: WindowSpec) -> "WindowExpr":
        return WindowExpr(self, window)

    def alias(self, name):
        return WindowFunction(self.fn, self.args, name)


class WindowExpr(E.Expr):
    """``func.over(window)``: evaluates to a hidden column computed by :func:`apply`."""

    def __init__(self, func, window: WindowSpec, name=None):
        self.key = f"{_PREFIX}{next(_IDS)}"
        self.func, self.window = func, window
        super().__init__(self._lookup, name or f"{func.name} OVER (...)", (self.key,))
        _REGISTRY[self.key] = self

    def _lookup(self, df):
        if self.key not in df.columns:
            raise RuntimeError("window expressions are evaluated by select()/withColumn()")
        return df._col(self.key)

    def alias(self, name):
        out = E.Expr(self._fn, name, self.refs)
        out._window_src = self                      # keep the registry entry alive
        return out


def over(func, window):
    """``Agg.over`` / ``WindowFunction.over`` entry point."""
    return WindowExpr(func, window)


def window_refs(exprs) -> list:
    keys = []
    for e in exprs:
        for r in getattr(e, "refs", ()):
            if isinstance(r, str) and r.startswith(_PREFIX) and r not in keys:
                keys.append(r)
    return keys


# --------------------------------------------------------------------------- evaluation
def apply(df, keys: list):
    """Exchange + sort ``df`` once per distinct window spec and attach every window
    column named in ``keys``.  Returns the re-ordered frame with hidden columns."""
    from ..frame.shuffle import _order_code, exchange, local_sort_perm, row_keys
    from ..parallel.comm import LocalComm
    wins = [_REGISTRY[k] for k in keys]
    groups: OrderedDict = OrderedDict()
    for w in wins:
        groups.setdefault(w.window._key(), []).append(w)
    cur = df
    for _, ws in groups.items():
        spec = ws[0].window
        comm = cur.comm
        dev = cur.device
        pnames = []
        tmp = OrderedDict(cur._cols)
        for i, e in enumerate(spec._partition):
            tmp[f"__wp{i}"] = e.eval(cur)
            pnames.append(f"__wp{i}")
        staged = cur._new(tmp)
        if comm.world_size > 1:
            if pnames:
                dest = row_keys(staged, pnames)[:, 0] % comm.world_size
            else:
                dest = torch.zeros(len(staged), dtype=torch.int64, device=dev)
            staged = exchange(staged, dest)
        lc = LocalComm(dev)
        pk = row_keys(staged, pnames) if pnames else torch.zeros(len(staged), 2, dtype=torch.int64, device=dev)
        ocodes = []
        for e in spec._order:
            a = not getattr(e, "_desc", False)
            nf = getattr(e, "_nulls_first", None)
            ocodes.append(_order_code(lc, e.eval(staged), a, a if nf is None else nf).to(dev))
        perm = local_sort_perm([pk[:, 0], pk[:, 1]] + ocodes) if len(staged) else \
            torch.zeros(0, dtype=torch.int64, device=dev)
        staged = staged._take(perm)
        pk = pk[perm]
        ocodes = [c[perm] for c in ocodes]
        ctx = _Ctx(staged, pk, ocodes, spec)
        out = OrderedDict((k, v) for k, v in staged._cols.items() if not k.startswith("__wp"))
        for w in ws:
            out[w.key] = ctx.compute(w.func)
        cur = staged._new(out)
    return cur


class _Ctx:
    def __init__(self, df, pk, ocodes, spec):
        self.df, self.spec = df, spec
        n = len(df)
        dev = df.device
        self.n = n
        ar = torch.arange(n, device=dev)
        new_seg = torch.ones(n, dtype=torch.bool, device=dev)
        if n > 1:
            new_seg[1:] = (pk[1:] != pk[:-1]).any(1)
        self.seg = torch.cumsum(new_seg.to(torch.int64), 0) - 1
        nseg = int(self.seg[-1].item()) + 1 if n else 0
        self.seg_start = torch.zeros(nseg, dtype=torch.int64, device=dev)
        if n:
            self.seg_start.scatter_reduce_(0, self.seg, ar, "amin", include_self=False)
        self.seg_len = torch.bincount(self.seg, minlength=nseg) if n else torch.zeros(0, dtype=torch.int64, device=dev)
        self.pos = ar - self.seg_start[self.seg] if n else ar
        self.cnt = self.seg_len[self.seg] if n else ar
        new_peer = new_seg.clone()
        for c in ocodes:
            if n > 1:
                new_peer[1:] |= c[1:] != c[:-1]
        self.peer = torch.cumsum(new_peer.to(torch.int64), 0) - 1
        npeer = int(self.peer[-1].item()) + 1 if n else 0
        self.peer_first = torch.zeros(npeer, dtype=torch.int64, device=dev)
        self.peer_last = torch.zeros(npeer, dtype=torch.int64, device=dev)
        if n:
            self.peer_first.scatter_reduce_(0, self.peer, ar, "amin", include_self=False)
            self.peer_last.scatter_reduce_(0, self.peer, ar, "amax", include_self=False)
        self.new_peer = new_peer
        self.ordered = bool(ocodes)

    # -- helpers ------------------------------------------------------------------
    def _int(self, t):
        return C.NumericColumn(t.to(torch.int64), None, T.IntegerType())

    def _dbl(self, t, valid=None):
        return C.NumericColumn(t.to(torch.float64), valid, T.DoubleType())

    def compute(self, func):
        if isinstance(func, WindowFunction):
            return getattr(self, "_f_" + func.fn)(*func.args)
        if isinstance(func, E.Agg):
            return self._agg(func)
        raise TypeError(f"{func!r} cannot be used over a window")

    # -- ranking ----------------------------------------------------------------------
    def _f_row_number(self):
        return self._int(self.pos + 1)

    def _f_rank(self):
        return self._int(self.peer_first[self.peer] - self.seg_start[self.seg] + 1)

    def _f_dense_rank(self):
        c = torch.cumsum(self.new_peer.to(torch.int64), 0)
        base = c[self.seg_start][self.seg] if self.n else c
        return self._int(c - base + 1)

    def _f_percent_rank(self):
        r = (self.peer_first[self.peer] - self.seg_start[self.seg]).to(torch.float64)
        d = (self.cnt - 1).to(torch.float64)
        return self._dbl(torch.where(d > 0, r / d.clamp(min=1), torch.zeros_like(r)))

    def _f_cume_dist(self):
        upto = (self.peer_last[self.peer] - self.seg_start[self.seg] + 1).to(torch.float64)
        return self._dbl(upto / self.cnt.to(torch.float64))

    def _f_ntile(self, n):
        n = int(n)
        # Spark: the first (cnt % n) buckets get one extra row
        cnt, pos = self.cnt, self.pos
        q, r = cnt // n, cnt % n
        big = (q + 1) * r
        tile = torch.where(pos < big, pos // (q + 1).clamp(min=1), r + (pos - big) // q.clamp(min=1))
        return self._int(tile + 1)

    # -- offsets ----------------------------------------------------------------------
    def _shift(self, col, offset, default):
        c = col.eval(self.df) if isinstance(col, E.Expr) else self.df._col(col)
        src = self.pos - offset
        ok = (src >= 0) & (src < self.cnt)
        idx = torch.where(ok, torch.arange(self.n, device=self.df.device) - offset, torch.zeros_like(self.pos))
        if isinstance(c, C.NumericColumn):
            dv = c.data.device
            okd, idd = ok.to(dv), idx.to(dv)
            data = c.data[idd]
            if default is not None:
                data = torch.where(okd, data, torch.tensor(default, dtype=data.dtype, device=dv))
            v_src = c.valid[idd] if c.valid is not None else torch.ones_like(okd)
            valid = torch.where(okd, v_src, torch.full_like(okd, default is not None))
            return C.NumericColumn(data, None if bool(valid.all()) else valid, c.dtype)
        vals = c.values if isinstance(c, C.HostColumn) else np.asarray(c.to_pylist(), dtype=object)
        okn, idn = ok.cpu().numpy(), idx.cpu().numpy()
        out = np.empty(self.n, dtype=object)
        out[:] = [vals[j] if o else default for o, j in zip(okn, idn)]
        return C.StringColumn(out) if isinstance(c, C.StringColumn) else C.from_numpy(out, "cpu")

    def _f_lag(self, col, offset=1, default=None):
        return self._shift(col, int(offset), default)

    def _f_lead(self, col, offset=1, default=None):
        return self._shift(col, -int(offset), default)

    def _f_nth_value(self, col, nth, ignoreNulls=False):
        c = col.eval(self.df) if isinstance(col, E.Expr) else self.df._col(col)
        end = self._frame_bounds()[1]
        tgt = self.seg_start[self.seg] + int(nth) - 1
        ok = tgt <= end
        idx = torch.where(ok, tgt, torch.zeros_like(tgt))
        return _gather(c, idx, ok)

    # -- frames ---------------------------------------------------------------------
    def _frame_bounds(self):
        """Inclusive [lo, hi] row index of every row's frame (global sorted positions)."""
        st = self.seg_start[self.seg]
        en = st + self.cnt - 1
        ar = torch.arange(self.n, device=self.df.device)
        fr = self.spec._frame
        if fr is None:
            if not self.ordered:
                return st, en
            return st, self.peer_last[self.peer]               # RANGE UNBOUNDED PRECEDING .. CURRENT ROW
        kind, a, b = fr
        if kind == "rows":
            lo = st if a <= unboundedPreceding else torch.maximum(st, ar + a)
            hi = en if b >= unboundedFollowing else torch.minimum(en, ar + b)
            return lo, hi
        if (a <= unboundedPreceding or a == 0) and (b >= unboundedFollowing or b == 0):
            lo = st if a <= unboundedPreceding else self.peer_first[self.peer]
            hi = en if b >= unboundedFollowing else self.peer_last[self.peer]
            return lo, hi
        return self._range_value_bounds(a, b, st, en)

    def _range_value_bounds(self, a, b, st, en):
        """RANGE BETWEEN with value offsets (Spark ``RangeFrame``): row j is in row i's frame
        when s_j lies in [s_i + a, s_i + b], with s the ORDER BY value (negated for DESC, so
        PRECEDING always runs against the sort direction).  Rows are sorted by s inside each
        partition with the nulls contiguous at one end, so both edges come from one
        vectorised binary search per side over the partition's non-null rows.  A null
        current row's frame is its null peers (the bound v + offset is null)."""
        if len(self.spec._order) != 1:
            raise ValueError("a RANGE frame with value offsets needs exactly one ORDER BY expression")
        e = self.spec._order[0]
        c = e.eval(self.df)
        if not isinstance(c, C.NumericColumn):
            raise TypeError("a RANGE frame with value offsets needs a numeric ORDER BY expression")
        dev = st.device
        n = self.n
        v = c.data.to(torch.float64).to(dev)
        null = c.null_mask().to(dev) | torch.isnan(v)
        s = -v if getattr(e, "_desc", False) else v
        ar = torch.arange(n, device=dev)
        nseg = self.seg_len.numel()
        nn_first = torch.full((nseg,), n, dtype=torch.int64, device=dev)
        nn_last = torch.full((nseg,), -1, dtype=torch.int64, device=dev)
        if bool((~null).any()):
            nn_first.scatter_reduce_(0, self.seg[~null], ar[~null], "amin", include_self=True)
            nn_last.scatter_reduce_(0, self.seg[~null], ar[~null], "amax", include_self=True)
        f0, f1 = nn_first[self.seg], nn_last[self.seg] + 1
        steps = max(1, int(n).bit_length() + 1)

        def first_at_least(target, strict):
            # first j in [f0, f1) with s_j >= target (> target when strict); f1 if none
            L, R = f0.clone(), f1.clone()
            for _ in range(steps):
                act = L < R
                mid = (L + R) // 2
                sm = s[mid.clamp(0, max(n - 1, 0))]
                right = act & ((sm <= target) if strict else (sm < target))
                L = torch.where(right, mid + 1, L)
                R = torch.where(act & ~right, mid, R)
            return L

        if a <= unboundedPreceding:
            lo = st
        elif a == 0:
            lo = self.peer_first[self.peer]
        else:
            lo = torch.where(null, self.peer_first[self.peer], first_at_least(s + a, False))
        if b >= unboundedFollowing:
            hi = en
        elif b == 0:
            hi = self.peer_last[self.peer]
        else:
            hi = torch.where(null, self.peer_last[self.peer], first_at_least(s + b, True) - 1)
        return lo, hi

    def _agg(self, a: E.Agg):
        lo, hi = self._frame_bounds()
        empty = hi < lo
        if a.fn == "count" and a.arg is None:
            return self._int(torch.where(empty, torch.zeros_like(lo), hi - lo + 1))
        c = a.arg.eval(self.df)
        if a.fn in ("first", "last"):
            idx = torch.where(empty, torch.zeros_like(lo), lo if a.fn == "first" else hi)
            return _gather(c, idx, ~empty)
        if a.fn == "collect_list":
            vals = c.to_pylist()
            lo_n, hi_n = lo.cpu().numpy(), hi.cpu().numpy()
            _warn_frame_volume(lo_n, hi_n, a.fn)
            memo: dict = {}
            arr = np.empty(self.n, dtype=object)
            out = []
            for x, y in zip(lo_n, hi_n):
                k = (int(x), int(y))
                if k not in memo:
                    memo[k] = [v for v in vals[x:y + 1] if v is not None]
                out.append(list(memo[k]))
            arr[:] = out
            return C.ArrayColumn(arr)
        if a.fn in _HOST_FRAME_AGGS or (a.distinct and a.fn in ("count", "sum", "avg")):
            # order statistics / sets / products: the group-by finaliser on every row's frame
            from ..frame.groupby import _host_final, _result_column
            vals = list(c.values) if isinstance(c, C.HostColumn) else c.to_pylist()
            lo_n, hi_n = lo.cpu().numpy(), hi.cpu().numpy()
            _warn_frame_volume(lo_n, hi_n, a.fn)
            memo: dict = {}                 # rows sharing a frame (peer groups, whole partitions) share one result

            def one(x, y):
                k = (int(x), int(y))
                r = memo.get(k, memo)
                if r is memo:
                    r = memo[k] = _host_final(a, list(enumerate(vals[x:y + 1])) if y >= x else [])
                return r
            return _result_column(a, [one(x, y) for x, y in zip(lo_n, hi_n)])
        if not isinstance(c, C.NumericColumn):
            raise TypeError(f"{a.fn} over a window needs a numeric column")
        d = c.data.to(torch.float64).to(lo.device)
        ok = ~c.null_mask().to(lo.device) & ~torch.isnan(d)
        dz = torch.where(ok, d, torch.zeros_like(d))
        okf = ok.to(torch.float64)

        def wsum(v):
            p = torch.cat([torch.zeros(1, dtype=torch.float64, device=v.device), torch.cumsum(v, 0)])
            return torch.where(empty, torch.zeros_like(v), p[hi + 1] - p[lo])
        cnt = wsum(okf)
        has = cnt > 0
        if a.fn == "count":
            return self._int(cnt.round().to(torch.int64))
        if a.fn == "sum":
            return self._dbl(wsum(dz), None if bool(has.all()) else has)
        if a.fn == "avg":
            return self._dbl(wsum(dz) / cnt.clamp(min=1), None if bool(has.all()) else has)
        if a.fn in ("stddev", "variance"):
            s1, s2 = wsum(dz), wsum(dz * dz)
            var = (s2 - s1 * s1 / cnt.clamp(min=1)) / (cnt - 1).clamp(min=1)
            var = var.clamp(min=0)
            good = cnt > 1
            return self._dbl(var.sqrt() if a.fn == "stddev" else var, None if bool(good.all()) else good)
        if a.fn in ("corr", "covar_pop", "covar_samp"):
            # co-moments over the frame rows where both columns are valid (groupby._final)
            cy = a.arg2.eval(self.df)
            if not isinstance(cy, C.NumericColumn):
                raise TypeError(f"{a.fn} over a window needs numeric columns")
            e = cy.data.to(torch.float64).to(lo.device)
            both = ok & ~cy.null_mask().to(lo.device) & ~torch.isnan(e)
            x, yv = torch.where(both, d, torch.zeros_like(d)), torch.where(both, e, torch.zeros_like(e))
            nb = wsum(both.to(torch.float64))
            n_ = nb.clamp(min=1)
            sx, sy = wsum(x), wsum(yv)
            cxy = wsum(x * yv) - sx * sy / n_
            if a.fn == "covar_pop":
                good = nb > 0
                r = cxy / n_
            elif a.fn == "covar_samp":
                good = nb > 1
                r = cxy / (nb - 1).clamp(min=1)
            else:
                cxx, cyy = wsum(x * x) - sx * sx / n_, wsum(yv * yv) - sy * sy / n_
                good = (nb > 0) & (cxx > 0) & (cyy > 0)
                r = cxy / torch.where(good, (cxx * cyy).sqrt(), torch.ones_like(cxx))
            return self._dbl(torch.where(good, r, torch.zeros_like(r)), None if bool(good.all()) else good)
        if a.fn in ("stddev_pop", "var_pop", "skewness", "kurtosis"):
            # population moments from frame power sums (the group-by formulas, groupby._final)
            n_ = cnt.clamp(min=1)
            s1, s2 = wsum(dz), wsum(dz * dz)
            mu = s1 / n_
            m2 = (s2 / n_ - mu * mu).clamp(min=0)
            if a.fn in ("stddev_pop", "var_pop"):
                return self._dbl(m2.sqrt() if a.fn == "stddev_pop" else m2, None if bool(has.all()) else has)
            s3 = wsum(dz * dz * dz)
            good = has & (m2 > 0)
            m2s = torch.where(good, m2, torch.ones_like(m2))
            if a.fn == "skewness":
                m3 = s3 / n_ - 3 * mu * s2 / n_ + 2 * mu ** 3
                r = m3 / m2s ** 1.5
            else:
                m4 = wsum(dz ** 4) / n_ - 4 * mu * s3 / n_ + 6 * mu * mu * s2 / n_ - 3 * mu ** 4
                r = m4 / (m2s * m2s) - 3.0
            return self._dbl(torch.where(good, r, torch.zeros_like(r)), None if bool(good.all()) else good)
        if a.fn in ("min", "max"):
            return self._minmax(d, ok, lo, hi, a.fn == "max")
        raise NotImplementedError(f"{a.fn} over a window")

    def _minmax(self, d, ok, lo, hi, is_max):
        """Frame min/max by a sparse table (log-step doubling) -> O(n log n), any frame."""
        fill = -math.inf if is_max else math.inf
        v = torch.where(ok, d, torch.full_like(d, fill))
        op = torch.maximum if is_max else torch.minimum
        levels = [v]
        k = 1
        while (1 << k) <= max(self.n, 1):
            prev = levels[-1]
            step = 1 << (k - 1)
            nxt = prev.clone()
            nxt[: self.n - step] = op(prev[: self.n - step], prev[step:])
            levels.append(nxt)
            k += 1
        length = (hi - lo + 1).clamp(min=1)
        lg = torch.floor(torch.log2(length.to(torch.float64))).to(torch.int64)
        table = torch.stack(levels)                    # [L, n]
        top = max(self.n - 1, 0)                       # empty frames may sit past the end
        a_ = table[lg, lo.clamp(0, top)]
        b_ = table[lg, (hi - (1 << lg) + 1).clamp(0, top)]
        r = op(a_, b_)
        good = torch.isfinite(r) & (hi >= lo)
        return self._dbl(torch.where(good, r, torch.zeros_like(r)), None if bool(good.all()) else good)


def _gather(c: C.Column, idx: torch.Tensor, ok: torch.Tensor) -> C.Column:
    if isinstance(c, C.NumericColumn):
        data = c.data[idx.to(c.data.device)]
        valid = ok.to(data.device)
        if c.valid is not None:
            valid = valid & c.valid[idx.to(c.data.device)]
        return C.NumericColumn(data, None if bool(valid.all()) else valid, c.dtype)
    vals = c.values if isinstance(c, C.HostColumn) else np.asarray(c.to_pylist(), dtype=object)
    out = np.empty(len(idx), dtype=object)
    out[:] = [vals[j] if o else None for j, o in zip(idx.cpu().numpy(), ok.cpu().numpy())]
    return C.StringColumn(out) if isinstance(c, C.StringColumn) else C.from_numpy(out, "cpu")


# --------------------------------------------------------------------------- constructors
def row_number():
    return WindowFunction("row_number", (), "row_number()")


def rank():
    return WindowFunction("rank", (), "rank()")


def dense_rank():
    return WindowFunction("dense_rank", (), "dense_rank()")


def percent_rank():
    return WindowFunction("percent_rank", (), "percent_rank()")


def cume_dist():
    return WindowFunction("cume_dist", (), "cume_dist()")


def ntile(n: int):
    return WindowFunction("ntile", (int(n),), f"ntile({n})")


def lag(col, offset: int = 1, default=None):
    e = E.col(col) if isinstance(col, str) else col
    return WindowFunction("lag", (e, offset, default), f"lag({e.name}, {offset}, {default})")


def lead(col, offset: int = 1, default=None):
    e = E.col(col) if isinstance(col, str) else col
    return WindowFunction("lead", (e, offset, default), f"lead({e.name}, {offset}, {default})")


def nth_value(col, offset: int, ignoreNulls: bool = False):
    e = E.col(col) if isinstance(col, str) else col
    return WindowFunction("nth_value", (e, offset, ignoreNulls), f"nth_value({e.name}, {offset})")
