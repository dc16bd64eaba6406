"""Distributed hash aggregation for ``groupBy().agg()`` / SQL GROUP BY.

Spark runs a partial aggregation per partition, shuffles the partials by key and merges
them.  Here, per rank:

1. the key columns are encoded to int64 codes on the device (numeric keys directly,
   strings through a host factorisation), and rows get a local group id from
   ``torch.unique(return_inverse=True)``;
2. partial aggregates are scatter-reductions on the device -- counts (``bincount``),
   sums / sums of squares (``index_add_``), min / max (``scatter_reduce``), first and
   last row (global row index min / max) -- so the per-row work never leaves the GPU;
3. the (small) per-group partial tables are all-gathered and merged by key on the host,
   and finals (avg, stddev, variance, first/last, distinct counts, collected lists)
   are computed from the merged partials.

Group order is the order of first appearance in the global row order (deterministic
and independent of the number of ranks).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch

from . import column as C
from . import expr as E

def _encode_key(c: C.Column, dev):
    """(codes int64 tensor [n], decode(list_of_codes) -> python values)."""
    if isinstance(c, C.NumericColumn):
        d = c.data
        null = c.null_mask() if c.valid is not None else None
        if d.is_floating_point():
            bits = d.to(torch.float64).view(torch.int64).clone()
            bits = torch.where(d == 0, torch.zeros_like(bits), bits)          # -0.0 == 0.0
            bits = torch.where(torch.isnan(d), torch.full_like(bits, 0x7FF8000000000000), bits)
        else:
            bits = d.to(torch.int64)
        if null is not None:
            bits = torch.where(null.to(bits.device), torch.full_like(bits, -(1 << 62) - 7), bits)

        def decode(codes, is_float=d.is_floating_point(), has_null=null is not None):
            t = torch.tensor(codes, dtype=torch.int64)
            vals = t.view(torch.float64).tolist() if is_float else t.tolist()
            if has_null:
                vals = [None if k == -(1 << 62) - 7 else v for k, v in zip(codes, vals)]
            return vals
        return bits.to(dev), decode, "num"
    values = c.values if isinstance(c, C.HostColumn) else np.asarray(c.to_pylist(), dtype=object)
    # host factorisation; codes are made global by the merge (keys travel as values)
    try:
        import pandas as pd
        codes, uniques = pd.factorize(pd.Series(values, dtype=object), use_na_sentinel=False)
        # decode to each key's first original object (pandas turns Row structs into plain tuples)
        _, first = np.unique(codes, return_index=True)
        uvals = [values[i] for i in first] if len(first) == len(uniques) else list(uniques)
        return (torch.from_numpy(codes.astype(np.int64)).to(dev),
                (lambda cs: [None if (isinstance(uvals[k], float) and math.isnan(uvals[k])) else uvals[k]
                             for k in cs]), "host")
    except TypeError:                     # unhashable values (lists, vectors): python path
        pass
    hashed = [_hashable(v) for v in values]
    uniq: dict = {}
    codes = np.empty(len(hashed), dtype=np.int64)
    for i, v in enumerate(hashed):
        j = uniq.get(v)
        if j is None:
            j = uniq[v] = len(uniq)
        codes[i] = j
    inv = list(uniq.keys())
    firsts = {}
    for i, v in enumerate(hashed):
        firsts.setdefault(v, values[i])
    return torch.from_numpy(codes).to(dev), (lambda cs: [firsts[inv[k]] for k in cs]), "host"


def _hashable(v):
    if isinstance(v, list):
        return tuple(v)
    if hasattr(v, "toArray"):
        return tuple(np.asarray(v.toArray()).tolist())
    if isinstance(v, float) and math.isnan(v):
        return "NaN"
    return v


def _values_valid(col: C.Column, dev):
    """(fp64 values, valid mask) of a numeric column (NaN counts as null, like Spark avg)."""
    d = col.data.to(dev, torch.float64)
    ok = ~col.null_mask().to(dev)
    return torch.where(ok, d, torch.zeros_like(d)), ok


def aggregate(df, keys: list, aggs: list):
    """Returns the FULL (replicated) result columns; the caller shards them."""
    comm = df.comm
    dev = df.device
    n = len(df)
    rows = df._global_rows()
    key_cols = [k.eval(df) for k in keys]
    if keys:
        enc = [_encode_key(c, dev) for c in key_cols]
        # dense per-column codes combined in mixed radix -> one 1-D unique (a row-wise
        # unique(dim=0) is a slow generic sort)
        dense, card, per_col_vals = [], [], []
        for codes, _, _ in enc:
            u, inv = torch.unique(codes, return_inverse=True)
            dense.append(inv)
            card.append(max(int(u.numel()), 1))
            per_col_vals.append(u)
        if math.prod(card) < (1 << 62):
            comb = torch.zeros(n, dtype=torch.int64, device=dev)
            for inv, cdim in zip(dense, card):
                comb = comb * cdim + inv
            ucomb, gid = torch.unique(comb, return_inverse=True)
            digits = []
            rest = ucomb.clone()
            for cdim in reversed(card):
                digits.append(rest % cdim)
                rest = rest // cdim
            digits.reverse()
            uk = torch.stack([per_col_vals[i][digits[i]] for i in range(len(keys))], 1) if ucomb.numel() else \
                torch.zeros((0, len(keys)), dtype=torch.int64, device=dev)
        else:
            K = torch.stack([e[0] for e in enc], 1)
            uk, gid = torch.unique(K, dim=0, return_inverse=True)
        G = uk.shape[0]
    else:
        enc = []
        gid = torch.zeros(n, dtype=torch.int64, device=dev)
        G = 1
    # Rows are grouped once by a stable sort of the group ids; every partial aggregate is
    # then a segmented reduction over the sorted order (torch.segment_reduce): no
    # contended atomics (a few thousand groups over millions of rows made scatter /
    # index_add atomics the bottleneck) and bitwise reproducible sums.
    if n and keys:
        perm = torch.argsort(gid, stable=True)
        counts = torch.bincount(gid, minlength=G)
    else:
        perm = None
        counts = torch.full((1,), n, dtype=torch.int64, device=dev) if G == 1 else torch.bincount(gid, minlength=G)
    ends = torch.cumsum(counts, 0)
    starts = ends - counts

    def red(x, op):
        """per-group reduction of a per-row fp64 tensor (op: sum / min / max)."""
        if n == 0:
            fill = {"sum": 0.0, "min": math.inf, "max": -math.inf}[op]
            return torch.full((G,), fill, dtype=torch.float64, device=dev)
        xs = x if perm is None else x[perm]
        return torch.segment_reduce(xs.to(torch.float64), op, lengths=counts, unsafe=True)

    rs = rows if perm is None else rows[perm]
    if n:
        first_row, last_row = rs[starts], rs[ends - 1]
    else:
        first_row = torch.full((G,), torch.iinfo(torch.int64).max, dtype=torch.int64, device=dev)
        last_row = torch.full((G,), -1, dtype=torch.int64, device=dev)
    parts: dict = {"__first": first_row, "__last": last_row, "__rows": counts.to(torch.float64)}
    host_parts: dict = {}
    host_tags: set = set()
    for j, a in enumerate(aggs):
        tag = f"a{j}"
        vals = a.arg.eval(df) if a.arg is not None else None
        if a.fn == "count" and not a.distinct:
            if vals is None:
                parts[tag + "n"] = parts["__rows"]
            else:
                ok = ~vals.null_mask().to(dev)
                parts[tag + "n"] = red(ok.double(), "sum")
            continue
        if a.distinct and isinstance(vals, C.NumericColumn) and a.fn in ("count", "sum", "avg"):
            # dedupe (group, value) on the device first; only distinct pairs go to the host
            ok = ~vals.null_mask().to(dev)
            v = vals.data.to(dev, torch.float64)[ok]
            uv, vinv = torch.unique(v, return_inverse=True)
            comb = gid[ok] * max(int(uv.numel()), 1) + vinv
            uc = torch.unique(comb)
            gg = (uc // max(int(uv.numel()), 1)).cpu().tolist()
            vv = uv[uc % max(int(uv.numel()), 1)].cpu().tolist()
            host_parts[tag] = [(g_, 0, x_) for g_, x_ in zip(gg, vv)]
            host_tags.add(tag)
            continue
        if a.fn in ("corr", "covar_pop", "covar_samp") and isinstance(vals, C.NumericColumn):
            # co-moments of the rows where both columns are valid: n, Sx, Sy, Sxx, Syy, Sxy
            x, okx = _values_valid(vals, dev)
            yv, oky = _values_valid(a.arg2.eval(df), dev)
            ok = okx & oky
            x, yv = torch.where(ok, x, torch.zeros_like(x)), torch.where(ok, yv, torch.zeros_like(yv))
            z = lambda v: red(v, "sum")  # noqa: E731
            parts[tag + "n"] = z(ok.double())
            for sfx, v in (("s", x), ("t", yv), ("q", x * x), ("r", yv * yv), ("p", x * yv)):
                parts[tag + sfx] = z(v)
            continue
        if a.distinct or a.fn in ("collect_list", "collect_set", "first", "last", "percentile", "median", "mode",
                                  "percentile_exact",
                                  "product", "bool_and", "bool_or", "max_by", "min_by", "bit_and", "bit_or",
                                  "bit_xor", "histogram_numeric") or \
                not isinstance(vals, C.NumericColumn):
            # host path: (group, value) pairs or per-group python reductions
            py = vals.to_pylist() if not isinstance(vals, C.HostColumn) else list(vals.values)
            g = gid.cpu().numpy()
            r = rows.cpu().numpy()
            host_parts[tag] = list(zip(g.tolist(), r.tolist(), py))
            host_tags.add(tag)
            continue
        x, ok = _values_valid(vals, dev)
        parts[tag + "n"] = red(ok.double(), "sum")
        moments = ("stddev", "variance", "stddev_pop", "var_pop", "skewness", "kurtosis")
        if a.fn in ("sum", "avg") + moments:
            parts[tag + "s"] = red(x, "sum")
        if a.fn in moments:
            parts[tag + "q"] = red(x * x, "sum")
        if a.fn in ("skewness", "kurtosis"):
            parts[tag + "c"] = red(x * x * x, "sum")
            parts[tag + "f"] = red(x * x * x * x, "sum")
        if a.fn in ("min", "max"):
            fill = math.inf if a.fn == "min" else -math.inf
            src = torch.where(ok, x, torch.full_like(x, fill))
            parts[tag + "m"] = red(src, a.fn)
    # ---- merge partials across ranks by key value
    local_keys = [e[1](uk[:, i].tolist()) for i, e in enumerate(enc)] if keys else []
    table = {name: t.cpu().numpy() for name, t in parts.items()}
    payload = (local_keys, table, host_parts)
    pieces = comm.all_gather_object(payload) if comm.world_size > 1 else [payload]
    merged: "OrderedDict[tuple, dict]" = OrderedDict()
    hosts: dict = {}
    for lk, tb, hp in pieces:
        ng = len(next(iter(tb.values()))) if tb else 0
        keylist = [tuple(_hashable(lk[i][g]) for i in range(len(keys))) for g in range(ng)] if keys else [()] * ng
        raw = [tuple(lk[i][g] for i in range(len(keys))) for g in range(ng)] if keys else [()] * ng
        for g, kk in enumerate(keylist):
            m = merged.get(kk)
            if m is None:
                m = merged[kk] = {"__key": raw[g]}
            for name, arr in tb.items():
                v = float(arr[g]) if arr.dtype.kind == "f" else int(arr[g])
                if name not in m:
                    m[name] = v
                elif name == "__first" or (name.endswith("m") and _is_min(name, aggs)):
                    m[name] = min(m[name], v)
                elif name == "__last" or name.endswith("m"):
                    m[name] = max(m[name], v)
                else:
                    m[name] = m[name] + v
        for tag, triples in hp.items():
            for g, r, v in triples:
                hosts.setdefault((keylist[g], tag), []).append((r, v))
    order = sorted(merged.keys(), key=lambda kk: merged[kk]["__first"])
    if not keys and not order:
        order = [()]
        merged[()] = {"__key": (), "__rows": 0.0}
    out = OrderedDict()
    for i, k in enumerate(keys):
        vals = [merged[kk]["__key"][i] for kk in order]
        src = key_cols[i]
        if isinstance(src, C.NumericColumn):
            dt = src.dtype
            arr = np.array([np.nan if v is None else v for v in vals],
                           dtype=np.float64 if src.data.is_floating_point() else np.int64) \
                if not any(v is None for v in vals) or src.data.is_floating_point() else \
                np.array([0 if v is None else v for v in vals], dtype=np.int64)
            valid = None
            if any(v is None for v in vals):
                valid = torch.tensor([v is not None for v in vals])
            out[k.name] = C.NumericColumn(torch.from_numpy(arr), valid, dt)
        else:
            arr = np.empty(len(vals), dtype=object)       # element-wise: equal-length structs must not
            for j, v in enumerate(vals):                    # become a 2-D array
                arr[j] = v
            out[k.name] = C.ArrayColumn(arr) if isinstance(src, C.ArrayColumn) else C.from_numpy(arr, "cpu")
    for j, a in enumerate(aggs):
        tag = f"a{j}"
        res = []
        for kk in order:
            m = merged[kk]
            if tag in host_tags:
                res.append(_host_final(a, sorted(hosts.get((kk, tag), []), key=lambda rv: rv[0])))
            else:
                res.append(_final(a, tag, m))
        out[a.name] = _result_column(a, res)
    return out


def _is_min(name, aggs):
    j = int(name[1:-1])
    return aggs[j].fn == "min"


def _final(a, tag, m):
    cnt = m.get(tag + "n", 0.0)
    if a.fn == "count":
        return int(cnt)
    if cnt == 0:
        return None
    if a.fn == "sum":
        return m[tag + "s"]
    if a.fn == "avg":
        return m[tag + "s"] / cnt
    if a.fn in ("min", "max"):
        return m[tag + "m"]
    if a.fn in ("stddev", "variance"):
        if cnt < 2:
            return None
        mean = m[tag + "s"] / cnt
        var = max((m[tag + "q"] - cnt * mean * mean) / (cnt - 1), 0.0)
        return math.sqrt(var) if a.fn == "stddev" else var
    if a.fn in ("stddev_pop", "var_pop"):
        mean = m[tag + "s"] / cnt
        var = max(m[tag + "q"] / cnt - mean * mean, 0.0)
        return math.sqrt(var) if a.fn == "stddev_pop" else var
    if a.fn in ("skewness", "kurtosis"):
        mu = m[tag + "s"] / cnt
        m2 = max(m[tag + "q"] / cnt - mu * mu, 0.0)
        if m2 == 0.0:
            return None
        if a.fn == "skewness":
            m3 = m[tag + "c"] / cnt - 3 * mu * m[tag + "q"] / cnt + 2 * mu ** 3
            return m3 / m2 ** 1.5
        m4 = (m[tag + "f"] / cnt - 4 * mu * m[tag + "c"] / cnt + 6 * mu * mu * m[tag + "q"] / cnt - 3 * mu ** 4)
        return m4 / (m2 * m2) - 3.0                       # excess kurtosis, like Spark
    if a.fn in ("corr", "covar_pop", "covar_samp"):
        sx, sy = m[tag + "s"], m[tag + "t"]
        cxy = m[tag + "p"] - sx * sy / cnt
        if a.fn == "covar_pop":
            return cxy / cnt
        if a.fn == "covar_samp":
            return cxy / (cnt - 1) if cnt > 1 else None
        cxx, cyy = m[tag + "q"] - sx * sx / cnt, m[tag + "r"] - sy * sy / cnt
        return cxy / math.sqrt(cxx * cyy) if cxx > 0 and cyy > 0 else None
    raise TypeError(f"unsupported aggregate {a.fn}")


def _host_final(a, pairs):
    """pairs: (global row, value) of one group, sorted by row."""
    vals = [v for _, v in pairs]
    nn = [v for v in vals if v is not None and not (isinstance(v, float) and math.isnan(v))]
    if a.fn == "count":
        return len({_hashable(v) for v in nn}) if a.distinct else len(nn)
    if a.fn == "first":
        return vals[0] if vals else None
    if a.fn == "last":
        return vals[-1] if vals else None
    if a.fn == "collect_list":
        return nn
    if a.fn == "collect_set":
        seen, out = set(), []
        for v in nn:
            h = _hashable(v)
            if h not in seen:
                seen.add(h)
                out.append(v)
        return out
    if a.fn in ("max_by", "min_by"):
        # values are [ordering, value] pairs; rows with a null ordering are skipped
        cand = [v for v in vals if v is not None and v[0] is not None
                and not (isinstance(v[0], float) and math.isnan(v[0]))]
        if not cand:
            return None
        pick = max if a.fn == "max_by" else min
        return pick(cand, key=lambda v: v[0])[1]
    if not nn:
        return None
    if a.fn == "median":
        vs = sorted(float(v) for v in nn)
        pos = 0.5 * (len(vs) - 1)
        lo = int(math.floor(pos))
        hi = min(lo + 1, len(vs) - 1)
        return vs[lo] + (vs[hi] - vs[lo]) * (pos - lo)
    if a.fn == "mode":
        counts: dict = {}
        for v in nn:
            counts[_hashable(v)] = counts.get(_hashable(v), 0) + 1
        best = max(counts.values())
        return next(v for v in nn if counts[_hashable(v)] == best)      # first-seen among ties
    if a.fn == "product":
        out = 1.0
        for v in nn:
            out *= float(v)
        return out
    if a.fn == "histogram_numeric":
        return _numeric_histogram(nn, int(a.param))
    if a.fn in ("bit_and", "bit_or", "bit_xor"):
        import functools
        import operator
        op = {"bit_and": operator.and_, "bit_or": operator.or_, "bit_xor": operator.xor}[a.fn]
        return functools.reduce(op, (int(v) for v in nn))
    if a.fn == "bool_and":
        return all(bool(v) for v in nn)
    if a.fn == "bool_or":
        return any(bool(v) for v in nn)
    if a.fn == "percentile_exact":                   # Spark percentile: linear interpolation
        vs = sorted(float(v) for v in nn)
        ps = a.param if isinstance(a.param, (list, tuple)) else [a.param]
        res = []
        for p in ps:
            pos = float(p) * (len(vs) - 1)
            lo = int(math.floor(pos))
            hi = min(lo + 1, len(vs) - 1)
            res.append(vs[lo] + (vs[hi] - vs[lo]) * (pos - lo))
        return res if isinstance(a.param, (list, tuple)) else res[0]
    if a.fn == "percentile":
        vs = sorted(nn)
        ps = a.param if isinstance(a.param, (list, tuple)) else [a.param]
        res = [vs[min(len(vs) - 1, max(0, math.ceil(p * len(vs)) - 1))] for p in ps]
        return res if isinstance(a.param, (list, tuple)) else res[0]
    if a.distinct:
        nn = list({_hashable(v): v for v in nn}.values())
    if a.fn == "min":
        return min(nn)
    if a.fn == "max":
        return max(nn)
    if a.fn == "sum":
        return sum(nn)
    if a.fn == "avg":
        return sum(nn) / len(nn)
    raise TypeError(f"aggregate {a.fn} not supported on this column type")


def _numeric_histogram(vals, nb):
    """Ben-Haim / Tom-Tov histogram (Spark ``histogram_numeric``): every distinct value a
    (centre, count) bin, then the two closest adjacent bins merged into their weighted
    centre until ``nb`` remain.  Returns [Row(x, y)] sorted by x."""
    from .dataframe import Row
    if not vals:
        return None
    xs, cnt = np.unique(np.asarray(vals, dtype=np.float64), return_counts=True)
    xs, cnt = xs.tolist(), cnt.astype(np.float64).tolist()
    while len(xs) > max(nb, 1):
        i = int(np.argmin(np.diff(xs)))
        w = cnt[i] + cnt[i + 1]
        xs[i:i + 2] = [(xs[i] * cnt[i] + xs[i + 1] * cnt[i + 1]) / w]
        cnt[i:i + 2] = [w]
    return [Row._make(["x", "y"], [x, y]) for x, y in zip(xs, cnt)]


def _result_column(a, res):
    if a.fn in ("bit_and", "bit_or", "bit_xor"):
        valid = torch.tensor([r is not None for r in res]) if any(r is None for r in res) else None
        return C.NumericColumn(torch.tensor([0 if r is None else r for r in res], dtype=torch.int64), valid)
    if a.fn == "count":
        return C.NumericColumn(torch.tensor(res, dtype=torch.int64))
    if a.fn in ("collect_list", "collect_set", "histogram_numeric") or (a.fn in ("percentile", "percentile_exact")
                                                    and isinstance(a.param, (list, tuple))):
        arr = np.empty(len(res), dtype=object)
        for i, r in enumerate(res):        # element-wise: equal-length lists must not broadcast
            arr[i] = r
        return C.ArrayColumn(arr)
    if a.fn in ("bool_and", "bool_or"):
        valid = torch.tensor([r is not None for r in res]) if any(r is None for r in res) else None
        return C.NumericColumn(torch.tensor([bool(r) for r in res], dtype=torch.bool), valid)
    if all(r is None or isinstance(r, (int, float, bool)) for r in res):
        arr = np.array([np.nan if r is None else r for r in res], dtype=np.float64)
        valid = torch.from_numpy(np.array([r is not None for r in res])) if any(r is None for r in res) else None
        return C.NumericColumn(torch.from_numpy(arr), valid)
    return C.from_numpy(np.array(res, dtype=object), "cpu")


_ = E
