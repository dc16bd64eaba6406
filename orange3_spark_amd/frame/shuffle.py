"""Row exchange between ranks and the operators built on it: distributed sort
(sample sort), key-hash de-duplication and the multiset operators
(intersect / subtract / exceptAll / intersectAll).

Spark implements these with a shuffle: ``orderBy`` is a range-partitioned exchange whose
boundaries come from a sample of the sort key, ``dropDuplicates`` / ``intersect`` /
``except`` hash-partition rows by their full key and merge per key.  Here, per rank:

* **row keys** are 128-bit (two int64) hashes of the selected columns computed on the
  device: numeric columns contribute their exact 64-bit pattern (+0.0 == -0.0, one NaN,
  a null sentinel), strings a deterministic seeded hash of the value (pandas'
  ``hash_array``, identical across processes, unlike Python's ``hash``);
* for de-duplication and set operators only ``(key, global row id)`` pairs travel -- 24 B
  per row -- to the key's owner rank (``key mod world``); the owner decides which row ids
  survive and sends the survivors back to the rows' home ranks, which apply a mask.  Rows
  never move, so output order is the input's global order (deterministic, independent of
  the number of GPUs);
* ``sort`` computes an order-preserving int64 code per sort column (IEEE bits remapped
  so signed comparison sorts floats, strings ranked against the global sorted set of
  distinct values), picks ``world-1`` splitters from an all-gathered sample of the
  leading code, moves every row to its range owner with one ``all_to_all_v`` per column
  (device columns over RCCL, host columns as one pickled byte buffer), and finishes with
  a stable local lexicographic sort.  Ties stay in source-rank/row order, so the result
  is a stable sort of the global row order.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch

from . import column as C

_NULL = -(1 << 62) - 7
_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1
_M1, _M2 = -7046029254386353131, -4658895280553007687        # splitmix64 constants as int64


def _mix(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser on int64 (wrapping arithmetic; logical shifts emulated)."""
    def srl(v, k):
        return (v >> k) & ((1 << (64 - k)) - 1)
    x = (x ^ srl(x, 30)) * _M1
    x = (x ^ srl(x, 27)) * _M2
    return x ^ srl(x, 31)


def _host_values(c: C.Column) -> np.ndarray:
    return c.values if isinstance(c, C.HostColumn) else np.asarray(c.to_pylist(), dtype=object)


def _column_codes(c: C.Column, dev) -> tuple[torch.Tensor, torch.Tensor]:
    """Two independent 64-bit codes per row (exact for numeric columns)."""
    if isinstance(c, C.NumericColumn):
        d = c.data
        if d.is_floating_point():
            d64 = d.to(torch.float64)
            bits = d64.view(torch.int64).clone()
            bits = torch.where(d64 == 0, torch.zeros_like(bits), bits)
            bits = torch.where(torch.isnan(d64), torch.full_like(bits, 0x7FF8000000000000), bits)
        else:
            bits = d.to(torch.int64)
        if c.valid is not None:
            bits = torch.where(c.null_mask().to(bits.device), torch.full_like(bits, _NULL), bits)
        bits = bits.to(dev)
        return bits, _mix(bits ^ 0x5851F42D4C957F2D)
    if isinstance(c, C.VectorColumn):
        d = c.dense().to(torch.float64)
        bits = torch.where(d == 0, torch.zeros_like(d), d).view(torch.int64)
        h1 = torch.zeros(d.shape[0], dtype=torch.int64, device=d.device)
        h2 = torch.full_like(h1, 0x2545F4914F6CDD1D)
        for j in range(d.shape[1]):
            h1 = _mix(h1 * 31 + bits[:, j])
            h2 = _mix(h2 ^ bits[:, j])
        return h1.to(dev), h2.to(dev)
    import pandas as pd
    vals = _host_values(c)
    norm = np.array([None if v is None or (isinstance(v, float) and math.isnan(v))
                     else (repr(tuple(v)) if isinstance(v, (list, tuple)) else
                           repr(tuple(np.asarray(v.toArray()).tolist())) if hasattr(v, "toArray") else v)
                     for v in vals], dtype=object)
    h1 = pd.util.hash_array(norm, hash_key="o3s-key-01234567", categorize=False).view(np.int64)
    h2 = pd.util.hash_array(norm, hash_key="o3s-key-fedcba98", categorize=False).view(np.int64)
    return torch.from_numpy(h1.copy()).to(dev), torch.from_numpy(h2.copy()).to(dev)


def row_keys(df, cols=None) -> torch.Tensor:
    """[n, 2] int64 128-bit row key over ``cols`` (default: all columns)."""
    names = list(df.columns) if not cols else list(cols)
    dev = df.device
    k1 = torch.full((len(df),), 0x243F6A8885A308D3, dtype=torch.int64, device=dev)
    k2 = torch.full((len(df),), 0x13198A2E03707344, dtype=torch.int64, device=dev)
    for name in names:
        a, b = _column_codes(df._col(name), dev)
        k1 = _mix(k1 * 0x100000001B3 + a) if len(names) > 1 else a
        k2 = _mix(k2 ^ b)
    return torch.stack([k1, k2], 1)


def _exchange_tensors(comm, dest: torch.Tensor, tensors: list) -> list:
    """Send row i of every tensor to rank dest[i]; rows arrive in source-rank order."""
    w = comm.world_size
    if w == 1:
        return tensors
    perm = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=w).cpu().tolist()
    return [comm.all_to_all_v(t[perm].contiguous(), counts)[0] for t in tensors]


def _home_rank(comm, ids: torch.Tensor, sizes) -> torch.Tensor:
    bounds = torch.tensor(np.cumsum(sizes), dtype=torch.int64, device=ids.device)
    return torch.searchsorted(bounds, ids, right=True)


def _lexsort2(k: torch.Tensor, tie: torch.Tensor) -> torch.Tensor:
    """Permutation sorting rows by (k[:,0], k[:,1], tie)."""
    o = torch.argsort(tie, stable=True)
    o = o[torch.argsort(k[o, 1], stable=True)]
    return o[torch.argsort(k[o, 0], stable=True)]


def _segments(ks: torch.Tensor) -> torch.Tensor:
    """Segment id per row of key-sorted [m, 2] keys."""
    if ks.shape[0] == 0:
        return torch.zeros(0, dtype=torch.int64, device=ks.device)
    new = torch.ones(ks.shape[0], dtype=torch.bool, device=ks.device)
    new[1:] = (ks[1:] != ks[:-1]).any(1)
    return torch.cumsum(new.to(torch.int64), 0) - 1


def keep_mask(a, a_cols, rule: str, b=None, b_cols=None) -> torch.Tensor:
    """Per-row keep mask of ``a`` for: ``distinct`` (first occurrence of each key),
    ``intersect`` / ``subtract`` (first occurrence, key present / absent in ``b``),
    ``intersect_all`` (first min(ca, cb) occurrences), ``except_all`` (first
    max(ca - cb, 0) occurrences).  Occurrence order is the global row order."""
    comm, dev = a.comm, a.device
    w = comm.world_size
    ka = row_keys(a, a_cols)
    ida = a._global_rows()
    owner = (ka[:, 0] % w) if w > 1 else torch.zeros(len(a), dtype=torch.int64, device=dev)
    ka_r, ida_r = _exchange_tensors(comm, owner, [ka, ida])
    if b is not None:
        kb = row_keys(b, b_cols).to(dev)
        ob = (kb[:, 0] % w) if w > 1 else torch.zeros(len(b), dtype=torch.int64, device=dev)
        (kb_r,) = _exchange_tensors(comm, ob, [kb])
    m = ka_r.shape[0]
    o = _lexsort2(ka_r, ida_r)
    ks, ids = ka_r[o], ida_r[o]
    seg = _segments(ks)
    nseg = int(seg[-1].item()) + 1 if m else 0
    starts = torch.zeros(nseg, dtype=torch.int64, device=dev)
    if m:
        starts.scatter_reduce_(0, seg, torch.arange(m, device=dev), "amin", include_self=False)
    occ = torch.arange(m, device=dev) - starts[seg] if m else seg
    if rule == "distinct":
        keep = occ == 0
    else:
        if nseg:
            uk = ks[starts]
            kb_all = torch.cat([uk, kb_r]) if kb_r.numel() else uk
            tag = torch.cat([torch.zeros(nseg, dtype=torch.int64, device=dev),
                             torch.ones(kb_r.shape[0], dtype=torch.int64, device=dev)])
            oo = _lexsort2(kb_all, tag)                       # each a-key first, then its b rows
            s2 = _segments(kb_all[oo])
            cnt_b_per_s2 = torch.bincount(s2, weights=tag[oo].to(torch.float64)).to(torch.int64)
            a_pos = oo[tag[oo] == 0]                          # a-segment indices in sorted order
            cb = torch.zeros(nseg, dtype=torch.int64, device=dev)
            cb[a_pos] = cnt_b_per_s2[s2[tag[oo] == 0]]
        else:
            cb = torch.zeros(0, dtype=torch.int64, device=dev)
        cbr = cb[seg]
        if rule == "intersect":
            keep = (occ == 0) & (cbr > 0)
        elif rule == "subtract":
            keep = (occ == 0) & (cbr == 0)
        elif rule == "intersect_all":
            keep = occ < cbr
        elif rule == "except_all":
            ca = torch.bincount(seg, minlength=nseg)[seg]
            keep = occ < (ca - cbr)
        else:
            raise ValueError(rule)
    kept = ids[keep]
    if w > 1:
        home = _home_rank(comm, kept, a.partition_sizes())
        (kept,) = _exchange_tensors(comm, home, [kept])
    mask = torch.zeros(len(a), dtype=torch.bool, device=dev)
    mask[kept - a.row_offset()] = True
    return mask


# --------------------------------------------------------------------------- sorting
def _order_code(comm, c: C.Column, asc: bool, nulls_first: bool) -> torch.Tensor:
    """int64 per row whose signed order is the requested sort order."""
    if isinstance(c, C.NumericColumn):
        d = c.data
        if d.is_floating_point():
            d64 = d.to(torch.float64)
            bits = torch.where(d64 == 0, torch.zeros_like(d64), d64).view(torch.int64).clone()
            bits = torch.where(torch.isnan(d64), torch.full_like(bits, 0x7FF8000000000000), bits)
            code = torch.where(bits < 0, bits ^ 0x7FFFFFFFFFFFFFFF, bits)       # NaN sorts last (Spark)
        else:
            code = d.to(torch.int64)
        null = c.null_mask().to(code.device) if c.valid is not None else None
    else:
        vals = _host_values(c)
        isnull = np.array([v is None or (isinstance(v, float) and math.isnan(v)) for v in vals], dtype=bool)
        local = sorted({v for v, z in zip(vals, isnull) if not z})
        glob = sorted(set().union(*map(set, comm.all_gather_object(local)))) if comm.world_size > 1 else local
        arr = np.empty(len(glob), dtype=object)
        arr[:] = glob
        rank = np.searchsorted(arr, np.where(isnull, arr[0] if len(arr) else "", vals).astype(object)) \
            if len(arr) else np.zeros(len(vals), dtype=np.int64)
        code = torch.from_numpy(np.asarray(rank, dtype=np.int64))
        null = torch.from_numpy(isnull) if isnull.any() else None
    if not asc:
        code = ~code
    if null is not None:
        code = torch.where(null.to(code.device), torch.full_like(code, _I64_MIN if nulls_first else _I64_MAX), code)
    return code


def exchange(df, dest: torch.Tensor):
    """New DataFrame holding the rows sent here (row i of ``df`` goes to rank dest[i])."""
    from .dataframe import DataFrame
    comm = df.comm
    w = comm.world_size
    if w == 1:
        return df
    dest = dest.to(df.device)
    perm = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=w).cpu().tolist()
    src = df._take(perm)
    out = OrderedDict((k, _exchange_column(comm, c, counts)) for k, c in src._cols.items())
    if out:
        n = len(next(iter(out.values())))
    else:
        n = sum(cs[comm.rank] for cs in comm.all_gather_object(counts))
    return DataFrame(df.session, out, n)


def _exchange_column(comm, c: C.Column, counts) -> C.Column:
    dev = comm.device
    if isinstance(c, C.NumericColumn):
        d = c.data
        is_bool = d.dtype == torch.bool
        send = d.to(torch.uint8) if is_bool else d
        recv, _ = comm.all_to_all_v(send.to(dev), counts)
        has_valid = comm.max_scalar(1.0 if c.valid is not None else 0.0) > 0
        valid = None
        if has_valid:
            v = c.valid if c.valid is not None else torch.ones(len(c), dtype=torch.bool, device=d.device)
            valid = comm.all_to_all_v(v.to(torch.uint8).to(dev), counts)[0].bool()
        return C.NumericColumn(recv.bool() if is_bool else recv, valid, c.dtype)
    if isinstance(c, C.VectorColumn):
        recv, _ = comm.all_to_all_v(c.data.to(dev), counts)
        return C.VectorColumn(recv, c.size)
    if isinstance(c, C.SparseVectorColumn):
        lens = (c.indptr[1:] - c.indptr[:-1]).to(dev)
        nnz_counts, off = [], 0
        cs = torch.cumsum(lens, 0).cpu().tolist()
        for cnt in counts:
            end = off + cnt
            nnz_counts.append(int((cs[end - 1] if end > 0 else 0) - (cs[off - 1] if off > 0 else 0)) if cnt else 0)
            off = end
        rl, _ = comm.all_to_all_v(lens, counts)
        ri, _ = comm.all_to_all_v(c.indices.to(dev), nnz_counts)
        rv, _ = comm.all_to_all_v(c.values.to(dev), nnz_counts)
        ptr = torch.zeros(rl.numel() + 1, dtype=torch.int64, device=dev)
        ptr[1:] = torch.cumsum(rl, 0)
        return C.SparseVectorColumn(ptr, ri, rv, c.size)
    vals = c.values
    parts, off = [], 0
    for cnt in counts:
        parts.append(vals[off:off + cnt])
        off += cnt
    got = comm.all_to_all_object(parts)
    merged = np.empty(sum(len(g) for g in got), dtype=object)
    if len(merged):
        merged[:] = [v for g in got for v in g]
    return _host_like(c, merged)


def _host_like(c: C.HostColumn, values: np.ndarray) -> C.HostColumn:
    out = c.slice(0, 0)
    out.values = values
    return out


def local_sort_perm(codes: list[torch.Tensor]) -> torch.Tensor:
    n = codes[0].numel()
    o = torch.arange(n, device=codes[0].device)
    for k in reversed(codes):
        o = o[torch.argsort(k[o], stable=True)]
    return o


def sort(df, exprs: list, ascending: list, nulls_first: list):
    """Distributed sample sort (see module docstring)."""
    comm = df.comm
    w = comm.world_size
    cols = [e.eval(df) for e in exprs]
    codes = [_order_code(comm, c, a, nf).to(df.device) for c, a, nf in zip(cols, ascending, nulls_first)]
    if w > 1:
        lead = codes[0]
        s = min(len(df), 64 * w)
        if s:
            pick = torch.linspace(0, len(df) - 1, s, device=df.device).round().long()
            sample = lead[pick]
        else:
            sample = lead[:0]
        allsamp = torch.sort(comm.all_gather_v(sample.to(comm.device))).values
        if allsamp.numel():
            q = torch.linspace(0, allsamp.numel() - 1, w + 1, device=allsamp.device)[1:-1].round().long()
            splitters = allsamp[q].to(df.device)
        else:
            splitters = torch.zeros(w - 1, dtype=torch.int64, device=df.device)
        dest = torch.searchsorted(splitters, lead, right=True)
        tmp = df._new(OrderedDict(list(df._cols.items()) +
                                  [(f"__sort{i}", C.NumericColumn(k)) for i, k in enumerate(codes)]))
        moved = exchange(tmp, dest)
        codes = [moved._cols.pop(f"__sort{i}").data for i in range(len(codes))]
        df = moved._new(moved._cols, len(moved))
    return df._take(local_sort_perm(codes))
