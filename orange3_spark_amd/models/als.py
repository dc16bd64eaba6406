"""Alternating least squares (explicit + implicit feedback) over row-sharded ratings.

Replaces Spark ALS (reached through the Recommendation widget,
orangecontrib/spark/widgets/ml/spark_ml_recommendation.py:15).  Layout per rank:
ratings are exchanged twice with ``all_to_all`` so that each rank holds the CSR of its
user block AND of its item block (Spark's in/out blocks); factor tables are sharded by
block and the *other* side is all-gathered each half-iteration (an item-side
all-reduce of normal equations would be ~330 GB; the factor all-gather is 25.6 GB users /
2.56 GB items at rank 128).

Each half-iteration solves, for every local row u,
    (YtY[implicit] + sum_j w_j y_j y_j^T + lambda n_u I) x_u = sum_j b_j y_j
(Spark's formulation: implicit w = alpha|r|, b = (1 + alpha|r|)[r > 0], n_u = #positive;
explicit w = 1, b = r, n_u = #ratings) EXACTLY by default, like Spark's per-row Cholesky:
the ``als_exact`` gfx950 kernels (Woodbury against the eigendecomposition of YtY for rows
with <= 32 ratings, register Gram + LDS Cholesky for longer rows; ops/als.py).  With
``cg_iters > 0`` (ALS ``cgIters``) large problems instead run that many warm-started
conjugate-gradient steps whose matvec is the ``als_pass`` kernel (opt-in approximation).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import als as A
from ..ops import sampling
from ..runtime.tracing import trace
from ..runtime import progress


@dataclass
class Csr:
    indptr: torch.Tensor      # int64 [nrows+1]
    cols: torch.Tensor        # int32 dense index of the other side
    vals: torch.Tensor        # float32 ratings
    row_lo: int               # first dense row index owned by this rank
    nrows: int
    cache: dict = field(default_factory=dict)   # per-(implicit, alpha, reg) solve constants


# ids spanning at most this many values per distinct id take the bitmap / lookup-table
# paths (O(n) scatters) instead of sorting: Spark ids are ints, usually dense-ish
DENSE_ID_SPAN = 8


def _id_range(comm, ids: torch.Tensor):
    lo = int(ids.min()) if ids.numel() else 1 << 62
    hi = int(ids.max()) if ids.numel() else -(1 << 62)
    if comm.world_size > 1:
        lo, hi = -comm.max_scalar(-lo), comm.max_scalar(hi)
    return int(lo), int(hi)


def global_ids(comm, ids: torch.Tensor) -> torch.Tensor:
    """Sorted unique ids over all ranks (replicated).  Dense id ranges use a presence
    bitmap (one scatter, one max all-reduce of span bytes, one nonzero) instead of a sort of
    every id (1B ids: a 150 ms radix sort)."""
    if ids.dtype not in (torch.int32, torch.int64):
        ids = ids.to(torch.int64)
    lo, hi = _id_range(comm, ids)
    span = hi - lo + 1
    # the path choice picks the collective (max all-reduce vs all_gather_v), so it must be
    # made from values every rank agrees on: the global id count, not a local estimate
    n_total = comm.sum_scalar(int(ids.numel())) if comm.world_size > 1 else int(ids.numel())
    if hi >= lo and span <= DENSE_ID_SPAN * max(1, n_total) and span <= (1 << 33):
        mark = torch.zeros(span, dtype=torch.uint8, device=ids.device)
        mark[_offsets(ids, lo, span)] = 1
        if comm.world_size > 1:
            comm.all_reduce(mark, "max")
        return torch.nonzero(mark).reshape(-1) + lo
    u = torch.unique(ids.to(torch.int64))
    if comm.world_size > 1:
        u = torch.unique(comm.all_gather_v(u))
    return u


def _offsets(ids: torch.Tensor, lo: int, span: int) -> torch.Tensor:
    """ids - lo, in int32 when the ids are int32 and the span fits (no int64 copy of a
    billion ids), else in int64."""
    if ids.dtype == torch.int32 and span < (1 << 31) and lo >= -(1 << 31):
        return ids - lo if lo == 0 or -(1 << 31) <= -lo < (1 << 31) else ids.to(torch.int64) - lo
    return ids.to(torch.int64) - lo


def dense_index(uid: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """Position of every id in the sorted unique table ``uid``: a lookup table over the id
    span when it is dense (one scatter + one gather; int32 positions when they fit), else a
    binary search (int64)."""
    if ids.dtype not in (torch.int32, torch.int64):
        ids = ids.to(torch.int64)
    if uid.numel() == 0:
        return torch.zeros(ids.shape, dtype=torch.int64, device=ids.device)
    lo, hi = int(uid[0]), int(uid[-1])
    span = hi - lo + 1
    if span <= DENSE_ID_SPAN * uid.numel() and span <= (1 << 33):
        lut = torch.empty(span, dtype=torch.int32 if uid.numel() < (1 << 31) else torch.int64, device=uid.device)
        lut[uid - lo] = torch.arange(uid.numel(), dtype=lut.dtype, device=uid.device)
        return lut[_offsets(ids, lo, span)]
    return torch.searchsorted(uid, ids.to(torch.int64))


def block_bounds(n: int, world: int, r: int) -> tuple[int, int]:
    return (n * r) // world, (n * (r + 1)) // world


def partition(comm, rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n_rows: int) -> Csr:
    """Route each rating to the rank owning its row block; build CSR sorted by row."""
    W, r = comm.world_size, comm.rank
    if W > 1:
        # the rank r with block_bounds(n_rows, W, r) containing the row:
        # floor(n r / W) <= x  <=>  r <= ceil((x + 1) W / n) - 1
        rows = rows.to(torch.int64)
        owner = torch.div((rows + 1) * W + n_rows - 1, n_rows, rounding_mode="floor") - 1
        order = torch.argsort(owner, stable=True)
        counts = torch.bincount(owner, minlength=W).tolist()
        packed = torch.stack([rows[order].to(torch.float64), cols[order].to(torch.float64),
                              vals[order].to(torch.float64)], 1)
        recv, _ = comm.all_to_all_v(packed, counts)
        rows, cols, vals = recv[:, 0].long(), recv[:, 1].long(), recv[:, 2].float()
    lo, hi = block_bounds(n_rows, W, r)
    # local row keys in 32 bits when they fit (half the radix passes of int64 keys); the
    # sorted row ids themselves are never needed -- the counts come from the unsorted keys
    key = rows - lo
    if hi - lo < (1 << 31):
        key = key.to(torch.int32)
    o = torch.argsort(key, stable=True)
    cols, vals = cols.to(torch.int32)[o], vals[o]
    cnt = torch.bincount(key, minlength=hi - lo) if key.numel() else torch.zeros(hi - lo, dtype=torch.int64,
                                                                                  device=rows.device)
    del key, o
    indptr = torch.zeros(hi - lo + 1, dtype=torch.int64, device=rows.device)
    indptr[1:] = torch.cumsum(cnt, 0)
    return Csr(indptr, cols.contiguous(), vals.contiguous(), lo, hi - lo)


def init_factors(n_lo: int, n: int, rank: int, seed: int, device, nonneg: bool) -> torch.Tensor:
    """Unit-norm gaussian rows keyed on (seed, global index): partition invariant.

    GPU: ``als_init_kernel`` (one wave per row); CPU: the same draws in torch."""
    out = torch.empty((n, rank), dtype=torch.float32, device=device)
    if out.is_cuda and 0 < rank <= 512:
        from ..ops import _native as N
        N.check(N.kernels().o3s_als_init(int(n_lo), int(n), int(rank), int(seed) & 0xFFFFFFFF, int(bool(nonneg)),
                                         out.data_ptr(), N.stream_of(out)), "als_init")
        return out
    s1 = [2 * k + 11 for k in range(rank)]
    s2 = [2 * k + 12 for k in range(rank)]
    step = max(1, (1 << 25) // max(rank, 1))                 # bounded int64 temporaries
    for a in range(0, n, step):
        idx = torch.arange(n_lo + a, n_lo + min(n, a + step), dtype=torch.int64, device=device)
        u1 = sampling.uniform_streams(idx, seed, s1).clamp_min(1e-12)
        u2 = sampling.uniform_streams(idx, seed, s2)
        out[a:a + idx.numel()] = (torch.sqrt(-2 * torch.log(u1)) * torch.cos(2 * math.pi * u2)).float()
    out /= out.norm(dim=1, keepdim=True).clamp_min(1e-12)
    return out.abs() if nonneg else out


def _weights(vals: torch.Tensor, implicit: bool, alpha: float):
    if implicit:
        c1 = alpha * vals.abs()
        b = torch.where(vals > 0, 1.0 + c1, torch.zeros_like(c1))
        return c1.float().contiguous(), b.float().contiguous(), (vals > 0)
    return torch.ones_like(vals).float().contiguous(), vals.float().contiguous(), torch.ones_like(vals, dtype=torch.bool)


def _row_counts(indptr: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
    """Per CSR row, the number of True entries of ``pos`` (fp32): differences of one
    prefix sum at the row bounds (no per-rating row-id tensor, no scatter-add)."""
    n = indptr.numel() - 1
    if pos.numel() == 0:
        return torch.zeros(n, dtype=torch.float32, device=pos.device)
    cs = torch.cumsum(pos, 0, dtype=torch.int32 if pos.numel() < (1 << 31) else torch.int64)
    ends, starts = indptr[1:], indptr[:-1]
    hi = torch.where(ends > 0, cs[(ends - 1).clamp_min(0)], torch.zeros((), dtype=cs.dtype, device=cs.device))
    lo = torch.where(starts > 0, cs[(starts - 1).clamp_min(0)], torch.zeros((), dtype=cs.dtype, device=cs.device))
    return (hi - lo).to(torch.float32)


FUSED_CG = True        # False: CG bookkeeping as separate torch ops (reference path)
# rows averaging at least this many ratings are solved exactly (MFMA Gram + batched
# Cholesky, Spark's per-row solve) instead of by warm-started CG; 0 disables.  Off by
# default: on the rank-128 item side of the ALS config it measured 0.58 s/iteration vs
# 0.154 s with CG (the batched rocSOLVER Cholesky and the gather-latency-bound Gram cost
# more than the 4 CG gather passes; profiles/als_dense_solve_experiment.json).
DENSE_MIN_AVG = 0


def solve_side(csr: Csr, Ffull: torch.Tensor, X0: torch.Tensor, reg: float, implicit: bool, alpha: float,
               FtF: torch.Tensor | None, cg_iters: int, nonneg: bool, exact: bool | None = None,
               row_range: tuple[int, int] | None = None, eig_basis: bool = False) -> torch.Tensor:
    """New factors of the rows of ``csr`` (all of them, or the CG solve of rows [a, b)
    written IN PLACE into ``X0[a:b]``, which is returned -- the chunked path of
    :func:`fit_als`, whose per-chunk results are all-gathered while later chunks solve)."""
    n, R = csr.nrows, Ffull.shape[1]
    dev = Ffull.device
    key = (implicit, float(alpha), float(reg))
    if key not in csr.cache:          # the ratings do not change between iterations
        with trace("als.weights"):
            w, b, pos = _weights(csr.vals, implicit, alpha)
            nu = _row_counts(csr.indptr, pos)
            csr.cache.clear()
            csr.cache[key] = (w, b, (reg * nu).to(torch.float32).contiguous())
            del pos
    w, b, lam = csr.cache[key]
    nnz = int(csr.cols.numel())
    if exact is None:
        exact = cg_iters <= 0 or nnz * R * R <= (1 << 26)
    if exact:
        # Spark's per-row exact solve: gfx950 kernels (Woodbury for short rows, register
        # Gram + LDS Cholesky for long ones), the fp64 torch path elsewhere
        out = X0 if row_range is not None else torch.empty((n, R), dtype=torch.float32, device=dev)
        with trace("als.exact_solve"):
            if A.exact_kernel_ok(Ffull) and out.is_contiguous():
                A.exact_solve(csr.indptr, csr.cols, w, b, Ffull, FtF if implicit else None, lam, implicit, out,
                              row_range, eig_basis=eig_basis)
            else:
                assert not eig_basis, "eig_basis needs the exact-solve kernels"
                A.exact_solve_torch(csr.indptr, csr.cols, w, b, Ffull, FtF if implicit else None, lam, out,
                                    row_range)
        if nonneg:
            sl = out if row_range is None else out[row_range[0]:row_range[1]]
            sl.clamp_(min=0)
        return out
    indptr = csr.indptr
    if row_range is not None:
        a, e = row_range
        indptr, lam, X0, n = csr.indptr[a:e + 1], lam[a:e], X0[a:e], e - a
    if row_range is None and not exact and not nonneg and DENSE_MIN_AVG and A.gram_ok(Ffull) and nnz >= DENSE_MIN_AVG * max(n, 1):
        # many ratings per row (the item side): exact solves, Gram on MFMA + batched Cholesky
        with trace("als.dense_solve"):
            return A.dense_solve(csr.indptr, csr.cols, w, b, Ffull, FtF if implicit else None, lam)

    def Amul(v):
        out = A.pass_(0, indptr, csr.cols, w, Ffull, v)
        if implicit and FtF is not None:
            out = out + v @ FtF
        return out + lam[:, None] * v

    x = X0 if row_range is not None else X0.clone()
    # first residual: the rhs and A x0 gather the same factor rows -> one fused pass
    ax, rhs = A.pass_both(indptr, csr.cols, w, Ffull, x, b)
    if FUSED_CG and A.cg_kernel_ok(Ffull) and x.is_contiguous() and x.dtype == torch.float32:
        # device path: every CG vector update is one fused row-wise kernel (als_cg_kernel)
        use_g = implicit and FtF is not None
        lam_c = lam.contiguous()
        r, p, rs = A.cg_init(x, ax, (x @ FtF) if use_g else None, rhs, lam_c)
        del ax, rhs
        for _ in range(cg_iters):
            ap = A.pass_(0, indptr, csr.cols, w, Ffull, p)
            A.cg_step(x, r, p, ap, (p @ FtF) if use_g else None, lam_c, rs)
        return x.clamp_(min=0) if nonneg else x
    if implicit and FtF is not None:
        ax = ax + x @ FtF
    r = rhs - (ax + lam[:, None] * x)
    p = r.clone()
    rs = (r * r).sum(1)
    for _ in range(cg_iters):
        Ap = Amul(p)
        den = (p * Ap).sum(1)
        al = torch.where(den > 0, rs / den.clamp_min(1e-30), torch.zeros_like(rs))
        x += al[:, None] * p
        r = r - al[:, None] * Ap
        rs_new = (r * r).sum(1)
        beta = torch.where(rs > 0, rs_new / rs.clamp_min(1e-30), torch.zeros_like(rs))
        p = r + beta[:, None] * p
        rs = rs_new
    return x.clamp_(min=0) if nonneg else x


def gram(F: torch.Tensor, chunk: int = 1 << 20) -> torch.Tensor:
    """F^T F (fp64 [R, R]).  On the GPU (fp32, R <= 128): ``ftf_kernel`` -- exact fp32
    products on the matrix cores, each wave summing its own row range, the wave partials
    added in fp64 in a fixed order.  Elsewhere: chunked fp32 GEMMs accumulated in fp64 (one
    fp64 GEMM over millions of rows runs on the fp64 matrix path, ~180 ms for 6.25M x 128;
    hipBLASLt's fp32 GEMM of this shape keeps a few CUs busy: ~1.8 ms per 1M rows)."""
    R = F.shape[1]
    if (F.is_cuda and F.dtype == torch.float32 and F.dim() == 2 and 0 < R <= 128 and F.stride(1) == 1
            and F.shape[0] > 0):
        with trace("als.gram", rows=F.shape[0]):
            return A.ftf(F)
    out = torch.zeros((R, R), dtype=torch.float64, device=F.device)
    for a in range(0, F.shape[0], chunk):
        Fc = F[a:a + chunk].float()
        out += (Fc.T @ Fc).double()
    return out


# implicit exact fits keep the factor tables in the eigenbasis of the previous Gram (see
# fit_als): False rotates every user-side Woodbury row back each iteration instead
EIG_BASIS = True


# row chunks per half-iteration on several ranks: chunk c's all-gather (RCCL, its own
# stream) overlaps the solve of chunk c+1; only the last chunk's transfer is exposed.
# GATHER_CHUNKS = None: from the comm model below (BASELINE.md "ALS at N = 2/4/8: comm
# budget"); an int forces that many chunks.
GATHER_CHUNKS: int | None = None
# all-gather rate each rank RECEIVES at (bytes/s) -- an estimate for RCCL over the 7 xGMI
# links of an MI355X node until a multi-GPU run measures it (O3S_ALS_GATHER_GBPS overrides)
GATHER_BPS = float(__import__("os").environ.get("O3S_ALS_GATHER_GBPS", "300")) * 1e9
GATHER_TAIL_S = 2e-3          # target exposed tail (the last chunk's transfer)
GATHER_MAX_CHUNKS = 16        # per-chunk fixed costs (launches, collective latency) cap it


def gather_chunks(rows: int, rank: int, world: int) -> int:
    """Chunks for the slot-layout all-gather of a [rows, rank] fp32 table at ``world``
    ranks: the transfer each rank receives, (W-1)/W of the table at GATHER_BPS, split so
    the exposed last chunk stays under GATHER_TAIL_S (2..GATHER_MAX_CHUNKS chunks)."""
    if GATHER_CHUNKS is not None:
        return max(1, int(GATHER_CHUNKS))
    t_gather = rows * rank * 4 * (world - 1) / max(world, 1) / GATHER_BPS
    return int(min(GATHER_MAX_CHUNKS, max(2, math.ceil(t_gather / GATHER_TAIL_S))))


def _slot_len(n: int, world: int, chunks: int) -> int:
    blk = -(-n // world)                 # largest row block of any rank
    return max(1, -(-blk // chunks))


def _slot_pos(idx: torch.Tensor, n: int, world: int, L: int) -> torch.Tensor:
    """Row of global index ``idx`` in the slot-layout table: rank r's local row o sits in
    chunk c = o // L at c*world*L + r*L + o % L (the order all_gather_into_tensor of
    equal L-row chunks writes)."""
    idx = idx.to(torch.int64)
    los = torch.tensor([block_bounds(n, world, r)[0] for r in range(world)], dtype=torch.int64, device=idx.device)
    owner = torch.searchsorted(los, idx, right=True) - 1
    o = idx - los[owner]
    c = torch.div(o, L, rounding_mode="floor")
    return c * (world * L) + owner * L + (o - c * L)


def _gather_slots(comm, F: torch.Tensor, table: torch.Tensor, L: int, solve) -> None:
    """For each chunk c of this rank's rows: ``solve(a, e)`` updates F[a:e] in place (if
    given), then F[a:e] (zero-padded to L rows) is all-gathered asynchronously into the
    table's chunk-c slots; returns after ordering the stream behind every transfer."""
    n, W = F.shape[0], comm.world_size
    chunks = table.shape[0] // (W * L)
    works, keep = [], []
    for c in range(chunks):
        a, e = min(c * L, n), min((c + 1) * L, n)
        if solve is not None and e > a:
            solve(a, e)
        src = F[a:e]
        if e - a != L:
            src = torch.zeros((L, F.shape[1]), dtype=F.dtype, device=F.device)
            src[: e - a] = F[a:e]
        keep.append(src)
        with trace("als.gather_chunk"):
            works.append(comm.all_gather_into(table[c * W * L:(c + 1) * W * L], src, async_op=True))
    for w in works:
        if w is not None:
            w.wait()


@dataclass
class AlsResult:
    user_ids: torch.Tensor
    item_ids: torch.Tensor
    U: torch.Tensor            # full user factors [nU, R] (replicated)
    V: torch.Tensor            # full item factors [nI, R]
    seconds: float = 0.0
    iter_seconds: list = field(default_factory=list)


def fit_als(comm, users: torch.Tensor, items: torch.Tensor, ratings: torch.Tensor, rank: int = 10,
            max_iter: int = 10, reg: float = 0.1, implicit: bool = False, alpha: float = 1.0, seed: int = 0,
            nonneg: bool = False, cg_iters: int = 0, exact: bool | None = None, keep_full: bool = True,
            ckpt=None) -> AlsResult:
    try:
        return _fit_als(comm, users, items, ratings, rank, max_iter, reg, implicit, alpha, seed, nonneg, cg_iters,
                        exact, keep_full, ckpt)
    finally:
        # also when the fit stops early (FitCancelled from a progress report, a device
        # error): the rotated factor table and the padded copy are as large as a factor
        # table and must not outlive the fit
        A.EIG_CACHE.clear()
        A.PAD_CACHE.clear()


def _fit_als(comm, users, items, ratings, rank, max_iter, reg, implicit, alpha, seed, nonneg, cg_iters, exact,
             keep_full, ckpt) -> AlsResult:
    t0 = time.time()
    dev = ratings.device
    with trace("als.setup.ids"):
        uid = global_ids(comm, users)
        iid = global_ids(comm, items)
        uix = dense_index(uid, users)
        iix = dense_index(iid, items)
        nU, nI = uid.numel(), iid.numel()
    with trace("als.setup.partition"):
        by_user = partition(comm, uix, iix, ratings.float(), nU)
        by_item = partition(comm, iix, uix, ratings.float(), nI)
    with trace("als.setup.init"):
        X = init_factors(by_user.row_lo, by_user.nrows, rank, seed, dev, nonneg)
        Y = init_factors(by_item.row_lo, by_item.nrows, rank, seed ^ 0x5A5A, dev, nonneg)
    its = []
    start = 0
    last = ckpt.latest() if ckpt is not None else None
    if last is not None and tuple(last[1]["X"].shape) == tuple(X.shape) \
            and tuple(last[1]["Y"].shape) == tuple(Y.shape):
        start, st, _ = last              # resume: this rank's factor shards (runtime/checkpoint.py)
        X = torch.from_numpy(st["X"]).to(dev, X.dtype)
        Y = torch.from_numpy(st["Y"]).to(dev, Y.dtype)
    small = max(by_user.cols.numel(), by_item.cols.numel()) * rank * rank <= (1 << 26)
    chunked = comm.world_size > 1 and not small
    # implicit exact solves on the kernels keep both tables in a moving orthonormal basis B
    # (X B, Y B): the user side returns its rows in the eigenbasis of the item Gram (no
    # x = Q y rotation of the 50M-row side per iteration), the item side solves in that
    # basis unchanged, and B accumulates the per-iteration eigenbases (fp64, host); the
    # tables are rotated back once, when the fit ends (or a checkpoint is written)
    eigmode = (EIG_BASIS and implicit and not nonneg and dev.type == "cuda" and rank in A.EXACT_RANKS
               and X.dtype == torch.float32 and (exact is True or (exact is None and cg_iters <= 0)))
    basis = [None]                       # [R, R] fp64 (host); None = the identity
    if eigmode and comm.world_size > 1:
        A.EIG_CACHE.comm = comm          # the eigenbasis comes from rank 0

    def to_orig(T):
        if basis[0] is None:
            return T
        return A.rotated_table(T.contiguous(), basis[0].t().contiguous().float().to(T.device))
    if chunked:
        # factor tables in "slot" layout: every all-gather lands in place (no staging copy,
        # no concatenation) and chunk c of every rank is gathered while chunk c+1 solves
        Cu, Ci = gather_chunks(nU, rank, comm.world_size), gather_chunks(nI, rank, comm.world_size)
        Ls, Li = _slot_len(nU, comm.world_size, Cu), _slot_len(nI, comm.world_size, Ci)
        by_user.cols = _slot_pos(by_user.cols, nI, comm.world_size, Li).to(torch.int32)
        by_item.cols = _slot_pos(by_item.cols, nU, comm.world_size, Ls).to(torch.int32)
        Xf = torch.zeros((Cu * comm.world_size * Ls, rank), dtype=X.dtype, device=dev)
        Yf = torch.zeros((Ci * comm.world_size * Li, rank), dtype=Y.dtype, device=dev)
        _gather_slots(comm, Y, Yf, Li, None)
    for it in range(start, max_iter):
        progress.iteration(it, max_iter)
        with trace("als.iter"):
            ti = time.time()
            if not chunked:
                Yf = comm.all_gather_v(Y) if comm.world_size > 1 else Y
            YtY = None
            if implicit:
                YtY = gram(Y)
                comm.all_reduce(YtY)
                YtY = YtY.float()
            if chunked:
                _gather_slots(comm, X, Xf, Ls, lambda a, e: solve_side(
                    by_user, Yf, X, reg, implicit, alpha, YtY, cg_iters, nonneg, exact, row_range=(a, e),
                    eig_basis=eigmode))
            else:
                X = solve_side(by_user, Yf, X, reg, implicit, alpha, YtY, cg_iters, nonneg, exact,
                               eig_basis=eigmode)
            if eigmode:                  # X now holds X (B Q): the basis moves on by Q
                q = A.EIG_CACHE.get(Yf, YtY, True, shared=True)[1].double().cpu()
                basis[0] = q if basis[0] is None else basis[0] @ q
            if not chunked:
                del Yf
                Xf = comm.all_gather_v(X) if comm.world_size > 1 else X
            XtX = None
            if implicit:
                XtX = gram(X)
                comm.all_reduce(XtX)
                XtX = XtX.float()
            if chunked:
                _gather_slots(comm, Y, Yf, Li, lambda a, e: solve_side(
                    by_item, Xf, Y, reg, implicit, alpha, XtX, cg_iters, nonneg, exact, row_range=(a, e)))
            else:
                Y = solve_side(by_item, Xf, Y, reg, implicit, alpha, XtX, cg_iters, nonneg, exact)
                del Xf
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            its.append(time.time() - ti)
            if ckpt is not None and ckpt.due(it + 1):
                ckpt.save(it + 1, {"X": to_orig(X).cpu().numpy(), "Y": to_orig(Y).cpu().numpy()})
    if ckpt is not None:
        ckpt.clear()                     # finished: a later fit must not resume from this run
    with trace("als.basis_restore"):
        X, Y = to_orig(X), to_orig(Y)
    Uf = comm.all_gather_v(X) if (keep_full and comm.world_size > 1) else X
    Vf = comm.all_gather_v(Y) if (keep_full and comm.world_size > 1) else Y
    A.EIG_CACHE.clear()                  # drops the rotated factor table
    A.PAD_CACHE.clear()
    return AlsResult(uid, iid, Uf, Vf, time.time() - t0, its)


_ = np
