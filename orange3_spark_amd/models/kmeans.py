"""KMeans engine: k-means|| initialisation + Lloyd iterations over row-sharded data.

Per Lloyd iteration on each rank: ``kmeans_assign`` (MFMA GEMM + fused argmin) ->
``kmeans_update`` (sorted segmented sums into block slabs) -> ONE all-reduce of a
single fp64 buffer [sums (K*D) | counts (K) | cost] over RCCL.  Spark semantics
(mllib KMeans): empty clusters keep their previous centre; converged when every centre
moved less than ``tol`` (euclidean); cost = sum of squared distances.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import kmeans as K
from ..ops import sampling
from ..runtime.tracing import trace
from ..runtime import progress


@dataclass
class KMeansResult:
    centers: torch.Tensor          # [k, D] fp64 (host)
    cost: float
    iterations: int
    sizes: list
    history: list = field(default_factory=list)
    seconds: float = 0.0


def _centred_moments(comm, X: torch.Tensor):
    """(global mean row m fp64, this rank's sum ||x - m||^2) in ONE pass over X: the rows'
    sums are taken about a shift s (rank 0's first row, shared), then
    sum ||x - m||^2 = sum ||x - s||^2 - 2 (m - s).sum (x - s) + n ||m - s||^2 exactly, with
    m - s small -- no cancellation for data far from the origin."""
    D = X.shape[1]
    s = torch.zeros(D + 1, dtype=torch.float64, device=X.device)
    if comm.rank == 0 and X.shape[0]:
        s[:D] = X[0].to(torch.float64)
        s[D] = 1.0
    comm.all_reduce(s)                   # rank 0's row (or zeros when it has no rows)
    shift = s[:D].float()                # an fp32 row: exactly the kernel's shift
    s1, s2 = K.moments(X, shift)
    buf = torch.cat([s1, torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device)])
    comm.all_reduce(buf)
    n = buf[D].clamp_min(1.0)
    ms = buf[:D] / n                     # m - s
    local = s2 - 2.0 * (ms * s1).sum() + float(X.shape[0]) * (ms * ms).sum()
    return shift.to(torch.float64) + ms, local


def _global_rows(comm, n_local, device):
    sizes = comm.all_gather_object(int(n_local))
    off = sum(sizes[: comm.rank])
    return torch.arange(off, off + n_local, dtype=torch.int64, device=device), sum(sizes)


def kmeans_parallel_init(comm, X: torch.Tensor, k: int, steps: int, seed: int) -> torch.Tensor:
    """k-means|| (Bahmani et al.): oversample ~2k candidates per round, then weighted
    k-means++ on the (small) candidate set, replicated on every rank."""
    dev = X.device
    rows, n = _global_rows(comm, X.shape[0], dev)
    # first centre: one uniformly random global row
    rng = np.random.default_rng(seed)
    pick = int(rng.integers(0, max(n, 1)))
    mine = (rows == pick).nonzero()
    c0 = X[mine[0, 0]].to(torch.float64) if mine.numel() else torch.zeros(X.shape[1], dtype=torch.float64, device=dev)
    c0 = c0.contiguous()
    comm.all_reduce(c0)
    centers = c0[None, :]
    last = None                        # (labels, distances) of the last round's assign
    n_before = 0                       # candidates the last round assigned against
    for step in range(steps):
        with trace("kmeans.init.round"):
            a, d = K.assign(X, centers.float(), mode="approx")
            cost = torch.sum(d, dtype=torch.float64)        # no fp64 copy of d
            comm.all_reduce(cost)
            if float(cost) <= 0:
                break
            last, n_before = (a, d), centers.shape[0]
            p = (d * (2.0 * k / float(cost))).clamp_(max=1.0)
            u = sampling.uniform(rows, seed + 1 + step, stream=7)
            new = X[u < p].to(torch.float64)
            del p, u
            new = comm.all_gather_v(new) if comm.world_size > 1 else new
            centers = torch.cat([centers, new.to(dev)])
    # weights = number of points closest to each candidate.  The last round already holds
    # every row's nearest candidate among the first n_before: only the candidates that
    # round added are assigned now, and a row moves to one of them only if it is strictly
    # nearer (ties keep the lower index, as one argmin over all candidates would)
    with trace("kmeans.init.weights"):
        if last is not None and centers.shape[0] > n_before:
            a_old, d_old = last
            a_new, d_new = K.assign(X, centers[n_before:].float(), mode="approx")
            a = torch.where(d_new < d_old, a_new.to(torch.int64) + n_before, a_old.to(torch.int64))
            del a_new, d_new
        elif last is not None:
            a = last[0].to(torch.int64)
        else:
            a, _ = K.assign(X, centers.float(), mode="approx")
        del last
        # integer histogram (LDS-privatised): an fp64 index_add_ of ones into a few hundred
        # candidates serialises on global atomics
        wts = torch.bincount(a.long(), minlength=centers.shape[0])[: centers.shape[0]].to(torch.float64)
        comm.all_reduce(wts)
    with trace("kmeans.init.local"):
        return _local_kmeanspp(centers, wts, k, seed)


# greedy k-means++ (best of 2 + ln k draws per step, scikit-learn's variant).  False: one
# draw per step, as Spark's LocalKMeans.kMeansPlusPlus -- on the 100M x 128, k = 1024
# blobs its seeding leaves a 1.9x higher cost after 10 Lloyd iterations (25.0e9 vs
# 13.3e9, profiles/kmeans_init_phases_r5.json), so the greedy variant is the default
GREEDY_KMEANSPP = True


def _local_kmeanspp(P: torch.Tensor, w: torch.Tensor, k: int, seed: int, iters: int = 30,
                    kernel: bool = True) -> torch.Tensor:
    """Weighted k-means++ + Lloyd on candidates (Spark LocalKMeans), fp64 on device.

    Greedy k-means++ (best of ``2 + ln k`` weighted draws per step; ``GREEDY_KMEANSPP =
    False``: one draw per step, as Spark's LocalKMeans).  The whole seeding
    loop stays on the device -- draws are counter-hash uniforms keyed on (seed, step,
    trial) inverted through the cumulative weights by ``searchsorted`` -- so its k
    sequential steps issue kernels without a single host round trip (the host-side
    multinomial per step cost two syncs each: ~2 s of a 3 s fit at k = 1024)."""
    m = P.shape[0]
    dev = P.device
    if m <= k:
        extra = k - m
        return torch.cat([P, P[:1].expand(extra, -1)]) if extra else P
    trials = 2 + int(math.log(k)) if GREEDY_KMEANSPP else 1
    keys = torch.arange(k * (trials + 1), dtype=torch.int64, device=dev).view(k, trials + 1)
    U = sampling.uniform(keys.reshape(-1), seed, stream=31).view(k, trials + 1)

    def draw(t, prob, n):
        cs = torch.cumsum(prob, 0)
        tot = cs[-1]
        u = U[t, :n] * tot
        idx = torch.searchsorted(cs, u, right=True).clamp_max(m - 1)
        rnd = (U[t, :n] * m).long().clamp_max(m - 1)
        return torch.where(tot > 0, idx, rnd)

    # the seeding distances use fp32-rounded coordinates (products and sums in fp64) on both
    # paths: the kernel then streams half the bytes and keeps the candidates L2-resident;
    # the centres themselves are the fp64 candidates
    Pr = P.float().double()
    pn = (Pr * Pr).sum(1)
    with trace("kmeans.init.local.seed"):
        if kernel and P.is_cuda and trials <= 16 and trials * P.shape[1] * 8 <= 64 * 1024:
            # the k greedy steps as 2 launches each (kpp_dist_kernel over every candidate row,
            # kpp_pick_kernel in one block): no host round trip inside the loop
            from ..ops import _native as N
            wc, pc = w.to(torch.float64).contiguous(), pn.contiguous()
            PT = P.float().t().contiguous()           # fp32 [D][m]: coalesced candidate reads
            Uc = U.contiguous()
            d2 = torch.empty(m, dtype=torch.float64, device=dev)
            cs = torch.empty(m, dtype=torch.float64, device=dev)
            cd = torch.empty((trials, m), dtype=torch.float64, device=dev)
            partial = torch.empty((-(-m // 256), 16), dtype=torch.float64, device=dev)
            cand = torch.empty(16, dtype=torch.int32, device=dev)
            picks32 = torch.empty(k, dtype=torch.int32, device=dev)
            N.check(N.kernels().o3s_kmeanspp(PT.data_ptr(), wc.data_ptr(), pc.data_ptr(), m, P.shape[1], k, trials,
                                             Uc.data_ptr(), d2.data_ptr(), cs.data_ptr(), cd.data_ptr(),
                                             partial.data_ptr(), cand.data_ptr(), picks32.data_ptr(), N.stream_of(PT)),
                    "kmeanspp")
            picks = picks32.to(torch.int64)
        else:
            first = draw(0, w, 1)[0]
            picks = torch.empty(k, dtype=torch.int64, device=dev)
            picks[0] = first
            d2 = ((Pr - Pr[first]) ** 2).sum(1)
            for t in range(1, k):
                cand = draw(t, w * d2, trials)
                # [trials, m] squared distances as |p|^2 + |c|^2 - 2 c.p: one small fp64 GEMM
                # instead of a [trials, m, D] difference tensor per step
                cd = (pn[None, :] + pn[cand][:, None] - 2.0 * (Pr[cand] @ Pr.T)).clamp_min_(0.0)
                pot = (w[None, :] * torch.minimum(d2[None, :], cd)).sum(1)
                best = pot.argmin()
                picks[t] = cand[best]
                d2 = torch.minimum(d2, cd[best])
        C = P[picks]
    with trace("kmeans.init.local.lloyd"):
        return _local_lloyd(P, w, C, k, iters)


def _local_lloyd(P, w, C, k, iters):
    # GPU: the candidates are assigned by the split-precision assign kernel (fp32-exact
    # argmin, no GEMM library call: a process's first hipBLASLt call cost ~0.1 s of a cold
    # fit, profiles/kmeans_init_phases_r5.json); elsewhere the fp64 distance GEMM
    Pf = P.float().contiguous() if P.is_cuda else None
    use_kernel = Pf is not None and K.kernel_ok(Pf)
    for _ in range(iters):
        if use_kernel:
            a = K.assign(Pf, C.float(), mode="split", need_dist=False)[0].long()
        else:
            dist = (P * P).sum(1, keepdim=True) - 2 * P @ C.T + (C * C).sum(1)[None, :]
            a = dist.argmin(1)
        sums = torch.zeros_like(C).index_add_(0, a, P * w[:, None])
        cnt = torch.zeros(k, dtype=P.dtype, device=P.device).index_add_(0, a, w)
        newC = torch.where(cnt[:, None] > 0, sums / cnt.clamp_min(1e-300)[:, None], C)
        if torch.allclose(newC, C):
            break
        C = newC
    return C


def random_init(comm, X, k, seed):
    rows, n = _global_rows(comm, X.shape[0], X.device)
    rng = np.random.default_rng(seed)
    picks = torch.from_numpy(rng.choice(max(n, 1), size=min(k, n), replace=False)).to(X.device)
    C = torch.zeros((k, X.shape[1]), dtype=torch.float64, device=X.device)
    hit = torch.isin(rows, picks)
    for r_, x in zip(rows[hit].tolist(), X[hit].to(torch.float64)):
        C[(picks == r_).nonzero()[0, 0]] = x
    comm.all_reduce(C)
    return C


# ------------------------------------------------------------------ streamed rows
def _blocks_init(comm, B, k: int, steps: int, seed: int, init: str) -> torch.Tensor:
    """k-means|| / random initialisation over RowBlocks (resident + host-streamed rows):
    the same draws as the resident path (keyed on global rows), one streamed pass per
    round."""
    dev = B.device
    rows_all, n = _global_rows(comm, B.n, dev)
    off = int(rows_all[0]) if B.n else 0
    rng = np.random.default_rng(seed)
    if init == "random":
        picks = rng.choice(max(n, 1), size=min(k, n), replace=False)
        C = torch.zeros((k, B.D), dtype=torch.float64, device=dev)
        for j, r in enumerate(picks.tolist()):
            if off <= r < off + B.n:
                C[j] = B.rows(torch.tensor([r - off], device=dev))[0].to(torch.float64)
        comm.all_reduce(C)
        return C
    pick = int(rng.integers(0, max(n, 1)))
    c0 = torch.zeros(B.D, dtype=torch.float64, device=dev)
    if off <= pick < off + B.n:
        c0 = B.rows(torch.tensor([pick - off], device=dev))[0].to(torch.float64).contiguous()
    comm.all_reduce(c0)
    centers = c0[None, :]
    for step in range(steps):
        with trace("kmeans.init.round"):
            d = torch.empty(B.n, dtype=torch.float32, device=dev)
            Cf = centers.float()
            B.run(lambda X, a: d[a:a + X.shape[0]].copy_(K.assign(X, Cf, mode="split")[1]))
            cost = d.to(torch.float64).sum()
            comm.all_reduce(cost)
            if float(cost) <= 0:
                break
            p = (2.0 * k * d.to(torch.float64) / float(cost)).clamp(max=1.0)
            u = sampling.uniform(rows_all, seed + 1 + step, stream=7)
            sel = torch.nonzero(u < p).reshape(-1)
            new = B.rows(sel).to(torch.float64) if sel.numel() else torch.zeros((0, B.D), dtype=torch.float64,
                                                                               device=dev)
            new = comm.all_gather_v(new) if comm.world_size > 1 else new
            centers = torch.cat([centers, new.to(dev)])
    with trace("kmeans.init.weights"):
        wts = torch.zeros(centers.shape[0], dtype=torch.float64, device=dev)
        Cf = centers.float()

        def wfn(X, a):
            lab, _ = K.assign(X, Cf, mode="split")
            wts.add_(torch.bincount(lab.long(), minlength=centers.shape[0])[: centers.shape[0]].to(torch.float64))
        B.run(wfn)
        comm.all_reduce(wts)
    with trace("kmeans.init.local"):
        return _local_kmeanspp(centers, wts, k, seed)


def _fit_kmeans_blocks(comm, B, k, max_iter, tol, seed, init, init_steps, initial, cosine, ckpt) -> KMeansResult:
    """Lloyd iterations over RowBlocks: every block is assigned (split-precision kernel: no
    per-chunk host sync) and folded into the slab update; the host-streamed chunks' H2D
    copies overlap the previous chunk's kernels (frame/spill.HostStreamer)."""
    t0 = time.time()
    dev, D = B.device, B.D
    C = initial.to(dev, torch.float64) if initial is not None else _blocks_init(comm, B, k, init_steps, seed, init)
    Kp = ((k + 31) // 32) * 32
    ws = K.UpdateWorkspace(dev, Kp, D) if dev.type == "cuda" and D <= 256 else None
    hist, sizes, it = [], None, 0
    for it in range(1, max_iter + 1):
        progress.iteration(it - 1, max_iter)
        with trace("kmeans.iter"):
            Cf = C.float()
            prep = K.prepare_centers(Cf) if dev.type == "cuda" else None
            sums = torch.zeros((k, D), dtype=torch.float64, device=dev)
            cnt = torch.zeros(k, dtype=torch.float64, device=dev)
            cost = torch.zeros(1, dtype=torch.float64, device=dev)

            def step(X, a0):
                lab, d = K.assign(X, Cf, prep, mode="split")
                if ws is not None and K.update_kernel_ok(X):
                    s_, c_ = K.update(X, lab, ws.K, ws)
                    sums.add_(s_[:k])
                    cnt.add_(c_[:k])
                else:
                    s_, c_ = K.update_torch(X, lab, k)
                    sums.add_(s_)
                    cnt.add_(c_)
                cost.add_(d.to(torch.float64).sum())
            B.run(step)
            buf = torch.cat([sums.reshape(-1), cnt, cost])
            comm.all_reduce(buf)
            sums, cnt, c = buf[: k * D].reshape(k, D), buf[k * D: k * D + k], float(buf[-1])
            hist.append(c)
            newC = torch.where(cnt[:, None] > 0, sums / cnt.clamp_min(1e-300)[:, None], C)
            if cosine:
                newC = newC / newC.norm(dim=1, keepdim=True).clamp_min(1e-300)
            moved = ((newC - C) ** 2).sum(1).max().item()
            C = newC
            sizes = cnt
            if moved <= tol * tol:
                break
    cnt = torch.zeros(k, dtype=torch.float64, device=dev)
    cost = torch.zeros(1, dtype=torch.float64, device=dev)
    Cf = C.float()

    def final(X, a0):
        lab, d = K.assign(X, Cf, mode="split")
        cnt.add_(torch.bincount(lab.long(), minlength=k)[:k].to(torch.float64))
        cost.add_(d.to(torch.float64).sum())
    B.run(final)
    buf = torch.cat([cnt, cost])
    comm.all_reduce(buf)
    _ = sizes
    return KMeansResult(C.cpu(), float(buf[-1]), it, [int(x) for x in buf[:k].tolist()], hist, time.time() - t0)


HAMERLY = True                 # False: every Lloyd iteration screens every row (reference path)
HAMERLY_FULL_FRACTION = 0.5    # more rows than this to recheck: screen them all (contiguous)
LAST_HAMERLY_STATS: list = []  # per iteration: rows screened / changed (diagnostics)


def _hamerly_step(X, C, prep, ws, k, hs, sums=True):
    """One Lloyd assignment + cluster-sum step with Hamerly bounds (state ``hs`` carried
    across iterations): returns this rank's (sums fp64 [k, D], counts fp64 [k], stats).
    ``sums=False`` (the final assignment): counts only, sums None -- the state is then
    spent."""
    n = X.shape[0]
    dev = X.device
    full = hs["a"] is None
    rows = None
    need = None
    if not full:
        # centre shifts (fp64, rounded up to a safe fp32)
        delta = (C.to(torch.float64) - hs["C"].to(torch.float64)).pow(2).sum(1).sqrt()
        delta = (delta * (1 + 1e-6) + 1e-30).float()
        dmax = float(delta.max()) * (1 + 1e-6)
        need, rows = K.bounds_recheck(hs["a"], hs["bnd"], delta, dmax, int(HAMERLY_FULL_FRACTION * n))
        full = rows is None
    if full:
        a = torch.empty(n, dtype=torch.int32, device=dev) if hs["a"] is None else hs["a"]
        bnd = torch.empty((n, 2), dtype=torch.float32, device=dev) if hs["bnd"] is None else hs["bnd"]
        K.assign_bounded(X, prep, a, bnd, None)
        if not sums:
            cnt = torch.bincount(a.long(), minlength=k)[:k].to(torch.float64)
            hs.update(a=a, bnd=bnd)
            return None, cnt, {"screened": n}
        S, cnt = K.update(X, a, ws.K, ws)
        S, cnt = S[:k].clone(), cnt[:k].clone()
        st = {"screened": n, "changed": None, "recheck": None if hs["a"] is None else need}
    else:
        a, bnd = hs["a"], hs["bnd"]
        a_old = a[rows.long()].clone()
        K.assign_bounded(X, prep, a, bnd, rows)
        a_new = a[rows.long()]
        ch = rows[a_new != a_old]
        S, cnt = hs["S"], hs["n"]
        if not sums:
            moved = a_new != a_old
            cnt = cnt.clone()
            cnt.index_add_(0, a_new[moved].long(), torch.ones(int(moved.sum()), dtype=cnt.dtype, device=dev))
            cnt.index_add_(0, a_old[moved].long(), -torch.ones(int(moved.sum()), dtype=cnt.dtype, device=dev))
            hs.update(a=a, bnd=bnd)
            return None, cnt, {"screened": int(rows.numel()), "changed": int(ch.numel())}
        if ch.numel():
            Xc = X[ch.long()]
            # a grid sized to the changed rows (every block zeroes and sums a [Kp, D] slab)
            sub = hs.get("ws_sub")
            g = int(max(1, min(ws.grid, -(-ch.numel() // 16384))))
            if sub is None or sub.grid != g:
                sub = hs["ws_sub"] = K.UpdateWorkspace(dev, ws.K, X.shape[1], grid=g)
            s1, c1 = K.update(Xc, a_new[a_new != a_old].contiguous(), ws.K, sub)
            s1, c1 = s1[:k].clone(), c1[:k].clone()
            s0, c0 = K.update(Xc, a_old[a_new != a_old].contiguous(), ws.K, sub)
            S = S + (s1 - s0[:k])
            cnt = cnt + (c1 - c0[:k])
        st = {"screened": int(rows.numel()), "changed": int(ch.numel())}
    hs.update(a=a, bnd=bnd, S=S, n=cnt, C=C.clone())
    return S, cnt, st


def fit_kmeans(comm, X, k: int, max_iter: int = 20, tol: float = 1e-4, seed: int = 0,
               init: str = "k-means||", init_steps: int = 2, initial: torch.Tensor | None = None,
               weights: torch.Tensor | None = None, cosine: bool = False, ckpt=None) -> KMeansResult:
    """``X``: this rank's [n, D] rows, or a ``frame.spill.RowBlocks`` (MEMORY_AND_DISK rows:
    resident + host-streamed; unweighted)."""
    from ..frame.spill import RowBlocks
    if isinstance(X, RowBlocks):
        if weights is not None:
            raise ValueError("weighted KMeans over host-streamed rows is not supported; persist with MEMORY_ONLY")
        return _fit_kmeans_blocks(comm, X, k, max_iter, tol, seed, init, init_steps, initial, cosine, ckpt)
    try:
        return _fit_kmeans_rows(comm, X, k, max_iter, tol, seed, init, init_steps, initial, weights, cosine, ckpt)
    finally:
        # also when the fit stops early (FitCancelled from a progress report, a device
        # error): the split copy of X is as large as X and must not outlive the fit
        K.clear_presplit()


def _fit_kmeans_rows(comm, X, k, max_iter, tol, seed, init, init_steps, initial, weights, cosine, ckpt):
    t0 = time.time()
    if cosine:
        X = X / X.norm(dim=1, keepdim=True).clamp_min(1e-300)
    last = ckpt.latest() if ckpt is not None else None
    if last is not None and tuple(last[1]["C"].shape) != (k, X.shape[1]):
        last = None                      # incompatible state: start afresh
    if last is not None:
        C = None                         # resumed below; skip the initialisation passes
    elif initial is not None:
        C = initial.to(X.device, torch.float64)
    elif init == "random":
        C = random_init(comm, X, k, seed)
    else:
        C = kmeans_parallel_init(comm, X, k, init_steps, seed)
    D = X.shape[1]
    # the update kernel has its own gate (D <= 256, any D % 4) -- wider than the assign
    # kernel's register-bound one, so e.g. D = 200 still gets the slab update
    ws = K.UpdateWorkspace(X.device, ((k + 31) // 32) * 32, D) if K.update_kernel_ok(X) and weights is None else None
    hist = []
    it = start = 0
    if last is not None:                 # resume from the last saved centres
        start, st, _ = last
        C = torch.from_numpy(st["C"]).to(X.device, torch.float64)
        hist = [float(v) for v in st["hist"]]
    sizes = None
    cost = float("nan")
    # unweighted: an iteration's cost comes from its cluster sums S_a and counts n_a,
    #   sum_x ||x - c_a(x)||^2 = sum_x ||x'||^2 - sum_a (2 c'_a.S'_a - n_a ||c'_a||^2)
    # (fp64, every point and centre taken relative to the global mean m: x' = x - m,
    # S'_a = S_a - n_a m -- about the origin the identity cancels catastrophically for data
    # far from 0), so the assign pass needs no per-row distance (the screen kernel then
    # skips the exact-distance epilogue and half of its row reads)
    if weights is None:
        mean, sumsq = _centred_moments(comm, X)
    else:
        mean = sumsq = None
    # Hamerly bounds (unweighted, screen kernel): per row an upper bound on the distance to
    # its centre and a lower bound on the distance to every other one; after the centres
    # move by delta, ub += delta[a] and lb -= max delta, and only rows with ub >= lb are
    # screened again -- the others provably keep their centre (exact Lloyd, not an
    # approximation).  The cluster sums are then updated by the rows that changed centre
    # (fp64 running sums, deterministic slab kernel on the changed rows).
    ham = (HAMERLY and weights is None and ws is not None and K.screen_ok(X) and X.shape[0] > 0
           and not cosine)
    hs = {"a": None, "bnd": None, "S": None, "n": None, "C": None, "ws_sub": None}
    stats_it = []
    for it in range(start + 1, max_iter + 1):
        progress.iteration(it - 1, max_iter)
        with trace("kmeans.iter"):
            prep = K.prepare_centers(C.float()) if K.kernel_ok(X) else None
            if ham:
                sums, cnt, st_ = _hamerly_step(X, C, prep, ws, k, hs)
                stats_it.append(st_)
            else:
                a, d = K.assign(X, C.float(), prep, need_dist=weights is not None)
                if ws is not None:
                    sums, cnt = K.update(X, a, ws.K, ws)
                    sums, cnt = sums[:k], cnt[:k]
                else:
                    sums, cnt = K.update_torch(X, a, k, weights)
            if weights is None:
                Cd = C.to(sums.device, torch.float64) - mean
                Sd = sums.to(torch.float64) - cnt.to(torch.float64)[:, None] * mean
                local = sumsq - (2.0 * (Cd * Sd).sum() - (cnt * (Cd * Cd).sum(1)).sum())
            else:
                local = (d.to(torch.float64) * weights.to(torch.float64)).sum()
            buf = torch.cat([sums.reshape(-1), cnt, local.reshape(1)])
            comm.all_reduce(buf)
            sums, cnt, cost = buf[: k * D].reshape(k, D), buf[k * D: k * D + k], max(0.0, float(buf[-1]))
            hist.append(cost)
            newC = torch.where(cnt[:, None] > 0, sums / cnt.clamp_min(1e-300)[:, None], C)
            if cosine:
                newC = newC / newC.norm(dim=1, keepdim=True).clamp_min(1e-300)
            moved = ((newC - C) ** 2).sum(1).max().item()
            C = newC
            sizes = cnt
            if ckpt is not None and ckpt.due(it):
                ckpt.save(it, {"C": C.cpu().numpy(), "hist": np.asarray(hist)})
            if moved <= tol * tol:
                break
    LAST_HAMERLY_STATS[:] = stats_it
    if ckpt is not None:
        ckpt.clear()                     # finished: a later fit must not resume from this run
    # final cost/sizes w.r.t. the returned centres (Spark reports the last assignment's)
    if ham:
        # one more bounded step: only the rows whose bounds no longer certify their centre
        # are screened (the sizes follow the rows that moved), then the cost straight from
        # the rows and their centres in one streaming pass -- per-row distances, not the
        # loop's cluster-sum identity (whose fp32 slab sums cost it ~1e-6 relative when the
        # clusters are tight), and no full screen
        with trace("kmeans.final"):
            _, cnt, _ = _hamerly_step(X, C, K.prepare_centers(C.float()), ws, k, hs, sums=False)
            local = K.cost(X, hs["a"], C.float())
            buf = torch.cat([cnt.to(torch.float64), local.reshape(1)])
            comm.all_reduce(buf)
            cost = float(buf[-1])
        return KMeansResult(C.cpu(), cost, it, [int(round(x)) for x in buf[:k].tolist()], hist, time.time() - t0)
    a, d = K.assign(X, C.float())
    cnt = torch.bincount(a.long(), minlength=k)[:k].to(torch.float64)
    buf = torch.cat([cnt, d.to(torch.float64).sum().reshape(1)])
    comm.all_reduce(buf)
    return KMeansResult(C.cpu(), float(buf[-1]), it, [int(x) for x in buf[:k].tolist()], hist, time.time() - t0)


def predict(X: torch.Tensor, C: torch.Tensor, cosine=False) -> torch.Tensor:
    if cosine:
        X = X / X.norm(dim=1, keepdim=True).clamp_min(1e-300)
    a, _ = K.assign(X.float() if X.is_cuda else X, C.to(X.device).float() if X.is_cuda else C.to(X.device))
    K.clear_presplit()                   # one-shot transform: do not keep the split copy of X
    return a


_ = math
