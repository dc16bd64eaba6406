"""Bisecting k-means, Gaussian mixtures (EM), online variational LDA and power
iteration clustering over row-sharded data.

All four follow the same MI355X pattern as the other estimators: per iteration every
rank turns its rows into small sufficient statistics with GEMM-shaped torch ops on its
GPU (hipBLASLt) -- per-cluster sums, per-component ``(X*r)^T X`` Gram blocks,
``expElogtheta^T (cts/phinorm)`` topic statistics, sparse mat-vecs -- and one
all-reduce (RCCL over xGMI) combines them; the tiny model update runs replicated.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import binsum as BS
from ..ops.gram import rows_t_matmul
from ..ops import sampling
from . import kmeans as KM


def _rows(comm, n_local, device):
    return KM._global_rows(comm, n_local, device)


# =========================================================== bisecting k-means
@dataclass
class BisectingResult:
    centers: dict            # node id -> centre (np.ndarray); root = 1
    children: dict           # node id -> (left id, right id) for split nodes
    leaves: list             # leaf node ids in output (left-to-right) order
    cost: float
    sizes: list


def _summaries(comm, X, lab, nodes, D):
    """Per node in ``nodes``: (count, sum vector, sum of squared norms), all-reduced
    (one ``bin_sums`` pass: per-wave LDS bins, no global atomics)."""
    dev = X.device
    m = len(nodes)
    lut = torch.full((int(max(nodes)) + 2,), -1, dtype=torch.int64, device=dev)
    lut[torch.tensor(nodes, device=dev)] = torch.arange(m, device=dev)
    slot = torch.where(lab < lut.shape[0], lut[lab.clamp(0, lut.shape[0] - 1)], torch.full_like(lab, -1))
    st = BS.bin_sums(X, slot, m)                              # [m, D + 2]
    buf = torch.cat([st[:, D], st[:, :D].reshape(-1), st[:, D + 1]])
    comm.all_reduce(buf)
    cnt, sums, sq = buf[:m], buf[m:m + m * D].reshape(m, D), buf[m + m * D:]
    centers = sums / cnt.clamp_min(1)[:, None]
    cost = (sq - cnt * (centers * centers).sum(1)).clamp_min(0)
    return cnt.cpu().numpy(), centers.cpu().numpy(), cost.cpu().numpy()


def fit_bisecting(comm, X: torch.Tensor, k: int, max_iter: int, seed: int, min_divisible: float,
                  cosine: bool = False) -> BisectingResult:
    dev = X.device
    X = X.to(torch.float64)
    if cosine:
        X = X / X.norm(dim=1, keepdim=True).clamp_min(1e-300)
    D = X.shape[1]
    lab = torch.ones(X.shape[0], dtype=torch.int64, device=dev)       # root = 1
    n_total = float(comm.sum_scalar(X.shape[0]))
    min_size = min_divisible if min_divisible >= 1.0 else math.ceil(min_divisible * n_total)
    cnt, cen, cost = _summaries(comm, X, lab, [1], D)
    centers = {1: cen[0]}
    stats = {1: (cnt[0], cost[0])}
    leaves = [1]
    children: dict = {}
    next_id = 2
    rng = np.random.default_rng(seed)
    while len(leaves) < k:
        div = [i for i in leaves if stats[i][0] >= max(min_size, 2) and stats[i][1] > 0]
        if not div:
            break
        div.sort(key=lambda i: -stats[i][1])         # split the highest-cost clusters first
        div = div[: k - len(leaves)]
        m = len(div)
        # initial children: centre +/- a small random offset (scaled by the cluster spread)
        C2 = np.zeros((m, 2, D))
        for j, i in enumerate(div):
            c = centers[i]
            scale = 1e-4 * max(np.sqrt(stats[i][1] / max(stats[i][0], 1)), 1e-12)
            noise = rng.normal(size=D) * scale
            C2[j, 0], C2[j, 1] = c + noise, c - noise
        lut = torch.full((int(max(div)) + 2,), -1, dtype=torch.int64, device=dev)
        lut[torch.tensor(div, device=dev)] = torch.arange(m, device=dev)
        slot = torch.where(lab < lut.shape[0], lut[lab.clamp_max(lut.shape[0] - 1)], torch.full_like(lab, -1))
        act = slot >= 0
        Xa, sa = X[act], slot[act]
        side = torch.zeros_like(sa)
        for _ in range(max(1, max_iter)):
            Ct = torch.from_numpy(C2).to(dev)
            d0 = ((Xa - Ct[sa, 0]) ** 2).sum(1)
            d1 = ((Xa - Ct[sa, 1]) ** 2).sum(1)
            side = (d1 < d0).long()
            st = BS.bin_sums(Xa, sa * 2 + side, 2 * m)
            buf = torch.cat([st[:, D], st[:, :D].reshape(-1)])
            comm.all_reduce(buf)
            cnts, sums = buf[:2 * m].cpu().numpy(), buf[2 * m:].reshape(2 * m, D).cpu().numpy()
            newC = np.where(cnts[:, None] > 0, sums / np.maximum(cnts, 1)[:, None], C2.reshape(2 * m, D))
            if cosine:
                newC = newC / np.maximum(np.linalg.norm(newC, axis=1, keepdims=True), 1e-300)
            newC = newC.reshape(m, 2, D)
            done = np.allclose(newC, C2)
            C2 = newC
            if done:
                break
        ids = [(next_id + 2 * j, next_id + 2 * j + 1) for j in range(m)]
        next_id += 2 * m
        kid_tab = torch.tensor(ids, dtype=torch.int64, device=dev)          # [m, 2]
        lab[act] = kid_tab[sa, side]
        kids = [c for pair in ids for c in pair]
        cnt, cen, cost = _summaries(comm, X, lab, kids, D)
        for j, c in enumerate(kids):
            centers[c] = cen[j]
            stats[c] = (cnt[j], cost[j])
        new_leaves = []
        for j, i in enumerate(div):
            l, r = ids[j]
            if stats[l][0] > 0 and stats[r][0] > 0:
                children[i] = (l, r)
        for i in leaves:
            new_leaves.extend(children[i] if i in children and i in div else [i])
        if new_leaves == leaves:
            break
        leaves = new_leaves
    leaves = leaf_order(children)
    total = float(sum(stats[i][1] for i in leaves))
    return BisectingResult({i: centers[i] for i in _tree_nodes(children)}, children, leaves, total,
                           [int(stats[i][0]) for i in leaves])


def _tree_nodes(children: dict) -> list:
    out, stack = [], [1]
    while stack:
        i = stack.pop()
        out.append(i)
        stack.extend(children.get(i, ()))
    return out


def leaf_order(children: dict) -> list:
    """Leaves left-to-right (depth-first, left child first)."""
    out, stack = [], [1]
    while stack:
        i = stack.pop()
        if i in children:
            stack.extend(reversed(children[i]))
        else:
            out.append(i)
    return out


def bisecting_predict(X: torch.Tensor, centers: dict, children: dict, leaves: list,
                      cosine: bool = False) -> torch.Tensor:
    """Descend the tree choosing the closer child; returns the leaf's output index."""
    dev = X.device
    X = X.to(torch.float64)
    if cosine:
        X = X / X.norm(dim=1, keepdim=True).clamp_min(1e-300)
    maxn = max(centers) + 1
    Ctab = torch.zeros((maxn, X.shape[1]), dtype=torch.float64, device=dev)
    for i, c in centers.items():
        Ctab[i] = torch.from_numpy(np.asarray(c)).to(dev)
    left = torch.full((maxn,), -1, dtype=torch.int64)
    right = torch.full((maxn,), -1, dtype=torch.int64)
    for i, (l, r) in children.items():
        left[i], right[i] = l, r
    left, right = left.to(dev), right.to(dev)
    node = torch.ones(X.shape[0], dtype=torch.int64, device=dev)
    for _ in range(len(centers)):
        active = left[node] >= 0
        if not bool(active.any()):
            break
        na = node[active]
        l, r = left[na], right[na]
        dl = ((X[active] - Ctab[l]) ** 2).sum(1)
        dr = ((X[active] - Ctab[r]) ** 2).sum(1)
        node[active] = torch.where(dr < dl, r, l)
    lut = torch.full((maxn,), -1, dtype=torch.int64, device=dev)
    lut[torch.tensor(leaves, device=dev)] = torch.arange(len(leaves), device=dev)
    return lut[node]


# ================================================================ Gaussian mixture
@dataclass
class GMMResult:
    weights: np.ndarray
    means: np.ndarray
    covs: np.ndarray
    log_likelihood: float
    iterations: int
    history: list = field(default_factory=list)


def gmm_log_prob(X: torch.Tensor, means: torch.Tensor, covs: torch.Tensor, logw: torch.Tensor) -> torch.Tensor:
    """[n, K] log(w_k N(x | mu_k, Sigma_k)) via Cholesky factors."""
    n, D = X.shape
    L = torch.linalg.cholesky(covs)                                   # [K, D, D]
    # whiten with the explicit inverse factor (K tiny D x D solves): z = L^-1 x - L^-1 mu is
    # one row-parallel GEMM per component; a triangular solve against [K, D, n] right-hand
    # sides runs out of trsm workspace at millions of rows
    eye = torch.eye(D, dtype=X.dtype, device=X.device).expand_as(L)
    Linv = torch.linalg.solve_triangular(L, eye, upper=False)         # [K, D, D]
    mw = (Linv @ means[:, :, None])[:, :, 0]                          # [K, D]
    z = torch.matmul(X[None, :, :], Linv.transpose(1, 2)) - mw[:, None, :]   # [K, n, D]
    maha = (z * z).sum(2)                                             # [K, n]
    logdet = 2 * torch.log(torch.diagonal(L, dim1=1, dim2=2)).sum(1)  # [K]
    lp = -0.5 * (maha + logdet[:, None] + D * math.log(2 * math.pi))
    return (lp + logw[:, None]).T


def _psd(cov: torch.Tensor) -> torch.Tensor:
    """Symmetrise; add the smallest jitter that makes each matrix Cholesky-factorable."""
    cov = 0.5 * (cov + cov.transpose(-1, -2))
    eye = torch.eye(cov.shape[-1], dtype=cov.dtype, device=cov.device)
    jitter = 0.0
    for _ in range(12):
        _, info = torch.linalg.cholesky_ex(cov + jitter * eye)
        if int(info.max()) == 0:
            return cov + jitter * eye
        jitter = 1e-10 if jitter == 0 else jitter * 10
    return cov + jitter * eye


def fit_gmm(comm, X: torch.Tensor, k: int, max_iter: int, tol: float, seed: int, w=None,
            chunk: int = 1 << 18) -> GMMResult:
    dev = X.device
    X = X.to(torch.float64)
    n, D = X.shape
    rows, N = _rows(comm, n, dev)
    # init (Spark): k groups of 5 random samples -> group means; shared diagonal covariance
    ns = 5
    rng = np.random.default_rng(seed)
    picks = torch.from_numpy(rng.choice(max(N, 1), size=k * ns, replace=N < k * ns)).to(dev)
    S = torch.zeros((k * ns, D), dtype=torch.float64, device=dev)
    hit = torch.isin(rows, picks)
    if bool(hit.any()):
        pos = torch.searchsorted(rows[hit], picks).clamp_max(int(hit.sum()) - 1)
        found = rows[hit][pos] == picks
        S[found] = X[hit][pos[found]]
    comm.all_reduce(S)
    means = S.reshape(k, ns, D).mean(1)
    var = S.var(0, unbiased=False) if k * ns > 1 else torch.ones(D, dtype=torch.float64, device=dev)
    covs = torch.diag_embed(var.clamp_min(1e-6).expand(k, D)).clone()
    weights = torch.full((k,), 1.0 / k, dtype=torch.float64, device=dev)
    wt = None if w is None else w.to(dev, torch.float64)
    ll_prev = -math.inf
    hist = []
    it = 0
    for it in range(1, max_iter + 1):
        covs = _psd(covs)
        Nk = torch.zeros(k, dtype=torch.float64, device=dev)
        Sk = torch.zeros((k, D), dtype=torch.float64, device=dev)
        Qk = torch.zeros((k, D, D), dtype=torch.float64, device=dev)
        ll = torch.zeros((), dtype=torch.float64, device=dev)
        logw = torch.log(weights.clamp_min(1e-300))
        for a in range(0, n, chunk):
            Xc = X[a:a + chunk]
            lp = gmm_log_prob(Xc, means, covs, logw)
            lse = torch.logsumexp(lp, dim=1)
            r = torch.exp(lp - lse[:, None])
            if wt is not None:
                r = r * wt[a:a + chunk, None]
                lse = lse * wt[a:a + chunk]
            ll += lse.sum()
            Nk += r.sum(0)
            Sk += rows_t_matmul(r, Xc)
            Qk += torch.stack([rows_t_matmul(Xc * r[:, j:j + 1], Xc) for j in range(k)])
        buf = torch.cat([Nk, Sk.reshape(-1), Qk.reshape(-1), ll[None]])
        comm.all_reduce(buf)
        Nk = buf[:k]
        Sk = buf[k:k + k * D].reshape(k, D)
        Qk = buf[k + k * D:k + k * D + k * D * D].reshape(k, D, D)
        llv = float(buf[-1])
        hist.append(llv)
        tot = Nk.sum()
        weights = Nk / tot
        means = Sk / Nk.clamp_min(1e-300)[:, None]
        covs = Qk / Nk.clamp_min(1e-300)[:, None, None] - means[:, :, None] * means[:, None, :]
        if abs(llv - ll_prev) < tol:
            break
        ll_prev = llv
    covs = _psd(covs)
    return GMMResult(weights.cpu().numpy(), means.cpu().numpy(), covs.cpu().numpy(), hist[-1] if hist else 0.0,
                     it, hist)


# ================================================================ online LDA
def _dirichlet_expectation(a: torch.Tensor) -> torch.Tensor:
    return torch.digamma(a) - torch.digamma(a.sum(-1, keepdim=True))


@dataclass
class LDAState:
    lam: torch.Tensor          # [k, V] variational topic parameters
    alpha: torch.Tensor        # [k]
    eta: float
    iterations: int = 0


def lda_e_step(rows, cols, vals, ndocs, exp_elog_beta, alpha, gen, max_inner=100, tol=1e-3):
    """Per-document variational inference for a CSR/COO chunk.

    rows/cols/vals: nonzeros (doc index within chunk, term, count).  Returns (gamma
    [ndocs, k], sstats [k, V]) where sstats = expElogtheta^T (cts / phinorm) .* expElogbeta.
    """
    dev = exp_elog_beta.device
    k, V = exp_elog_beta.shape
    gamma = _gamma_sample(ndocs, k, gen).to(dev)
    Eb = exp_elog_beta[:, cols].T                                    # [nnz, k]
    for _ in range(max_inner):
        last = gamma
        Et = torch.exp(_dirichlet_expectation(gamma))                # [ndocs, k]
        phinorm = (Et[rows] * Eb).sum(1) + 1e-100                    # [nnz]
        ratio = vals / phinorm
        acc = torch.zeros((ndocs, k), dtype=torch.float64, device=dev).index_add_(0, rows, ratio[:, None] * Eb)
        gamma = alpha[None, :] + Et * acc
        if float((gamma - last).abs().mean()) < tol:
            break
    Et = torch.exp(_dirichlet_expectation(gamma))
    phinorm = (Et[rows] * Eb).sum(1) + 1e-100
    ratio = vals / phinorm
    sst = torch.zeros((V, k), dtype=torch.float64, device=dev).index_add_(0, cols, ratio[:, None] * Et[rows])
    return gamma, sst.T * exp_elog_beta


def _gamma_sample(n, k, gen):
    # Gamma(100, 1/100) via numpy (seeded, rank-count invariant when keyed per document)
    return torch.from_numpy(gen.gamma(100.0, 1.0 / 100.0, size=(n, k)))


def update_alpha(alpha: torch.Tensor, gammas: torch.Tensor, rho: float) -> torch.Tensor:
    """Newton step on the document concentration (Hoffman et al.; Spark updateAlpha)."""
    N = gammas.shape[0]
    if N == 0:
        return alpha
    logphat = _dirichlet_expectation(gammas).sum(0) / N
    gradf = N * (-torch.digamma(alpha) + torch.digamma(alpha.sum()) + logphat)
    c = N * torch.special.polygamma(1, alpha.sum())
    q = -N * torch.special.polygamma(1, alpha)
    b = (gradf / q).sum() / (1.0 / c + (1.0 / q).sum())
    dalpha = -(gradf - b) / q
    new = alpha + rho * dalpha
    return new if bool((new > 0).all()) else alpha


def lda_bound(rows, cols, vals, ndocs, state: LDAState, gen):
    """Evidence lower bound terms for a chunk (document part; topic part added by caller)."""
    Elogbeta = _dirichlet_expectation(state.lam)
    gamma, _ = lda_e_step(rows, cols, vals, ndocs, torch.exp(Elogbeta), state.alpha, gen)
    Elogtheta = _dirichlet_expectation(gamma)
    # sum_d sum_w n_dw log sum_k exp(Elogtheta_dk + Elogbeta_kw)
    t = torch.logsumexp(Elogtheta[rows] + Elogbeta[:, cols].T, dim=1)
    score = (vals * t).sum()
    a = state.alpha
    score += ((a[None, :] - gamma) * Elogtheta).sum()
    score += (torch.lgamma(gamma) - torch.lgamma(a)[None, :]).sum()
    score += (torch.lgamma(a.sum()) - torch.lgamma(gamma.sum(1))).sum()
    return score, gamma


def topic_bound(state: LDAState) -> torch.Tensor:
    lam, eta = state.lam, state.eta
    V = lam.shape[1]
    Elogbeta = _dirichlet_expectation(lam)
    s = ((eta - lam) * Elogbeta).sum()
    s += (torch.lgamma(lam) - math.lgamma(eta)).sum()
    s += (math.lgamma(eta * V) - torch.lgamma(lam.sum(1))).sum()
    return s


# =========================================================== power iteration
def power_iteration_embedding(src: torch.Tensor, dst: torch.Tensor, w: torch.Tensor, n: int, max_iter: int,
                              init: str, seed: int) -> torch.Tensor:
    """Lin & Cohen PIC: v <- D^-1 W v (L1-normalised) on the symmetric affinity graph."""
    dev = src.device
    i = torch.cat([src, dst])
    j = torch.cat([dst, src])
    v_ = torch.cat([w, w]).to(torch.float64)
    W = torch.sparse_coo_tensor(torch.stack([i, j]), v_, (n, n)).coalesce()
    deg = torch.sparse.sum(W, dim=1).to_dense()
    inv = torch.where(deg > 0, 1.0 / deg, torch.zeros_like(deg))
    if init == "degree":
        v = deg / deg.sum()
    else:
        g = np.random.default_rng(seed)
        v = torch.from_numpy(g.random(n)).to(dev)
        v = v / v.sum()
    prev_delta = math.inf
    tol = 1e-5 / max(n, 1)
    for _ in range(max_iter):
        nv = inv * torch.sparse.mm(W, v[:, None])[:, 0]
        nv = nv / nv.abs().sum().clamp_min(1e-300)
        delta = float((nv - v).abs().sum())
        v = nv
        if abs(delta - prev_delta) < tol:
            break
        prev_delta = delta
    return v


_ = sampling
