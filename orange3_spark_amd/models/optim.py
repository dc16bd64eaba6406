"""Host-side first-order optimisers over small (D <= a few thousand) fp64 vectors.

The expensive part of every iteration -- one pass over the sharded rows -- happens in
the device kernels plus an RCCL all-reduce; what remains is O(D) vector algebra that
is cheaper on the host than a chain of tiny kernels.  Mirrors Breeze's LBFGS/OWLQN as
used by Spark ML (StrongWolfe line search, m = 10 corrections, relative function-value
and gradient-norm convergence).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable

import numpy as np

from ..runtime import progress

Fn = Callable[[np.ndarray], tuple[float, np.ndarray]]


@dataclass
class OptimResult:
    x: np.ndarray
    f: float
    iterations: int
    history: list = field(default_factory=list)
    converged: bool = False
    reason: str = ""


def _strong_wolfe(fg: Fn, x, f0, g0, d, t0=1.0, c1=1e-4, c2=0.9, max_evals=20):
    """Strong-Wolfe line search (bracketing + cubic/bisection zoom)."""
    dg0 = float(g0 @ d)
    if dg0 >= 0:
        return None
    t_prev, f_prev, dg_prev = 0.0, f0, dg0
    t = t0
    evals = 0
    best = (0.0, f0, g0)
    lo = hi = None
    while evals < max_evals:
        f, g = fg(x + t * d)
        evals += 1
        dg = float(g @ d)
        if np.isfinite(f) and f < best[1]:
            best = (t, f, g)
        if not np.isfinite(f) or f > f0 + c1 * t * dg0 or (evals > 1 and f >= f_prev):
            lo, hi = (t_prev, f_prev, dg_prev), (t, f, dg)
            break
        if abs(dg) <= -c2 * dg0:
            return t, f, g
        if dg >= 0:
            lo, hi = (t, f, dg), (t_prev, f_prev, dg_prev)
            break
        t_prev, f_prev, dg_prev = t, f, dg
        t *= 2.0
    if lo is None:
        return best if best[0] > 0 else None
    # zoom
    while evals < max_evals:
        (ta, fa, da), (tb, fb, db) = lo, hi
        t = _cubic_min(ta, fa, da, tb, fb, db)
        lo_t, hi_t = min(ta, tb), max(ta, tb)
        if not (lo_t + 0.1 * (hi_t - lo_t) <= t <= hi_t - 0.1 * (hi_t - lo_t)):
            t = 0.5 * (ta + tb)
        f, g = fg(x + t * d)
        evals += 1
        dg = float(g @ d)
        if np.isfinite(f) and f < best[1]:
            best = (t, f, g)
        if not np.isfinite(f) or f > f0 + c1 * t * dg0 or f >= fa:
            hi = (t, f, dg)
        else:
            if abs(dg) <= -c2 * dg0:
                return t, f, g
            if dg * (tb - ta) >= 0:
                hi = lo
            lo = (t, f, dg)
        if abs(hi[0] - lo[0]) < 1e-12:
            break
    return best if best[0] > 0 else None


def _cubic_min(a, fa, da, b, fb, db):
    d1 = da + db - 3 * (fa - fb) / (a - b) if a != b else 0.0
    sq = d1 * d1 - da * db
    if sq < 0 or a == b:
        return 0.5 * (a + b)
    d2 = np.sign(b - a) * np.sqrt(sq)
    den = db - da + 2 * d2
    if den == 0:
        return 0.5 * (a + b)
    return b - (b - a) * (db + d2 - d1) / den


def lbfgs(fg: Fn, x0: np.ndarray, max_iter: int = 100, tol: float = 1e-6, m: int = 10,
          callback=None) -> OptimResult:
    x = np.array(x0, dtype=np.float64)
    f, g = fg(x)
    hist = [f]
    S, Y = [], []
    res = OptimResult(x, f, 0, hist)
    for it in range(1, max_iter + 1):
        progress.iteration(it - 1, max_iter)
        # two-loop recursion
        q = g.copy()
        alphas = []
        for s, y in reversed(list(zip(S, Y))):
            rho = 1.0 / float(y @ s)
            a = rho * float(s @ q)
            alphas.append((a, rho, s, y))
            q -= a * y
        if S:
            gamma = float(S[-1] @ Y[-1]) / float(Y[-1] @ Y[-1])
            q *= gamma
        for a, rho, s, y in reversed(alphas):
            b = rho * float(y @ q)
            q += (a - b) * s
        d = -q
        t0 = 1.0 if S else min(1.0, 1.0 / max(np.linalg.norm(g), 1e-12))
        ls = _strong_wolfe(fg, x, f, g, d, t0)
        if ls is None:
            res.reason = "line search failed"
            break
        t, fn, gn = ls
        s, y = t * d, gn - g
        if float(s @ y) > 1e-10 * float(y @ y):
            S.append(s)
            Y.append(y)
            if len(S) > m:
                S.pop(0)
                Y.pop(0)
        x = x + s
        rel = abs(f - fn) / max(abs(fn), abs(f), 1e-12)
        f, g = fn, gn
        hist.append(f)
        res.iterations = it
        if callback:
            callback(it, x, f)
        if rel < tol:
            res.converged, res.reason = True, "function values converged"
            break
        if np.linalg.norm(g) <= tol * max(1.0, abs(f)):
            res.converged, res.reason = True, "gradient converged"
            break
    res.x, res.f, res.history = x, f, hist
    if not res.reason:
        res.reason = "max iterations reached"
    return res


def owlqn(fg: Fn, x0: np.ndarray, l1: np.ndarray, max_iter: int = 100, tol: float = 1e-6, m: int = 10,
          callback=None) -> OptimResult:
    """Orthant-wise limited-memory quasi-Newton (Andrew & Gao 2007) for f(x) + sum l1_j |x_j|."""
    x = np.array(x0, dtype=np.float64)
    l1 = np.asarray(l1, dtype=np.float64)

    def total(xv, fv):
        return fv + float(np.sum(l1 * np.abs(xv)))

    def pseudo_grad(xv, gv):
        pg = gv.copy()
        pos, neg, zero = xv > 0, xv < 0, xv == 0
        pg[pos] += l1[pos]
        pg[neg] -= l1[neg]
        gp, gm = gv[zero] + l1[zero], gv[zero] - l1[zero]
        pz = np.where(gm > 0, gm, np.where(gp < 0, gp, 0.0))
        pg[zero] = pz
        return pg

    f, g = fg(x)
    F = total(x, f)
    hist = [F]
    S, Y = [], []
    res = OptimResult(x, F, 0, hist)
    for it in range(1, max_iter + 1):
        progress.iteration(it - 1, max_iter)
        pg = pseudo_grad(x, g)
        q = pg.copy()
        alphas = []
        for s, y in reversed(list(zip(S, Y))):
            rho = 1.0 / float(y @ s)
            a = rho * float(s @ q)
            alphas.append((a, rho, s, y))
            q -= a * y
        if S:
            q *= float(S[-1] @ Y[-1]) / float(Y[-1] @ Y[-1])
        for a, rho, s, y in reversed(alphas):
            b = rho * float(y @ q)
            q += (a - b) * s
        d = -q
        d[d * pg >= 0] = 0.0  # constrain to descent on pseudo-gradient
        if not np.any(d):
            res.converged, res.reason = True, "zero direction"
            break
        orthant = np.where(x != 0, np.sign(x), np.sign(-pg))
        t = 1.0 if S else min(1.0, 1.0 / max(np.linalg.norm(pg), 1e-12))
        ok = False
        for _ in range(30):
            xn = x + t * d
            xn[np.sign(xn) != orthant] = 0.0
            fn, gn = fg(xn)
            Fn = total(xn, fn)
            if Fn <= F + 1e-4 * float(pg @ (xn - x)):
                ok = True
                break
            t *= 0.5
        if not ok:
            res.reason = "line search failed"
            break
        s, y = xn - x, gn - g
        if float(s @ y) > 1e-10:
            S.append(s)
            Y.append(y)
            if len(S) > m:
                S.pop(0)
                Y.pop(0)
        rel = abs(F - Fn) / max(abs(Fn), abs(F), 1e-12)
        x, f, g, F = xn, fn, gn, Fn
        hist.append(F)
        res.iterations = it
        if callback:
            callback(it, x, F)
        if rel < tol:
            res.converged, res.reason = True, "function values converged"
            break
    res.x, res.f, res.history = x, F, hist
    if not res.reason:
        res.reason = "max iterations reached"
    return res
