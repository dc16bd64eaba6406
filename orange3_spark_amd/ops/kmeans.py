"""KMeans assign/update ops: gfx950 kernels (csrc/kmeans.hip) with PyTorch references.

``assign`` returns (cluster index int32 [n], squared distance f32 [n]); ``update`` returns
fp64 per-cluster (sums [K, D], counts [K]) of this rank's rows (caller all-reduces).
"""
from __future__ import annotations

import ctypes as Ct
import math
import os

import torch

from . import _native as N

MAX_KERNEL_D = 160


class Prepared:
    """Centre-side operands of the assign kernels, built once per Lloyd iteration:
    bf16 hi/lo split of -2*C [Kp, Dp] (zero padded; split kernel), fp16 of -2*C*ms with a
    power-of-two scale ms (screen kernel), ||c||^2 [Kp] (+inf padded), the fp32 centres
    [K, D] (exact distance of screened rows), and for the screen bound max ||c||, the largest
    fp16 rounding error max_c ||m^_c - m_c|| of a centre row (``dm``, m = -2c exact in fp64)
    and max ||m^_c|| (``mmax``)."""

    __slots__ = ("hi", "lo", "cn", "c32", "cmax", "h16", "ms", "dm", "mmax")

    def __init__(self, hi, lo, cn, c32, cmax, h16=None, ms=1.0, dm=None, mmax=None):
        self.hi, self.lo, self.cn, self.c32, self.cmax = hi, lo, cn, c32, cmax
        self.h16, self.ms = h16, ms
        # without the measured errors: the worst case of fp16 rounding (2^-11 per element)
        self.dm = 2.0 ** -10 * cmax if dm is None else dm
        self.mmax = 2.0 * cmax * (1 + 2.0 ** -10) if mmax is None else mmax

    def __iter__(self):                         # legacy (hi, lo, cn) unpacking
        return iter((self.hi, self.lo, self.cn))


def prepare_centers(C: torch.Tensor) -> Prepared:
    K, D = C.shape
    Kp, Dp = (K + 31) // 32 * 32, (D + 31) // 32 * 32
    Cd = C.to(torch.float64)
    m2 = torch.zeros((Kp, Dp), dtype=torch.float32, device=C.device)
    m2[:K, :D] = (-2.0 * Cd).float()
    hi = m2.to(torch.bfloat16)
    lo = (m2 - hi.float()).to(torch.bfloat16)
    cn = torch.full((Kp,), float("inf"), dtype=torch.float32, device=C.device)
    norms = (Cd * Cd).sum(1)
    cn[:K] = norms.float()
    if not K:
        return Prepared(hi.contiguous(), lo.contiguous(), cn, torch.zeros((Kp, D), device=C.device), 0.0,
                        torch.zeros((Kp, Dp), dtype=torch.float16, device=C.device), 1.0, 0.0, 0.0)
    ms = _pow2_scale(float(m2.abs().max()))
    h16 = (m2 * ms).to(torch.float16)
    # the bound's centre terms from the rounded operands themselves (fp64): one host copy
    mh = h16[:K, :D].double() / ms
    stats = torch.stack([norms.max().sqrt(), (mh + 2.0 * Cd).norm(dim=1).max(), mh.norm(dim=1).max()]).cpu()
    cmax, dm, mmax = (float(v) for v in stats)
    # fp32 centres padded to Kp rows (zeros): every index the screen kernel can form is a
    # valid row
    c32 = torch.zeros((Kp, D), dtype=torch.float32, device=C.device)
    c32[:K] = C.float()
    return Prepared(hi.contiguous(), lo.contiguous(), cn, c32, cmax, h16.contiguous(), ms, dm, mmax)


def _pow2_scale(amax: float, top: float = 2.0 ** 15) -> float:
    """Largest power of two s with amax * s <= 2^15 (fp16 keeps its 11 bits up there and
    cannot overflow); 1 for empty / non-finite input."""
    if not math.isfinite(amax) or amax <= 0.0:
        return 1.0
    return 2.0 ** max(-126, min(126, math.floor(math.log2(top / amax))))


_XSCALE: list = [None, None, 0.0]      # [weakref to X, (shape, version), scale]


def x_scale(X: torch.Tensor) -> float:
    """Power-of-two fp16 scale of the data (max |x| over X: one reduction per data
    version, cached for the Lloyd iterations on the same tensor).  The cache holds a weak
    reference to X itself -- never its address, which a later tensor can reuse."""
    ref, key, v = _XSCALE
    if ref is None or ref() is not X or key != (tuple(X.shape), X._version):
        lo, hi = torch.aminmax(X)
        v = _pow2_scale(max(-float(lo), float(hi)))
        import weakref
        _XSCALE[:] = [weakref.ref(X), (tuple(X.shape), X._version), v]
    return v


# Pre-split data for the screen kernel (kmeans_presplit_kernel): the scaled fp16 hi / lo
# halves of every row (D * 4 bytes per row, as much as X itself), ||x||^2 and the squared norm
# of the row's scaled fp16 rounding error (the screen bound's row term), built once per
# data version and reused by every Lloyd iteration -- the kernel's prologue then loads its
# MFMA fragments instead of converting fp32 rows.  PRESPLIT: None = auto (when X is at least
# PRESPLIT_MIN_ROWS rows and the copy fits in half of the free HBM), True / False forces.
PRESPLIT: bool | None = None
PRESPLIT_MIN_ROWS = 1 << 20
_XSPLIT: list = [None, None, None]     # [weakref to X, (shape, version, xs), (XP, XN)]


def presplit(X: torch.Tensor, xs: float):
    """(XP, XN) for the screen kernel, cached per (X, version, scale); None when off."""
    import weakref
    D = (X.shape[1] + 31) // 32 * 32
    if D > 128 or PRESPLIT is False or X.shape[0] == 0:
        return None
    ref, key, val = _XSPLIT
    k = (tuple(X.shape), X._version, xs)
    if ref is not None and ref() is X and key == k:
        return val
    _XSPLIT[:] = [None, None, None]
    need = X.shape[0] * (D * 4 + 8)
    if PRESPLIT is None:
        if X.shape[0] < PRESPLIT_MIN_ROWS:
            return None
        free, _ = torch.cuda.mem_get_info(X.device)
        if need > free // 2:
            return None
    XP = torch.empty((X.shape[0], D), dtype=torch.int32, device=X.device)
    XN = torch.empty((X.shape[0], 2), dtype=torch.float32, device=X.device)
    N.check(N.kernels().o3s_kmeans_presplit(X.data_ptr(), X.shape[0], X.stride(0), X.shape[1], Ct.c_float(xs),
                                            XP.data_ptr(), XN.data_ptr(), N.stream_of(X)), "kmeans_presplit")
    # the split copy lives no longer than X itself (and fit_kmeans drops it when it ends)
    _XSPLIT[:] = [weakref.ref(X, _drop_presplit), k, (XP, XN)]
    return XP, XN


def _drop_presplit(ref) -> None:
    if _XSPLIT[0] is ref:
        _XSPLIT[:] = [None, None, None]


def clear_presplit() -> None:
    """Free the presplit copy of the last X (as large as X itself)."""
    _XSPLIT[:] = [None, None, None]


def screen_bound(P: "Prepared", xs: float, D: int) -> tuple[float, float, float]:
    """(eps_x, eps0, eps_e) of the screen kernel's error bound on |d~_c - d_c| (unscaled
    partial distances d_c = ||c||^2 - 2 x.c):

        E(x) = eps_x ||x|| + eps_e ||dx|| + eps0,     dx = x^ - x

    With x^ = fp16(x xs)/xs, m^ = fp16(m ms)/ms and m = -2c (fp64):
    x^.m^ - x.m = dx.m^ + x.dm, so by Cauchy-Schwarz on the ACTUAL rounding errors
    |x^.m^ - x.m| <= ||dx|| max||m^|| + ||x|| max||dm|| -- dm and max||m^|| measured on the
    rounded centres (``prepare_centers``), ||dx|| per row by the kernel.  The fp32
    accumulation of S ||c||^2 and the D exact fp16 products adds <= g (||c||^2 + ||x^|| ||m^||)
    with g = 2 (D + 2) 2^-24 (twice the textbook gamma: no assumption on the matrix core's
    rounding mode), ||x^|| <= ||x|| + ||dx||; the fp32 ||c||^2 adds 2^-24 ||c||^2; a 2^-10
    margin covers the bound's own fp32 evaluation.  On data with full mantissas ||dx|| is
    ~2^-12 ||x|| against the 2^-11 per-element worst case, so E is ~5x below the
    per-element bound this replaced (E = 2^-8 ||x|| max||c||)."""
    Dp = (D + 31) // 32 * 32
    g = 2.0 * (Dp + 2) * 2.0 ** -24
    mg = 1.0 + 2.0 ** -10
    eps_x = (P.dm + g * P.mmax) * mg
    eps_e = P.mmax * (1.0 + g) * mg
    eps0 = (g + 2.0 ** -23) * P.cmax * P.cmax * mg
    return eps_x, eps0, eps_e


def row_bound(X: torch.Tensor, P: "Prepared", xs: float) -> torch.Tensor:
    """The screen bound E(x) of every row (fp64, torch: tests and diagnostics)."""
    eps_x, eps0, eps_e = screen_bound(P, xs, X.shape[1])
    Xd = X.double()
    dx = (X * xs).half().double() / xs - Xd
    return eps_x * Xd.norm(dim=1) + eps_e * dx.norm(dim=1) + eps0


def kernel_ok(X: torch.Tensor) -> bool:
    return (X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and X.shape[1] % 4 == 0
            and X.shape[1] <= MAX_KERNEL_D and X.stride(1) == 1 and X.stride(0) % 4 == 0)


def update_kernel_ok(X: torch.Tensor) -> bool:
    """The slab-update kernel streams whole rows (D <= 256), independent of the assign
    kernel's register-bound D limit."""
    return (X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and X.shape[1] <= 256
            and X.stride(1) == 1)


def assign_torch(X: torch.Tensor, C: torch.Tensor, chunk: int = 1 << 16):
    n = X.shape[0]
    a = torch.empty(n, dtype=torch.int32, device=X.device)
    d = torch.empty(n, dtype=torch.float32, device=X.device)
    Cd = C.to(torch.float64)
    cn = (Cd * Cd).sum(1)
    for s in range(0, n, chunk):
        Xc = X[s:s + chunk].to(torch.float64)
        dist = (Xc * Xc).sum(1, keepdim=True) - 2 * Xc @ Cd.T + cn[None, :]
        v, i = dist.min(1)
        a[s:s + chunk] = i.to(torch.int32)
        d[s:s + chunk] = v.clamp_min(0).float()
    return a, d


# screen-pass bound: see screen_bound (fp16 operands, Cauchy-Schwarz on the actual errors)
# auto mode: the plain screen until it flags SCREEN_MAX_FLAG_FRACTION of the rows, then the
# split kernel for every row (re-probing the screen every SPLIT_REPROBE calls).  The pair
# screen (top-3 tracking, two-centre near ties settled exactly in-kernel) joins the chain
# when PAIR_FROM is set: on uniform data it flags ~3x fewer rows than the plain screen but
# runs one 32-row tile per wave (register budget), which costs what it saves on MI355X
# (profiles/kmeans_fp16_screen_r3.json), so auto leaves it off by default.
PAIR_FROM: float | None = None
SCREEN_MAX_FLAG_FRACTION = 0.5
SPLIT_REPROBE = 6             # split calls before the pair screen is tried again
SCREEN_TT = 0                 # 32-row tiles per wave in the screen kernel (0: by D)

_screen_state: dict = {}      # (id(X), shape, Cpad) -> (weakref to X, mode, flagged fraction, countdown)


def _state_get(key, X):
    e = _screen_state.get(key)
    if e is None or e[0]() is not X:          # a new tensor (maybe at a reused address)
        return ("screen", 0.0, 0)
    return e[1:]


def _state_set(key, X, *val):
    import weakref
    if len(_screen_state) > 64:
        for k in [k for k, e in _screen_state.items() if e[0]() is None]:
            del _screen_state[k]
    _screen_state[key] = (weakref.ref(X),) + val


class _ScreenWs:
    """Per-device near-tie buffers: a counter and a row list (grown on demand)."""

    def __init__(self):
        self.cnt = None
        self.rows = None

    def get(self, n: int, dev):
        if self.cnt is None or self.cnt.device != dev:
            self.cnt = torch.zeros(1, dtype=torch.int32, device=dev)
            self.rows = None
        if self.rows is None or self.rows.numel() < n:
            self.rows = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        return self.cnt, self.rows


_SWS = _ScreenWs()


def screen_ok(X: torch.Tensor) -> bool:
    return kernel_ok(X) and X.shape[0] < 2 ** 31


def assign(X: torch.Tensor, C: torch.Tensor, prepared=None, mode: str = "auto", stats: dict | None = None,
           need_dist: bool = True):
    """(cluster int32 [n], squared distance f32 [n]) of every row of X.  ``need_dist=False``
    returns (cluster, None) and lets the screen kernel skip the per-row exact distance (the
    lo half of the pre-split rows and the chosen centre's fp32 row are then never read).

    GPU: ``mode='screen'`` runs the one-MFMA screen kernel and re-solves only its near-tie
    rows with the split-precision kernel; ``'pair'`` is the screen that also settles
    two-centre near ties exactly in-kernel; ``'split'`` runs the split kernel on every
    row; ``'auto'`` moves screen (-> pair when ``PAIR_FROM`` is set) -> split as the
    previous call on this X flagged more than ``SCREEN_MAX_FLAG_FRACTION`` of its rows, and
    re-probes the screen every ``SPLIT_REPROBE`` split calls; ``'approx'`` is the screen
    without the near-tie re-solve (k-means|| sampling: the chosen centre is within the
    screen bound of the nearest, its distance exact)."""
    if not kernel_ok(X):
        a, d = assign_torch(X, C)
        return a, (d if need_dist else None)
    P = prepared if isinstance(prepared, Prepared) else prepare_centers(C)
    n = X.shape[0]
    a = torch.empty(n, dtype=torch.int32, device=X.device)
    d = torch.empty(n, dtype=torch.float32, device=X.device) if need_dist else None
    lib = N.kernels()
    st = N.stream_of(X)
    # near-tie rates depend on the centre set: keyed by the padded centre count too, so
    # k-means|| candidate passes (thousands of close candidates: mostly near ties) do not
    # push the later Lloyd iterations (k centres) onto the split path
    key = (id(X), tuple(X.shape), P.hi.shape[0])
    if mode == "auto":
        m, f, cd = _state_get(key, X)
        if not screen_ok(X):
            mode = "split"
        elif m == "split" and cd > 0:
            mode = "split"
            _state_set(key, X, "split", f, cd - 1)
        else:
            mode = ("pair" if PAIR_FROM is not None else "screen") if m == "split" else m
    approx = mode == "approx"
    if approx:
        # k-means|| rounds / candidate weights: the screen's pick and its exact fp32 distance
        # are used as they are (a near tie may go to a centre within the screen bound of the
        # nearest -- irrelevant to the sampling probabilities), no re-solve, no host sync
        mode = "screen" if screen_ok(X) else "split"
    if stats is not None:
        stats["mode"] = mode
    if approx and mode == "screen":
        cnt, rows = _SWS.get(n, X.device)
        cnt.zero_()                              # the kernel still lists its near ties (< n rows)
        xs = x_scale(X)
        eps_x, eps0, eps_e = screen_bound(P, xs, X.shape[1])
        ps = presplit(X, xs)
        tt = SCREEN_TT or (2 if X.shape[1] <= 128 else 1)
        N.check(lib.o3s_kmeans_screen2(X.data_ptr(), n, X.stride(0), X.shape[1], P.h16.data_ptr(), P.cn.data_ptr(),
                                       P.c32.data_ptr(), P.c32.stride(0), P.hi.shape[0], Ct.c_float(eps_x),
                                       Ct.c_float(eps0), Ct.c_float(eps_e * P.ms), Ct.c_float(xs),
                                       Ct.c_float(xs * P.ms), a.data_ptr(), N.ptr(d), cnt.data_ptr(), rows.data_ptr(),
                                       tt, 0, N.ptr(ps[0]) if ps else None, N.ptr(ps[1]) if ps else None, None, None,
                                       st),
                "kmeans_screen")
        return a, d
    if mode in ("screen", "pair") and screen_ok(X):
        cnt, rows = _SWS.get(n, X.device)
        cnt.zero_()
        tt = SCREEN_TT or (2 if X.shape[1] <= 128 else 1)
        xs = x_scale(X)
        eps_x, eps0, eps_e = screen_bound(P, xs, X.shape[1])
        ps = presplit(X, xs) if mode == "screen" else None
        N.check(lib.o3s_kmeans_screen2(X.data_ptr(), n, X.stride(0), X.shape[1], P.h16.data_ptr(), P.cn.data_ptr(),
                                       P.c32.data_ptr(), P.c32.stride(0), P.hi.shape[0], Ct.c_float(eps_x),
                                       Ct.c_float(eps0), Ct.c_float(eps_e * P.ms), Ct.c_float(xs),
                                       Ct.c_float(xs * P.ms), a.data_ptr(), N.ptr(d), cnt.data_ptr(), rows.data_ptr(),
                                       tt, int(mode == "pair"), N.ptr(ps[0]) if ps else None,
                                       N.ptr(ps[1]) if ps else None, None, None, st),
                "kmeans_screen")
        m = int(cnt.item())                      # the near-tie count sizes the re-solve grid
        frac = m / max(n, 1)
        if mode == "screen" and PAIR_FROM is not None and frac > PAIR_FROM:
            _state_set(key, X, "pair", frac, 0)
        elif frac > SCREEN_MAX_FLAG_FRACTION:
            _state_set(key, X, "split", frac, SPLIT_REPROBE)
        else:
            _state_set(key, X, mode, frac, 0)
        if stats is not None:
            stats["flagged"] = m
        if m:
            N.check(lib.o3s_kmeans_assign(X.data_ptr(), m, X.stride(0), X.shape[1], P.hi.data_ptr(),
                                          P.lo.data_ptr(), P.cn.data_ptr(), P.hi.shape[0], a.data_ptr(),
                                          N.ptr(d), rows.data_ptr(), st), "kmeans_assign(recheck)")
        return a, d
    N.check(lib.o3s_kmeans_assign(X.data_ptr(), n, X.stride(0), X.shape[1], P.hi.data_ptr(), P.lo.data_ptr(),
                                  P.cn.data_ptr(), P.hi.shape[0], a.data_ptr(), N.ptr(d), None, st),
            "kmeans_assign")
    if stats is not None:
        stats["flagged"] = n
    return a, d


def assign_bounded(X: torch.Tensor, P: Prepared, a: torch.Tensor, bnd: torch.Tensor,
                   rows: torch.Tensor | None = None, stats: dict | None = None) -> None:
    """The plain screen (+ exact re-solve of its near ties) over ``rows`` of X (int32,
    ascending; None = every row), writing ``a[row]`` and the Hamerly bounds ``bnd[row]``
    = (upper bound on ||x - c_a||, lower bound on the distance to every other centre;
    (inf, 0) for re-solved near ties) -- models/kmeans.py skips rows whose bounds, moved
    by the centres' shifts, still certify the assignment."""
    n = X.shape[0] if rows is None else int(rows.numel())
    if n == 0:
        return
    lib = N.kernels()
    st = N.stream_of(X)
    cnt, flag = _SWS.get(n, X.device)
    cnt.zero_()
    xs = x_scale(X)
    eps_x, eps0, eps_e = screen_bound(P, xs, X.shape[1])
    ps = presplit(X, xs)
    tt = SCREEN_TT or (2 if X.shape[1] <= 128 else 1)
    if rows is not None and (rows.dtype != torch.int32 or not rows.is_contiguous()):
        raise ValueError("rows must be contiguous int32")
    if bnd.dtype != torch.float32 or tuple(bnd.shape) != (X.shape[0], 2) or not bnd.is_contiguous():
        raise ValueError("bnd must be fp32 [n, 2]")
    N.check(lib.o3s_kmeans_screen2(X.data_ptr(), n, X.stride(0), X.shape[1], P.h16.data_ptr(), P.cn.data_ptr(),
                                   P.c32.data_ptr(), P.c32.stride(0), P.hi.shape[0], Ct.c_float(eps_x),
                                   Ct.c_float(eps0), Ct.c_float(eps_e * P.ms), Ct.c_float(xs), Ct.c_float(xs * P.ms),
                                   a.data_ptr(), None,
                                   cnt.data_ptr(), flag.data_ptr(), tt, 0, N.ptr(ps[0]) if ps else None,
                                   N.ptr(ps[1]) if ps else None, N.ptr(rows), bnd.data_ptr(), st),
            "kmeans_screen(bounds)")
    m = int(cnt.item())
    if stats is not None:
        stats["screened"] = n
        stats["flagged"] = m
    if m:
        N.check(lib.o3s_kmeans_assign(X.data_ptr(), m, X.stride(0), X.shape[1], P.hi.data_ptr(), P.lo.data_ptr(),
                                      P.cn.data_ptr(), P.hi.shape[0], a.data_ptr(), None, flag.data_ptr(), st),
                "kmeans_assign(recheck)")


def moments(X: torch.Tensor, shift: torch.Tensor):
    """(sum over rows of (x - shift) [D], sum of ||x - shift||^2), fp64, in ONE pass over X
    (``kmeans_moments_kernel``: fp64 per-thread sums, per-block partials in a fixed order);
    torch on CPU / shapes the kernel does not take."""
    n, D = X.shape
    sh = shift.to(X.device, torch.float32).contiguous()
    if not (X.is_cuda and X.dtype == torch.float32 and D % 4 == 0 and D <= 1024 and X.stride(1) == 1
            and X.stride(0) % 4 == 0 and X.data_ptr() % 16 == 0 and n > 0):
        s1 = torch.zeros(D, dtype=torch.float64, device=X.device)
        s2 = torch.zeros((), dtype=torch.float64, device=X.device)
        step = max(1, (1 << 26) // max(1, D))
        for i in range(0, n, step):
            blk = X[i:i + step].to(torch.float64) - sh.to(torch.float64)
            s1 += blk.sum(0)
            s2 += (blk * blk).sum()
        return s1, s2
    grid = int(max(1, min(N.num_cus(X.device) * 8, -(-n // 4096))))
    part = torch.empty((grid, D + 1), dtype=torch.float64, device=X.device)
    N.check(N.kernels().o3s_kmeans_moments(X.data_ptr(), n, X.stride(0), D, sh.data_ptr(), grid, part.data_ptr(),
                                           N.stream_of(X)), "kmeans_moments")
    tot = part.sum(0)
    return tot[:D], tot[D]


def cost(X: torch.Tensor, a: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
    """sum over rows of ||x - C[a]||^2 (fp64 scalar) in one pass: ``kmeans_cost_kernel``
    (fp32 per float4 of a row, fp64 above, fixed-order block partials); torch elsewhere."""
    n, D = X.shape
    Cf = C.to(X.device, torch.float32).contiguous()
    if not (X.is_cuda and X.dtype == torch.float32 and D % 4 == 0 and D <= 1024 and X.stride(1) == 1
            and X.stride(0) % 4 == 0 and X.data_ptr() % 16 == 0 and n > 0 and a.dtype == torch.int32
            and a.is_contiguous()):
        tot = torch.zeros((), dtype=torch.float64, device=X.device)
        step = max(1, (1 << 24) // max(1, D))
        for i in range(0, n, step):
            d = X[i:i + step].to(torch.float64) - Cf[a[i:i + step].long()].to(torch.float64)
            tot += (d * d).sum()
        return tot
    grid = int(max(1, min(N.num_cus(X.device) * 8, -(-n // 4096))))
    part = torch.empty(grid, dtype=torch.float64, device=X.device)
    N.check(N.kernels().o3s_kmeans_cost(X.data_ptr(), n, X.stride(0), D, a.data_ptr(), Cf.data_ptr(), Cf.stride(0),
                                        grid, part.data_ptr(), N.stream_of(X)), "kmeans_cost")
    return part.sum()


def bounds_recheck(a: torch.Tensor, bnd: torch.Tensor, delta: torch.Tensor, dmax: float,
                   max_rows: int | None = None):
    """Move the Hamerly bounds by the centre shifts (ub += delta[a], lb -= dmax, in place);
    returns (count, rows): the rows (int32, ascending) whose bounds no longer certify their
    centre, or rows = None when there are more than ``max_rows`` of them (the caller then
    screens every row: no list is sorted)."""
    n = a.shape[0]
    if a.is_cuda:
        dev = a.device
        grid = int(max(1, min(N.num_cus(dev) * 8, -(-n // 4096))))
        cnt = torch.empty(grid, dtype=torch.int32, device=dev)
        d32 = delta.to(torch.float32).contiguous()
        lib, st = N.kernels(), N.stream_of(a)
        N.check(lib.o3s_kmeans_bounds(a.data_ptr(), bnd.data_ptr(), n, d32.data_ptr(), Ct.c_float(dmax), 0,
                                      cnt.data_ptr(), None, None, grid, st), "kmeans_bounds")
        offs = torch.cumsum(cnt.to(torch.int64), 0)
        m = int(offs[-1])
        if max_rows is not None and m > max_rows:
            return m, None
        rows = torch.empty(m, dtype=torch.int32, device=dev)
        if m:
            offs = offs - cnt.to(torch.int64)                  # exclusive prefix
            N.check(lib.o3s_kmeans_bounds(a.data_ptr(), bnd.data_ptr(), n, d32.data_ptr(), Ct.c_float(dmax), 1,
                                          cnt.data_ptr(), offs.data_ptr(), rows.data_ptr(), grid, st),
                    "kmeans_bounds(list)")
        return m, rows
    bnd[:, 0] += delta[a.long()].to(bnd.dtype)
    bnd[:, 1] -= dmax
    r = torch.nonzero(~(bnd[:, 0] < bnd[:, 1])).reshape(-1).to(torch.int32)
    m = int(r.numel())
    return m, (None if max_rows is not None and m > max_rows else r)


UPDATE_BLOCKS_PER_CU = int(os.environ.get("O3S_KM_UPDATE_BLOCKS", "4"))   # update-kernel blocks per CU (A/B: 1 / 2 / 4 / 8 -> 57.7 / 56.2 / 55.3 / 57.7 ms per uniform Lloyd iteration)


class UpdateWorkspace:
    """Slab workspace of the update kernel: ``grid`` blocks, each with a private [Kp, D]
    fp32 slab (zeroed per call, summed in a fixed order)."""

    def __init__(self, device, K: int, D: int, grid: int | None = None):
        self.K, self.D = K, D
        self.grid = grid or N.num_cus(device) * UPDATE_BLOCKS_PER_CU
        sf, cf, lb = Ct.c_int64(), Ct.c_int64(), Ct.c_int()
        # -3: K too large for the in-LDS counting sort -> update() takes the torch path
        self.ok = N.kernels().o3s_kmeans_update_ws(K, D, self.grid, Ct.byref(sf), Ct.byref(cf), Ct.byref(lb)) == 0
        if not self.ok:
            sf.value = cf.value = 0
        self.slab = torch.empty(sf.value, dtype=torch.float32, device=device)
        self.cnt = torch.empty(cf.value, dtype=torch.float32, device=device)
        self.sums = torch.empty((K, D), dtype=torch.float64, device=device)
        self.counts = torch.empty(K, dtype=torch.float64, device=device)


def update_torch(X, a, K: int, w=None):
    D = X.shape[1]
    sums = torch.zeros((K, D), dtype=torch.float64, device=X.device)
    Xd = X.to(torch.float64) if w is None else X.to(torch.float64) * w.to(torch.float64)[:, None]
    sums.index_add_(0, a.long(), Xd)
    cw = torch.ones(X.shape[0], dtype=torch.float64, device=X.device) if w is None else w.to(torch.float64)
    counts = torch.zeros(K, dtype=torch.float64, device=X.device).index_add_(0, a.long(), cw)
    return sums, counts


def update(X, a, K: int, ws: UpdateWorkspace | None = None, w=None):
    if not update_kernel_ok(X) or w is not None:
        return update_torch(X, a, K, w)
    ws = ws or UpdateWorkspace(X.device, K, X.shape[1])
    if not ws.ok:
        return update_torch(X, a, K, w)
    ws.slab.zero_()
    ws.cnt.zero_()
    N.check(N.kernels().o3s_kmeans_update(X.data_ptr(), X.shape[0], X.stride(0), X.shape[1], a.data_ptr(), K,
                                          ws.slab.data_ptr(), ws.cnt.data_ptr(), ws.grid, ws.sums.data_ptr(),
                                          ws.counts.data_ptr(), N.stream_of(X)), "kmeans_update")
    return ws.sums, ws.counts
