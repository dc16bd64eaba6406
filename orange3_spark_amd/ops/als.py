"""ALS ratings passes: gfx950 kernel (csrc/als.hip) with a PyTorch reference.

mode 0 (matvec): out[u] = sum_j coef_j * (F[c_j] . V[u]) * F[c_j]
mode 1 (rhs)   : out[u] = sum_j coef_j * F[c_j]
"""
from __future__ import annotations

import torch

from . import _native as N


def pass_torch(mode, indptr, cols, coef, F, V):
    n = indptr.numel() - 1
    R = F.shape[1]
    rows = torch.repeat_interleave(torch.arange(n, device=F.device), indptr[1:] - indptr[:-1])
    Fg = F[cols.long()].to(torch.float64)
    s = coef.to(torch.float64)
    if mode == 0:
        s = s * (Fg * V.to(torch.float64)[rows]).sum(1)
    out = torch.zeros((n, R), dtype=torch.float64, device=F.device).index_add_(0, rows, Fg * s[:, None])
    return out.to(F.dtype)


def pass_(mode, indptr, cols, coef, F, V=None):
    n = indptr.numel() - 1
    R = F.shape[1]
    if F.is_cuda and F.dtype == torch.float32 and R <= 512:
        out = torch.empty((n, R), dtype=torch.float32, device=F.device)
        Fc = F.contiguous()
        Vc = None if V is None else V.contiguous().float()
        N.check(N.kernels().o3s_als_pass(mode, indptr.data_ptr(), cols.data_ptr(), coef.data_ptr(), n,
                                         Fc.data_ptr(), R, N.ptr(Vc), out.data_ptr(), None, None,
                                         N.stream_of(Fc)), "als_pass")
        return out
    return pass_torch(mode, indptr, cols, coef, F, V)


def pass_both(indptr, cols, coef, F, V, coef2):
    """(matvec with coef at V, rhs with coef2) in ONE gather pass over the ratings."""
    n = indptr.numel() - 1
    R = F.shape[1]
    if F.is_cuda and F.dtype == torch.float32 and R <= 512:
        out = torch.empty((n, R), dtype=torch.float32, device=F.device)
        out2 = torch.empty((n, R), dtype=torch.float32, device=F.device)
        Fc = F.contiguous()
        N.check(N.kernels().o3s_als_pass(2, indptr.data_ptr(), cols.data_ptr(), coef.data_ptr(), n, Fc.data_ptr(),
                                         R, V.contiguous().float().data_ptr(), out.data_ptr(), coef2.data_ptr(),
                                         out2.data_ptr(), N.stream_of(Fc)), "als_pass2")
        return out, out2
    return pass_torch(0, indptr, cols, coef, F, V), pass_torch(1, indptr, cols, coef2, F, None)


def cg_kernel_ok(F: torch.Tensor) -> bool:
    return F.is_cuda and F.dtype == torch.float32 and F.shape[1] <= 512


def cg_init(x, ax, pf, rhs, lam):
    """Fused CG start (als_cg_kernel mode 0): returns (r, p, rs) for
    r = rhs - (ax + pf + lam*x)."""
    n, R = x.shape
    r = torch.empty_like(x)
    p = torch.empty_like(x)
    rs = torch.empty(n, dtype=torch.float32, device=x.device)
    N.check(N.kernels().o3s_als_cg(0, n, R, x.data_ptr(), r.data_ptr(), p.data_ptr(), ax.data_ptr(), N.ptr(pf),
                                   rhs.data_ptr(), lam.data_ptr(), rs.data_ptr(), N.stream_of(x)), "als_cg_init")
    return r, p, rs


def cg_step(x, r, p, ap, pf, lam, rs):
    """Fused CG step (als_cg_kernel mode 1): updates x, r, p, rs in place."""
    n, R = x.shape
    N.check(N.kernels().o3s_als_cg(1, n, R, x.data_ptr(), r.data_ptr(), p.data_ptr(), ap.data_ptr(), N.ptr(pf),
                                   None, lam.data_ptr(), rs.data_ptr(), N.stream_of(x)), "als_cg_step")
