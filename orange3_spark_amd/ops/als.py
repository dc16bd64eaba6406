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
