"""Per-bin row sums for a handful of bins (``bin_sums_kernel``, csrc/binsum.hip).

``bin_sums(X, bins, nbins, w)`` -> fp64 [nbins, D + 2] = [sum w x | sum w | sum w ||x||^2]
per bin.  torch's ``index_add_`` on few bins serialises on global fp64 atomics and a
one-hot GEMM with a tiny output tile and a millions-deep K runs on one or two
workgroups; the kernel keeps per-wave fp64 bins in LDS and is deterministic.  Rows whose
bin is outside [0, nbins) are ignored.  Host tensors use index_add_.
"""
from __future__ import annotations

import torch

from . import _native as N

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float64: 2}


def bin_sums_torch(X: torch.Tensor, bins: torch.Tensor, nbins: int, w: torch.Tensor | None = None) -> torch.Tensor:
    X2 = X.reshape(X.shape[0], -1).to(torch.float64)
    b = bins.to(X2.device).long()
    ok = (b >= 0) & (b < nbins)
    b, X2 = b[ok], X2[ok]
    ww = torch.ones(X2.shape[0], dtype=torch.float64, device=X2.device) if w is None else w.to(X2.device)[ok].double()
    out = torch.zeros((nbins, X2.shape[1] + 2), dtype=torch.float64, device=X2.device)
    out[:, :-2].index_add_(0, b, X2 * ww[:, None])
    out[:, -2].index_add_(0, b, ww)
    out[:, -1].index_add_(0, b, ww * (X2 * X2).sum(1))
    return out


def kernel_ok(X: torch.Tensor) -> bool:
    X2 = X if X.dim() == 2 else X.reshape(X.shape[0], -1)
    return X.is_cuda and X.dtype in _DT and X2.stride(-1) == 1 and 1 <= X2.shape[1] <= 256


def bin_sums(X: torch.Tensor, bins: torch.Tensor, nbins: int, w: torch.Tensor | None = None) -> torch.Tensor:
    if not kernel_ok(X) or nbins < 1:
        return bin_sums_torch(X, bins, nbins, w)
    X2 = X if X.dim() == 2 else X.reshape(X.shape[0], -1)
    n, D = X2.shape
    dev = X.device
    b64 = bins.to(dev, torch.int64).contiguous()
    wf = None if w is None else w.to(dev, torch.float32).contiguous()
    group = max(1, 2048 // (D + 2))                  # bins per launch: 4 waves x fp64 bins <= 64 KB of LDS
    grid = N.num_cus(dev) * 4
    out = torch.empty((nbins, D + 2), dtype=torch.float64, device=dev)
    for lo in range(0, nbins, group):
        g = min(group, nbins - lo)
        partial = torch.empty(grid * g * (D + 2), dtype=torch.float64, device=dev)
        N.check(N.kernels().o3s_bin_sums(X2.data_ptr(), _DT[X.dtype], n, X2.stride(0), D, b64.data_ptr(), lo,
                                         N.ptr(wf), g, partial.data_ptr(), grid, out[lo:lo + g].data_ptr(),
                                         N.stream_of(X2)), "bin_sums")
    return out
