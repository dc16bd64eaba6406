"""KMeans assign/update ops: gfx950 kernels (csrc/kmeans.hip) with PyTorch references.

``assign`` returns (cluster index int32 [n], squared distance f32 [n]); ``update`` returns
fp64 per-cluster (sums [K, D], counts [K]) of this rank's rows (caller all-reduces).
"""
from __future__ import annotations

import ctypes as Ct

import torch

from . import _native as N

MAX_KERNEL_D = 160


def prepare_centers(C: torch.Tensor):
    """Split -2*C into bf16 hi/lo [Kp, Dp] (zero padded) and ||c||^2 [Kp] (+inf padded)."""
    K, D = C.shape
    Kp, Dp = (K + 31) // 32 * 32, (D + 31) // 32 * 32
    Cd = C.to(torch.float64)
    m2 = torch.zeros((Kp, Dp), dtype=torch.float32, device=C.device)
    m2[:K, :D] = (-2.0 * Cd).float()
    hi = m2.to(torch.bfloat16)
    lo = (m2 - hi.float()).to(torch.bfloat16)
    cn = torch.full((Kp,), float("inf"), dtype=torch.float32, device=C.device)
    cn[:K] = (Cd * Cd).sum(1).float()
    return hi.contiguous(), lo.contiguous(), cn


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


def assign(X: torch.Tensor, C: torch.Tensor, prepared=None):
    if not kernel_ok(X):
        return assign_torch(X, C)
    hi, lo, cn = prepared or prepare_centers(C)
    n = X.shape[0]
    a = torch.empty(n, dtype=torch.int32, device=X.device)
    d = torch.empty(n, dtype=torch.float32, device=X.device)
    N.check(N.kernels().o3s_kmeans_assign(X.data_ptr(), n, X.stride(0), X.shape[1], hi.data_ptr(), lo.data_ptr(),
                                          cn.data_ptr(), hi.shape[0], a.data_ptr(), d.data_ptr(), N.stream_of(X)),
            "kmeans_assign")
    return a, d


class UpdateWorkspace:
    def __init__(self, device, K: int, D: int, grid: int | None = None):
        self.K, self.D = K, D
        self.grid = grid or N.num_cus(device) * 2
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
