"""Distributed isotonic regression (Spark's parallel pool-adjacent-violators).

1. range-partition the rows by feature value across ranks (splitters from an
   all-gathered sample, one ``all_to_all_v``) -- equal feature values land on one rank;
2. sort locally on the device and run PAV on the rank's contiguous x-range
   (C++ ``o3s_host_pav``);
3. all-gather the pooled blocks and run the final PAV over them.

Because each rank's range is contiguous, step 2 only coarsens the global solution, so
the result equals a single PAV over all rows.  Output: the block boundaries and their
fitted values, compressed like Spark's model (both ends of every constant block).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ..ops import _native as N


def pav(xlo, xhi, y, w):
    """PAV over x-sorted blocks (numpy fp64); returns the pooled (xlo, xhi, y, w)."""
    xlo, xhi, y, w = (np.ascontiguousarray(a, dtype=np.float64) for a in (xlo, xhi, y, w))
    n = xlo.shape[0]
    out = [np.empty(n) for _ in range(4)]
    if n == 0:
        return out
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    m = N.host().o3s_host_pav(ptr(xlo), ptr(xhi), ptr(y), ptr(w), n, *(ptr(o) for o in out))
    return [o[:m] for o in out]


def fit_isotonic(comm, x: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None, isotonic: bool = True,
                 sample_per_rank: int = 4096, seed: int = 0):
    """Returns (boundaries, predictions) as fp64 numpy arrays."""
    dev = x.device
    x = x.to(torch.float64)
    y = y.to(torch.float64) if isotonic else -y.to(torch.float64)
    w = torch.ones_like(x) if w is None else w.to(dev, torch.float64)
    world = comm.world_size
    if world > 1:
        g = torch.Generator(device="cpu").manual_seed(seed + comm.rank)
        k = min(sample_per_rank, x.shape[0])
        idx = torch.randperm(x.shape[0], generator=g)[:k].to(dev)
        samples = torch.sort(comm.all_gather_v(x[idx].contiguous()))[0]
        if samples.numel():
            q = torch.linspace(0, samples.numel() - 1, world + 1, device=dev)[1:-1].round().long()
            splitters = samples[q]
        else:
            splitters = torch.zeros(world - 1, dtype=torch.float64, device=dev)
        dest = torch.searchsorted(splitters, x, right=True)
        order = torch.argsort(dest, stable=True)
        counts = torch.bincount(dest, minlength=world).tolist()
        packed = torch.stack([x, y, w], dim=1)[order]
        recv, _ = comm.all_to_all_v(packed, counts)
        x, y, w = recv[:, 0], recv[:, 1], recv[:, 2]
    order = torch.argsort(x, stable=True)
    xs = x[order].cpu().numpy()
    bl = pav(xs, xs, y[order].cpu().numpy(), w[order].cpu().numpy())
    local = np.stack(bl, axis=1) if bl[0].size else np.zeros((0, 4))
    if world > 1:
        parts = comm.all_gather_object(local)
        allb = np.concatenate([p for p in parts if p.size] or [np.zeros((0, 4))])
        allb = allb[np.argsort(allb[:, 0], kind="stable")]
        bl = pav(allb[:, 0], allb[:, 1], allb[:, 2], allb[:, 3])
    xlo, xhi, yy, _ = bl
    bounds, preds = [], []
    for a, b, v in zip(xlo, xhi, yy):
        bounds.append(a)
        preds.append(v)
        if b != a:
            bounds.append(b)
            preds.append(v)
    preds = np.asarray(preds, dtype=np.float64)
    return np.asarray(bounds, dtype=np.float64), preds if isotonic else -preds


def predict(boundaries: torch.Tensor, predictions: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Piecewise-linear interpolation between boundaries, constant outside (Spark)."""
    if boundaries.numel() == 0:
        return torch.full_like(x, float("nan"))
    if boundaries.numel() == 1:
        return torch.full_like(x, float(predictions[0]))
    i = torch.searchsorted(boundaries, x, right=True).clamp(1, boundaries.numel() - 1)
    x0, x1 = boundaries[i - 1], boundaries[i]
    y0, y1 = predictions[i - 1], predictions[i]
    t = torch.where(x1 > x0, (x - x0) / (x1 - x0), torch.zeros_like(x))
    out = y0 + t.clamp(0, 1) * (y1 - y0)
    out = torch.where(x <= boundaries[0], predictions[0].expand_as(x), out)
    return torch.where(x >= boundaries[-1], predictions[-1].expand_as(x), out)
