"""Counter-based row sampling (``df.sample`` / ``randomSplit`` / SGD minibatches).

Spark samples per partition with a per-partition seeded RNG, so results change with
the partitioning.  Here the draw for a row is a pure function of (seed, global row
index) via the same fmix32 hash as the synthetic generators: a sample is identical on
1, 2, 4 or 8 GPUs.  Device tensors: one ``hash_uniform_kernel`` pass (csrc/sampling.hip,
SURVEY §2.8 row `df.sample`); host tensors: the same draws as int64 torch ops.
"""
from __future__ import annotations

import torch

from .glm import _fmix32, row_keys

_MASK = 0xFFFFFFFF


def _device_draw(rows: torch.Tensor, seed: int, stream: int, mode: int, p: float = 0.0):
    """GPU: ``hash_uniform_kernel`` (one pass; bitwise the torch draws below)."""
    from . import _native as N
    r = rows.to(torch.int64).contiguous()
    n = r.numel()
    out = torch.empty(n, dtype=torch.float64 if mode == 0 else torch.uint8, device=r.device)
    N.check(N.kernels().o3s_hash_uniform(r.data_ptr(), 0, n, int(seed) & _MASK, int(stream) & _MASK, mode, float(p),
                                         out.data_ptr() if mode == 0 else None,
                                         out.data_ptr() if mode == 1 else None, N.stream_of(r)), "hash_uniform")
    return out.view(rows.shape) if mode == 0 else out.view(rows.shape).to(torch.bool)


def uniform(rows: torch.Tensor, seed: int, stream: int = 0) -> torch.Tensor:
    """U[0,1) float64 per global row index."""
    if rows.is_cuda and rows.numel():
        return _device_draw(rows, seed, stream, 0)
    k = row_keys((seed * 0x2545F491 + stream * 0x9E3779B9) & _MASK, rows)
    k2 = _fmix32(k ^ 0x68E31DA4)
    hi = (k >> 5).to(torch.float64)          # 27 bits
    lo = (k2 >> 6).to(torch.float64)         # 26 bits
    return (hi * 67108864.0 + lo) * (1.0 / 9007199254740992.0)


def uniform_streams(rows: torch.Tensor, seed: int, streams) -> torch.Tensor:
    """[n, k] U[0,1) float64: column j equals ``uniform(rows, seed, streams[j])`` bitwise,
    computed in one broadcast pass (the per-row half of the key is hashed once)."""
    st = torch.as_tensor(list(streams), dtype=torch.int64, device=rows.device)
    seeds = ((seed * 0x2545F491 + st * 0x9E3779B9) & _MASK)[None, :]
    lo = rows & _MASK
    hi = rows >> 32
    inner = _fmix32((lo * 0x9E3779B1 + hi * 0x7FEB352D + 0x165667B1) & _MASK)[:, None]
    k = _fmix32(seeds ^ inner)
    k2 = _fmix32(k ^ 0x68E31DA4)
    return ((k >> 5).to(torch.float64) * 67108864.0 + (k2 >> 6).to(torch.float64)) * (1.0 / 9007199254740992.0)


def bernoulli_mask(rows: torch.Tensor, seed: int, fraction: float) -> torch.Tensor:
    if fraction >= 1.0:
        return torch.ones_like(rows, dtype=torch.bool)
    if fraction <= 0.0:
        return torch.zeros_like(rows, dtype=torch.bool)
    if rows.is_cuda and rows.numel():
        return _device_draw(rows, seed, 0, 1, fraction)
    return uniform(rows, seed) < fraction


def poisson_table(lam: float, device) -> torch.Tensor:
    """fp64 CDF table cdf_0..cdf_{kmax-1} of Poisson(lam), accumulated on ``device``."""
    kmax = int(lam + 12 * (lam ** 0.5) + 12)
    p = torch.exp(torch.tensor(-lam, dtype=torch.float64, device=device))
    cdf = [p]
    for i in range(1, kmax):
        p = p * (lam / i)
        cdf.append(cdf[-1] + p)
    return torch.stack(cdf).contiguous()


def poisson_counts(rows: torch.Tensor, seed: int, lam: float) -> torch.Tensor:
    """Poisson(lam) draw per row by inversion of the CDF (lam is small for sampling).

    k = #{j : cdf_j < u} over the CDF table cdf_0..cdf_{kmax-1} (the same fp64 partial
    sums, accumulated in the same order on the same device, as a per-row loop would
    build) -- one searchsorted instead of a loop with a device sync per term."""
    if lam <= 0:
        return torch.zeros_like(rows)
    u = uniform(rows, seed, stream=1)
    return torch.searchsorted(poisson_table(lam, rows.device), u, right=False).to(rows.dtype)
