"""Evaluator reductions: gfx950 kernels (csrc/eval.hip) with PyTorch references.

Each returns the LOCAL partial (fp64) that the evaluator all-reduces across ranks:

* :func:`regression_stats` -> [7]  {W, sum w e^2, sum w |e|, sum w y, sum w y^2, sum w p, sum w p^2}
* :func:`confusion`        -> [k, k] rows = label, cols = prediction
* :func:`score_hist`       -> [2, bins] per-class (positive, negative) weighted score histogram

On a GPU tensor the HIP kernel runs (and a missing/failed kernel library raises); CPU
tensors use the torch reference, which is also the numerics oracle in the tests.
"""
from __future__ import annotations

import torch

from . import _native as N

_DT = {torch.float32: 0, torch.float64: 1, torch.int64: 2, torch.int32: 3}


def _operand(t: torch.Tensor | None):
    """(tensor, dtype code) with a kernel-readable dtype; None stays None."""
    if t is None:
        return None, 0
    if t.dtype not in _DT:
        t = t.to(torch.float64 if t.is_floating_point() else torch.int64)
    return t.contiguous(), _DT[t.dtype]


def regression_stats_torch(y, p, w=None):
    y64, p64 = y.to(torch.float64), p.to(torch.float64)
    w64 = torch.ones_like(y64) if w is None else w.to(torch.float64)
    e = p64 - y64
    return torch.stack([w64.sum(), (w64 * e * e).sum(), (w64 * e.abs()).sum(), (w64 * y64).sum(),
                        (w64 * y64 * y64).sum(), (w64 * p64).sum(), (w64 * p64 * p64).sum()])


def regression_stats(y, p, w=None):
    if not y.is_cuda:
        return regression_stats_torch(y, p, w)
    (y, ydt), (p, pdt), (w, wdt) = _operand(y), _operand(p.to(y.device)), _operand(w)
    n = y.numel()
    g = N.kernels().o3s_eval_grid(n)
    slab = torch.empty(g * 8, dtype=torch.float64, device=y.device)
    out = torch.empty(7, dtype=torch.float64, device=y.device)
    N.check(N.kernels().o3s_regression_stats(y.data_ptr(), ydt, p.data_ptr(), pdt, N.ptr(w), wdt, n,
                                             slab.data_ptr(), out.data_ptr(), N.stream_of(y)), "regression_stats")
    return out


def confusion_torch(y, p, k, w=None):
    yl = y.to(torch.float64).long().clamp(0, k - 1)
    pl = p.to(torch.float64).long().clamp(0, k - 1)
    w64 = torch.ones(y.shape[0], dtype=torch.float64, device=y.device) if w is None else w.to(torch.float64)
    return torch.zeros(k * k, dtype=torch.float64, device=y.device).index_add_(0, yl * k + pl, w64).reshape(k, k)


def confusion(y, p, k, w=None):
    if not y.is_cuda or k > 64:
        return confusion_torch(y, p.to(y.device), k, w)
    (y, ydt), (p, pdt), (w, wdt) = _operand(y), _operand(p.to(y.device)), _operand(w)
    n = y.numel()
    g = N.kernels().o3s_eval_grid(n)
    slab = torch.empty(g * k * k, dtype=torch.float64, device=y.device)
    out = torch.empty(k * k, dtype=torch.float64, device=y.device)
    N.check(N.kernels().o3s_confusion(y.data_ptr(), ydt, p.data_ptr(), pdt, N.ptr(w), wdt, n, k,
                                      slab.data_ptr(), out.data_ptr(), N.stream_of(y)), "confusion")
    return out.reshape(k, k)


def score_hist_torch(score, y, lo, span, bins, w=None):
    s = score.to(torch.float64)
    b = ((s - lo) * ((bins - 1) / span)).to(torch.int64).clamp(0, bins - 1)
    neg = (y.to(torch.float64) <= 0.5).to(torch.int64)
    w64 = torch.ones_like(s) if w is None else w.to(torch.float64)
    return torch.zeros(2 * bins, dtype=torch.float64, device=s.device).index_add_(0, neg * bins + b, w64).reshape(2, bins)


def score_hist(score, y, lo, span, bins, w=None):
    """``score`` may be a column view of a [n, 2] rawPrediction matrix (any row stride)."""
    if not score.is_cuda:
        return score_hist_torch(score, y, lo, span, bins, w)
    pstride = 1
    if score.dim() == 1 and score.stride(0) != 1 and score.dtype in _DT:
        pstride = score.stride(0)                # read in place, no strided copy
        base = score
    else:
        base, _ = _operand(score)
    sdt = _DT[base.dtype]
    (y, ydt), (w, wdt) = _operand(y), _operand(w)
    hist = torch.zeros(2 * bins, dtype=torch.float64, device=base.device)
    N.check(N.kernels().o3s_score_hist(base.data_ptr(), sdt, pstride, y.data_ptr(), ydt, N.ptr(w), wdt,
                                       base.shape[0], float(lo), float(span), int(bins), hist.data_ptr(),
                                       N.stream_of(base)), "score_hist")
    return hist.reshape(2, bins)
