"""Data-parallel optimisation of small parametric models written as torch programs.

Used by the estimators whose per-row work is a short chain of GEMMs + elementwise ops
(MultilayerPerceptron, factorization machines, AFT survival regression, ...): the
forward/backward of a row chunk is a handful of hipBLASLt GEMMs on the rank's GPU, the
gradient of the flat parameter vector is summed across ranks with ONE all-reduce per
evaluation (RCCL over xGMI, the analogue of Spark's ``treeAggregate``), and the
optimiser itself runs on the (small) flat vector -- L-BFGS on the host in fp64 (as
Breeze does for Spark), or Adam(W)/GD on the device.

``local_loss(theta, a, b)`` must return the SUM of the per-row losses of local rows
[a, b) as a torch scalar differentiable in ``theta``; the objective is
``sum_loss / W + 0.5 * l2 * ||mask * theta||^2`` with W the global weight sum.
"""
from __future__ import annotations

import math
from typing import Callable

import numpy as np
import torch

from . import optim
from ..runtime import progress

LocalLoss = Callable[[torch.Tensor, int, int], torch.Tensor]


def compute_dtype(device: torch.device) -> torch.dtype:
    return torch.float32 if torch.device(device).type == "cuda" else torch.float64


def chunks(n: int, chunk: int):
    return [(a, min(n, a + chunk)) for a in range(0, n, chunk)] or [(0, 0)]


class Objective:
    """Global smooth objective over sharded rows; one all-reduce per evaluation."""

    def __init__(self, comm, device, n_local: int, local_loss: LocalLoss, W: float, l2: float = 0.0,
                 l2_mask: np.ndarray | None = None, chunk: int = 1 << 20, sw: torch.Tensor | None = None):
        self.comm, self.device = comm, torch.device(device)
        self.sw = sw
        self.dtype = compute_dtype(self.device)
        self.local_loss, self.W = local_loss, float(W)
        self.l2 = float(l2)
        self.mask = l2_mask
        self.parts = chunks(n_local, chunk)
        self.evals = 0

    def weight_of(self, parts) -> float:
        if self.sw is None:
            return float(sum(b - a for a, b in parts))
        return float(sum(float(self.sw[a:b].sum()) for a, b in parts))

    def local(self, theta: torch.Tensor, parts=None) -> tuple[torch.Tensor, torch.Tensor]:
        """(local loss sum, local grad) at device parameters theta (no communication)."""
        th = theta.detach().requires_grad_(True)
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        grad = torch.zeros_like(th, dtype=torch.float64)
        for a, b in parts or self.parts:
            if b <= a:
                continue
            loss = self.local_loss(th, a, b)
            g, = torch.autograd.grad(loss, th)
            grad += g.to(torch.float64)
            total += loss.detach().to(torch.float64)
        return total, grad

    def reduced(self, theta: torch.Tensor, parts=None, W: float | None = None):
        total, grad = self.local(theta, parts)
        buf = torch.cat([grad, total[None]])
        self.comm.all_reduce(buf)
        self.evals += 1
        W = self.W if W is None else W
        return buf[-1] / W, buf[:-1] / W

    def __call__(self, x: np.ndarray):
        theta = torch.from_numpy(np.asarray(x, dtype=np.float64)).to(self.device, self.dtype)
        f, g = self.reduced(theta)
        f = float(f)
        g = g.cpu().numpy()
        if self.l2:
            m = np.ones_like(x) if self.mask is None else self.mask
            f += 0.5 * self.l2 * float(np.sum(m * x * x))
            g = g + self.l2 * m * x
        return f, g


def lbfgs(obj: Objective, x0: np.ndarray, max_iter: int = 100, tol: float = 1e-6):
    return optim.lbfgs(obj, x0, max_iter=max_iter, tol=tol)


def gradient_descent(obj: Objective, x0: np.ndarray, max_iter: int, step: float, tol: float,
                     fraction: float = 1.0, seed: int = 0, adam: bool = False, weight_decay: float = 0.0,
                     betas=(0.9, 0.999), eps: float = 1e-8):
    """Mini-batch GD / AdamW over the sharded rows (device-side parameter state).

    A mini-batch is a seeded random subset (keyed by (seed, iteration)) of each rank's
    local row chunks of expected share ``fraction``; its gradient is normalised by the
    global weight in the batch.  ``fraction == 1`` is full-batch and rank-count invariant.
    """
    dev, dt = obj.device, obj.dtype
    theta = torch.from_numpy(np.asarray(x0, dtype=np.float64)).to(dev, dt)
    m = torch.zeros_like(theta)
    v = torch.zeros_like(theta)
    hist = []
    mask = None if obj.mask is None else torch.from_numpy(obj.mask).to(dev, dt)
    prev = None
    for it in range(1, max_iter + 1):
        progress.iteration(it - 1, max_iter)
        parts = obj.parts
        if fraction < 1.0:
            rng = np.random.default_rng([seed, it])
            keep = rng.random(len(parts)) < fraction
            parts = [p for p, k in zip(parts, keep) if k] or [parts[int(rng.integers(len(parts)))]]
        total, grad = obj.local(theta, parts)
        wb = torch.tensor([obj.weight_of(parts) if fraction < 1.0 else 0.0], dtype=torch.float64, device=dev)
        buf = torch.cat([grad, total[None], wb])
        obj.comm.all_reduce(buf)
        Wb = max(float(buf[-1]) if fraction < 1.0 else obj.W, 1e-300)
        g = (buf[:-2] / Wb).to(dt)
        f = float(buf[-2]) / Wb
        if obj.l2:
            reg = theta if mask is None else theta * mask
            g = g + obj.l2 * reg
            f += 0.5 * obj.l2 * float((reg * theta).sum())
        hist.append(f)
        if adam:
            if weight_decay:
                theta = theta * (1 - step * weight_decay)
            m = betas[0] * m + (1 - betas[0]) * g
            v = betas[1] * v + (1 - betas[1]) * g * g
            mh = m / (1 - betas[0] ** it)
            vh = v / (1 - betas[1] ** it)
            theta = theta - step * mh / (vh.sqrt() + eps)
        else:
            theta = theta - (step / math.sqrt(it)) * g
        if prev is not None and abs(prev - f) <= tol * max(abs(f), 1e-12) and fraction >= 1.0:
            break
        prev = f
    return optim.OptimResult(theta.to(torch.float64).cpu().numpy(), hist[-1] if hist else float("nan"),
                             len(hist), hist, False, "")
