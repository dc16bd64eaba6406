"""Generalised linear model engine: data view, objective, solvers.

Serves LogisticRegression (binomial + multinomial), LinearSVC and LinearRegression.
Replaces MLlib's LogisticRegression.train / LinearSVC.train loops (reached in the
reference via OWSparkEstimator.apply -> fit, orangecontrib/spark/base/spark_ml_estimator.py:22).

Per iteration on every rank:
  1. one fused pass over the local rows (``ops.glm``: HIP kernel on bf16 HBM data, plus
     the in-kernel regenerated lineage rows when the dataset exceeds HBM);
  2. ONE all-reduce of a single fp64 vector [grad | sum r | loss | weight] over RCCL;
  3. O(D) host (L-BFGS/OWL-QN) or device (SGD) update.

Objective (Spark ML): (1/W) sum_i w_i loss_i + regParam * ((1-a)/2 ||b||^2 + a ||b||_1),
optimised over *standardised* coefficients b~_j = b_j * std_j (penalty on b~ when
standardization=true, on b otherwise); the intercept is never penalised.
"""
from __future__ import annotations

import logging
import math
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..frame import column as C
from ..ops import _native as N
from ..ops import glm as G
from ..runtime.tracing import traced
from ..synthetic import LineageVectorColumn
from . import optim
from ..runtime import progress

log = logging.getLogger(__name__)

LOSS_ID = {"logistic": G.LOSS_LOGISTIC, "hinge": G.LOSS_HINGE, "squared": G.LOSS_SQUARED}


class GlmData:
    """This rank's (X, y, w) in the form the GLM pass consumes."""

    def __init__(self, comm, feat: C.Column, y: torch.Tensor, sw: torch.Tensor | None = None,
                 chunk_rows: int = 1 << 22):
        from ..frame.spill import SpilledVectorColumn
        self.comm = comm
        self.lineage = None
        self.spill = None            # HostStreamer of the rows kept in pinned host memory
        if isinstance(feat, C.SparseVectorColumn):
            feat = C.VectorColumn(feat.to_dense(torch.float32), feat.size)
        if isinstance(feat, LineageVectorColumn):
            X = feat.data
            self.lineage = (feat.spec, feat.row0 + feat.resident_rows, feat.lineage_rows)
        elif isinstance(feat, SpilledVectorColumn):
            X = feat.data
            if feat.spilled_rows:
                self.spill = feat.streamer()
        else:
            X = feat.data
        self.d = int(feat.size)
        self.X = X
        self.device = X.device if X.numel() or X.is_cuda else y.device
        self.kernel = X.is_cuda and X.dtype == torch.bfloat16 and X.is_contiguous()
        self.ld = int(X.shape[1])
        self.y = y.to(self.device, torch.float32).contiguous() if self.kernel else y.to(self.device)
        self.sw = None if sw is None else (sw.to(self.device, torch.float32).contiguous() if self.kernel else sw.to(self.device))
        self.nres = int(X.shape[0])
        self.n_local = self.nres + (self.lineage[2] if self.lineage else 0) + \
            (int(self.spill.host.shape[0]) if self.spill is not None else 0)
        self.n = int(comm.sum_scalar(self.n_local))
        self.chunk = chunk_rows
        self.ws = G.GlmWorkspace(self.device, self.ld) if self.kernel else None
        self.passes = 0
        # Resident rows stream HBM (memory bound) while lineage rows are regenerated
        # in-kernel (VALU bound).  Two kernels on two HIP streams barely overlap (the
        # first grid fills every CU slot; profiles/glm_overlap.json: 63.8 ms vs 67.2 ms
        # back to back at 1B x 256 on one GPU), so by default (O3S_GLM_MIXED=1) ONE
        # launch interleaves resident and lineage tiles inside every wave
        # (ops.glm.glm_grad_mixed): 46-47 ms for the same pass
        # (profiles/glm_mixed_sweep.json).  The grid is 32 blocks per CU: the dispatcher
        # then balances CUs that stream at different speeds (a persistent one-wave-set
        # grid was 8-10 % slower).
        self.overlap = None
        # (also without lineage rows: its LPR = 8 lane mapping streams 6.7 TB/s vs 6.4 TB/s
        # for glm_grad's, tools/bench_glm_roles.py)
        self.mixed = self.kernel and os.environ.get("O3S_GLM_MIXED", "1") == "1" \
            and (self.sw is None or self.sw.shape[0] == self.y.shape[0])
        self._row0 = int(feat.row0) if isinstance(feat, LineageVectorColumn) else None
        if self.spill is not None and self.kernel:
            self.mixed = True                  # chunks run through the mixed kernel (sampling, weights)
        self._setup_workspace()
        self.ws_stream = G.GlmWorkspace(self.device, self.ld) if (self.spill is not None and self.kernel) else None

    # ---------------------------------------------------------------- streamed rows
    def _res(self, t):
        """The resident rows' slice of a per-row column (labels / weights)."""
        return None if t is None else (t if self.spill is None else t[: self.nres])

    def _chunk_rows(self, t, off, rows):
        return None if t is None else t[self.nres + off: self.nres + off + rows]

    @property
    def mode(self) -> str:
        """How this rank's rows reach the pass: resident / resident+lineage / resident+streamed."""
        if self.lineage:
            return "resident+lineage" if self.nres else "lineage"
        if self.spill is not None:
            return "resident+streamed" if self.nres else "streamed"
        return "resident"

    def _setup_workspace(self):
        if self.mixed:
            cus = N.num_cus(self.device)
            # 16-row tiles, 4 waves per block: never more blocks than one tile per wave
            # (a small table would otherwise launch 8K mostly-idle blocks and make the
            # finish kernel sum 8K slab rows -- ~100 us per step on a 4K-row table)
            tiles = -(-int(self.X.shape[0]) // 16) + -(-int(self.lineage[2] if self.lineage else 0) // 16)
            if self.spill is not None:
                tiles = max(tiles, -(-int(self.spill.chunk_rows) // 16))
            grid = max(1, min(cus * 32, -(-tiles // 4)))
            self.ws = G.GlmWorkspace(self.device, self.ld,
                                     grid=int(os.environ.get("O3S_GLM_GRID_MIX", str(grid))))
        elif self.kernel and self.lineage and self.X.shape[0] and os.environ.get("O3S_GLM_OVERLAP", "1") == "1":
            cus = N.num_cus(self.device)
            res_grid = int(os.environ.get("O3S_GLM_GRID_RES", str(cus * 8)))
            lin_grid = int(os.environ.get("O3S_GLM_GRID_LIN", str(cus)))
            self.ws = G.GlmWorkspace(self.device, self.ld, grid=res_grid)
            self.overlap = (torch.cuda.Stream(self.device), G.GlmWorkspace(self.device, self.ld, grid=lin_grid))

    def global_row0(self) -> int:
        """Global index of this rank's first row (row-sharded frames: exclusive prefix sum
        of the local row counts in rank order) -- the key of the mini-batch sampler."""
        if self._row0 is None:
            counts = self.comm.all_gather_object(int(self.n_local))
            self._row0 = int(sum(counts[: self.comm.rank]))
        return self._row0

    def require_mixed(self) -> None:
        """Mini-batch sampling lives in the mixed kernel: switch to it if disabled."""
        if self.kernel and not self.mixed:
            self.mixed, self.overlap = True, None
            self._setup_workspace()

    # ---------------------------------------------------------------- moments
    def stats(self):
        """Fused summarizer + first-gradient pass (``ops.glm.glm_stats_mixed``), all-reduced,
        as host fp64 ``(s1, s2, syx, W, sum w y, sum w y^2)`` over the first ``d`` columns;
        None when this data has no fused pass (CPU dense rows use the torch reference)."""
        spec, r0, nl = self.lineage if self.lineage else (None, 0, 0)
        if self.kernel:
            if not self.mixed:
                return None
            st = G.glm_stats_mixed(self.X, self._res(self.y), self._res(self.sw), nl, spec.d if spec else self.d,
                                   spec.seed if spec else 0, r0)
            if st is None:
                return None
            dpad = self.ws.dpad
        else:
            st = G.glm_stats_torch(self.X, self._res(self.y), self._res(self.sw), nl, spec.d if spec else self.d,
                                   spec.seed if spec else 0, r0).to(self.device)
            dpad = G.layout(self.ld)[0]
        if self.spill is not None:
            acc = st

            def chunk(Xc, off):
                yc, wc = self._chunk_rows(self.y, off, Xc.shape[0]), self._chunk_rows(self.sw, off, Xc.shape[0])
                if self.kernel:
                    acc.add_(G.glm_stats_mixed(Xc, yc, wc, 0, self.d, 0, 0))
                else:
                    acc.add_(G.glm_stats_torch(Xc, yc, wc, 0, self.d, 0, 0).to(self.device))
            self.spill.run(chunk)
        self.comm.all_reduce(st)
        h = st.cpu().numpy()
        d = self.d
        self.passes += 1
        return (h[:d], h[dpad:dpad + d], h[2 * dpad:2 * dpad + d], float(h[3 * dpad]), float(h[3 * dpad + 1]),
                float(h[3 * dpad + 2]))

    def moments(self):
        """Global weighted (mean, variance (unbiased), weight sum, label moments)."""
        d = self.d
        def torch_stats(Xc, swc):
            Xd = Xc.to(torch.float64)
            w = torch.ones(Xd.shape[0], dtype=torch.float64, device=Xd.device) if swc is None \
                else swc.to(torch.float64)
            return torch.cat([w @ Xd, w @ (Xd * Xd), w.sum().reshape(1)])
        if self.kernel:
            parts = [G.glm_colstats(self.X, self._res(self.sw))] if self.X.shape[0] else []
            if self.lineage:
                spec, r0, nl = self.lineage
                parts.append(G.glm_colstats_synth(nl, self.ld, spec.d, spec.seed, r0, self.device))
            if parts:
                st = torch.stack(parts).sum(0)
            else:
                st = torch.zeros(2 * self.ld + 1, dtype=torch.float64, device=self.device)
        else:
            st = torch_stats(self.X, self._res(self.sw))
        if self.spill is not None:
            def chunk(Xc, off):
                wc = self._chunk_rows(self.sw, off, Xc.shape[0])
                st.add_(G.glm_colstats(Xc, wc) if self.kernel else torch_stats(Xc, wc).to(st.device))
            self.spill.run(chunk)
        ld = self.ld
        yw = self.y.to(torch.float64) * (1.0 if self.sw is None else self.sw.to(torch.float64))
        ystats = torch.stack([yw.sum(), (yw * self.y.to(torch.float64)).sum()]).to(st.device)
        full = torch.cat([st, ystats]).contiguous()
        self.comm.all_reduce(full)
        full = full.cpu().numpy()
        s1, s2, W = full[:ld], full[ld:2 * ld], full[2 * ld]
        ys1, ys2 = full[2 * ld + 1], full[2 * ld + 2]
        if self.lineage:
            # lineage rows carry unit weights but their labels are regenerated in-kernel;
            # label moments were taken from the materialised label column
            pass
        mean = s1 / max(W, 1e-300)
        var = (s2 - W * mean * mean) / max(W - 1.0, 1e-300)
        var = np.maximum(var, 0.0)
        ymean = ys1 / max(W, 1e-300)
        yvar = max((ys2 - W * ymean * ymean) / max(W - 1.0, 1e-300), 0.0)
        return mean[:self.d], var[:self.d], W, ymean, yvar

    # ---------------------------------------------------------------- one pass
    def pass_device(self, coef_eff: torch.Tensor, intercept: float | None, loss: int,
                    t_dev: torch.Tensor | None = None, sample: tuple | None = None) -> torch.Tensor:
        """Local pass; returns device fp64 [grad (dpad) | sum r | loss | wsum] (not reduced).

        Resident and lineage rows accumulate into the workspace's result buffer (valid
        until the next pass).  ``intercept=None``: ``coef_eff`` is the fp32 [dpad + 1]
        device operand (coefficients + intercept).  ``sample=(seed, fraction)`` with
        fraction < 1: mini-batch of iteration ``t_dev[0] + 1`` (in-kernel row mask).
        """
        ws = self.ws
        if sample is not None and sample[1] < 1.0:
            self.require_mixed()
            ws = self.ws
        if self.mixed:
            spec, r0, nl = self.lineage if self.lineage else (None, 0, 0)
            sseed, frac = sample if sample is not None else (0, 1.0)
            g0 = self.global_row0() if frac < 1.0 else 0
            if self.nres or nl:
                G.glm_grad_mixed(self.X, self._res(self.y), self._res(self.sw), nl, spec.d if spec else self.d,
                                 spec.seed if spec else 0, r0, coef_eff, intercept, loss, ws,
                                 res_row0=g0, t_dev=t_dev, sample_seed=sseed, fraction=frac)
            else:
                ws.out.zero_()
            if self.spill is not None:
                cf = G._coef_buf(coef_eff, ws.dpad, self.device, intercept=intercept)
                wss = self.ws_stream

                def chunk(Xc, off):
                    rows = Xc.shape[0]
                    G.glm_grad_mixed(Xc, self._chunk_rows(self.y, off, rows), self._chunk_rows(self.sw, off, rows),
                                     0, self.d, 0, 0, cf, None, loss, wss, res_row0=g0 + self.nres + off,
                                     t_dev=t_dev, sample_seed=sseed, fraction=frac)
                    ws.out.add_(wss.out)
                self.spill.run(chunk)
            self.passes += 1
            return ws.out
        if self.overlap is not None:
            return self._pass_overlapped(coef_eff, intercept, loss)
        filled = False
        if self.X.shape[0]:
            G.glm_grad(self.X, self.y, self.sw, coef_eff, intercept, loss, ws)
            filled = True
        if self.lineage:
            spec, r0, nl = self.lineage
            G.glm_grad_synth(nl, self.ld, spec.d, spec.seed, r0, spec.wtrue, spec.btrue, coef_eff,
                             intercept, loss, ws, accumulate=filled)
            filled = True
        if not filled:
            ws.out.zero_()
        self.passes += 1
        return ws.out

    def _pass_overlapped(self, coef_eff, intercept, loss):
        side, ws_l = self.overlap
        ws = self.ws
        main = torch.cuda.current_stream(self.device)
        cf = G._coef_buf(coef_eff, ws.dpad, self.device, intercept=intercept)   # operand ready on main
        side.wait_stream(main)
        spec, r0, nl = self.lineage
        with torch.cuda.stream(side):
            G.glm_grad_synth(nl, self.ld, spec.d, spec.seed, r0, spec.wtrue, spec.btrue, cf, None, loss, ws_l)
        G.glm_grad(self.X, self.y, self.sw, cf, None, loss, ws)
        main.wait_stream(side)
        ws.out += ws_l.out
        self.passes += 1
        return ws.out

    def pass_torch(self, coef_eff: torch.Tensor, intercept: float, loss: int, it: int = 1,
                   sample: tuple | None = None) -> torch.Tensor:
        dpad = self.ld
        acc = torch.zeros(dpad + 3, dtype=torch.float64, device=self.device)
        c = coef_eff.to(self.device, torch.float64)[: self.ld]
        sampled = sample is not None and sample[1] < 1.0
        g0 = self.global_row0() if sampled else 0

        def block(X, base):
            n = X.shape[0]
            for a in range(0, n, self.chunk):
                b = min(n, a + self.chunk)
                Xc = X[a:b].to(self.device, torch.float64)
                yc = self.y[base + a:base + b].to(torch.float64)
                wc = None if self.sw is None else self.sw[base + a:base + b].to(torch.float64)
                if sampled:
                    keep = G.sample_mask(sample[0], it, torch.arange(g0 + base + a, g0 + base + b),
                                         sample[1]).to(self.device)
                    wc = keep.to(torch.float64) if wc is None else wc * keep
                acc.add_(G.glm_grad_torch(Xc, yc, wc, c, intercept, loss))
        block(self.X, 0)
        if self.spill is not None:
            self.spill.run(lambda Xc, off: block(Xc, self.nres + off))
        self.passes += 1
        return acc

    @traced("glm.pass")
    def loss_grad(self, coef_eff: np.ndarray, intercept: float, loss: int):
        """Global (loss_sum, grad (d), grad_intercept, weight_sum) as fp64 numpy."""
        ct = torch.from_numpy(np.ascontiguousarray(coef_eff, dtype=np.float64))
        if self.kernel:
            cf = torch.zeros(self.ws.dpad, dtype=torch.float32)
            cf[: self.d] = ct.float()
            out = self.pass_device(cf.to(self.device), intercept, loss)
            dpad = self.ws.dpad
        else:
            cf = torch.zeros(self.ld, dtype=torch.float64)
            cf[: self.d] = ct
            out = self.pass_torch(cf, intercept, loss)
            dpad = self.ld
        self.comm.all_reduce(out)
        o = out.cpu().numpy()
        return float(o[dpad + 1]), o[: self.d].copy(), float(o[dpad]), float(o[dpad + 2])


class SparseGlmData:
    """This rank's CSR rows for the GLM solvers (HashingTF / CountVectorizer features):
    margins and X^T r by the sparse kernels (ops/sparse.py), never densified.  Spark's
    standardization is a per-column scale without centering, so sparsity is kept.
    Provides the interface GlmObjective / fit_glm use (d, comm, moments, loss_grad)."""

    kernel = False           # no device-resident SGD trainer for sparse rows
    lineage = None

    def __init__(self, comm, feat: C.SparseVectorColumn, y: torch.Tensor, sw: torch.Tensor | None = None):
        from ..ops.sparse import SparseRows
        self.comm = comm
        self.rows = SparseRows(feat.indptr, feat.indices, feat.values, feat.size)
        self.device = self.rows.device
        self.d = int(feat.size)
        self.y = y.to(self.device)
        self.sw = None if sw is None else sw.to(self.device)
        self.n_local = self.rows.n
        self.n = int(comm.sum_scalar(self.n_local))
        self.passes = 0

    def moments(self):
        w = None if self.sw is None else self.sw.to(torch.float32)
        s1 = self.rows.colsum(w)
        s2 = self.rows.colsum(w, square=True)
        wd = torch.ones(self.n_local, dtype=torch.float64, device=self.device) if self.sw is None \
            else self.sw.to(torch.float64)
        yd = self.y.to(torch.float64)
        full = torch.cat([s1, s2, torch.stack([wd.sum(), (wd * yd).sum(), (wd * yd * yd).sum()])]).contiguous()
        self.comm.all_reduce(full)
        full = full.cpu().numpy()
        d = self.d
        s1, s2, W, ys1, ys2 = full[:d], full[d:2 * d], full[2 * d], full[2 * d + 1], full[2 * d + 2]
        mean = s1 / max(W, 1e-300)
        var = np.maximum((s2 - W * mean * mean) / max(W - 1.0, 1e-300), 0.0)
        ymean = ys1 / max(W, 1e-300)
        yvar = max((ys2 - W * ymean * ymean) / max(W - 1.0, 1e-300), 0.0)
        return mean, var, W, ymean, yvar

    sample_state = None          # (seed, fraction, iteration) while a mini-batch SGD fit runs
    _row0 = None

    def global_row0(self) -> int:
        if self._row0 is None:
            counts = self.comm.all_gather_object(int(self.n_local))
            self._row0 = int(sum(counts[: self.comm.rank]))
        return self._row0

    @traced("glm.pass")
    def loss_grad(self, coef_eff: np.ndarray, intercept: float, loss: int):
        ct = torch.from_numpy(np.ascontiguousarray(coef_eff, dtype=np.float64))
        sw = self.sw
        st = self.sample_state
        if st is not None and st[1] < 1.0:
            g0 = self.global_row0()
            keep = G.sample_mask(st[0], st[2], torch.arange(g0, g0 + self.n_local), st[1]).to(self.device)
            sw = keep.to(torch.float64) if sw is None else sw.to(torch.float64) * keep
        out = self.rows.loss_grad(ct, intercept, loss, self.y, sw)
        self.comm.all_reduce(out)
        self.passes += 1
        o = out.cpu().numpy()
        d = self.d
        return float(o[d + 1]), o[:d].copy(), float(o[d]), float(o[d + 2])


def make_glm_data(comm, feat: C.Column, y: torch.Tensor, sw: torch.Tensor | None = None):
    """GlmData for dense / lineage features, SparseGlmData for CSR features."""
    if isinstance(feat, C.SparseVectorColumn):
        return SparseGlmData(comm, feat, y, sw)
    return GlmData(comm, feat, y, sw)


@dataclass
class GlmResult:
    coef: np.ndarray
    intercept: float
    history: list = field(default_factory=list)
    iterations: int = 0
    converged: bool = False
    seconds: float = 0.0
    passes: int = 0
    setup_seconds: float = 0.0


class GlmObjective:
    """Spark-ML objective over standardised coefficients (see module docstring)."""

    def __init__(self, data: GlmData, loss: str, reg: float, alpha: float, fit_intercept: bool,
                 standardization: bool, std: np.ndarray):
        self.data, self.loss = data, LOSS_ID[loss]
        self.reg, self.alpha = float(reg), float(alpha)
        self.fi, self.stdz = fit_intercept, standardization
        self.std = std
        self.inv_std = np.where(std > 0, 1.0 / np.where(std > 0, std, 1.0), 0.0)
        self.W = None
        d = data.d
        self.l2 = self.reg * (1.0 - self.alpha)
        # penalty weights on b~ (per coordinate)
        if self.stdz:
            self.pen2 = np.full(d, self.l2)
            self.pen1 = np.full(d, self.reg * self.alpha)
        else:
            self.pen2 = self.l2 * self.inv_std ** 2
            self.pen1 = self.reg * self.alpha * self.inv_std

    def split(self, x):
        d = self.data.d
        return x[:d], (x[d] if self.fi else 0.0)

    def smooth(self, x):
        """Data term + L2 part: value and gradient (L1 handled by OWL-QN)."""
        bt, b = self.split(x)
        ls, g, gb, W = self.data.loss_grad(bt * self.inv_std, b, self.loss)
        self.W = W
        f = ls / W + 0.5 * float(np.sum(self.pen2 * bt * bt))
        gx = g * self.inv_std / W + self.pen2 * bt
        if self.fi:
            return f, np.concatenate([gx, [gb / W]])
        return f, gx


def _initial_intercept(loss: str, fit_intercept: bool, ymean: float, init_intercept=None) -> float:
    if not fit_intercept:
        return 0.0
    if init_intercept is not None:
        return float(init_intercept)
    if loss == "logistic" and 0 < ymean < 1:
        return math.log(ymean / (1 - ymean))
    if loss == "squared":
        return float(ymean)
    return 0.0


def _first_step_out(loss: str, b0: float, s1, syx, W: float, wy: float, wyy: float):
    """[grad | sum r | loss | W] of the pass at the initial iterate (all coefficients 0,
    every margin = b0) from the fused stats, or None when it is not a closed form."""
    if loss == "logistic":
        p = 1.0 / (1.0 + math.exp(-b0))
        sp = max(b0, 0.0) + math.log1p(math.exp(-abs(b0)))
        return p * s1 - syx, p * W - wy, sp * W - b0 * wy
    if loss == "hinge":
        if abs(b0) >= 1.0:
            return None
        # every row active: r = -(2y - 1) w
        return s1 - 2.0 * syx, W - 2.0 * wy, W - b0 * (2.0 * wy - W)
    return b0 * s1 - syx, b0 * W - wy, 0.5 * (b0 * b0 * W - 2.0 * b0 * wy + wyy)


def fit_sgd(data: GlmData, loss: str, reg=0.0, alpha=0.0, fit_intercept=True, standardization=True,
            max_iter=100, tol=1e-6, step_size=1.0, mini_batch_fraction=1.0, seed=0, init_intercept=None,
            ckpt=None, check_every: int = 10) -> GlmResult:
    """``solver='sgd'`` fit on the device (mllib GradientDescent semantics: step
    stepSize/sqrt(t), per-iteration Bernoulli mini-batch of ``mini_batch_fraction`` keyed
    on (seed, t, global row), L2 shrink + L1 soft-threshold updater).

    The summarizer pass is fused with the first iteration's gradient (one pass over the
    rows instead of two, ``GlmData.stats``); every later iteration is one fused gradient
    pass + one all-reduce + an on-device update, graph-replayed, with no host sync except
    a convergence probe every ``check_every`` iterations when ``tol > 0``."""
    t0 = time.time()
    frac = float(mini_batch_fraction)
    G.sample_threshold(frac)                        # validates the fraction
    last = ckpt.latest() if ckpt is not None else None
    st = data.stats() if (frac >= 1.0 and last is None and max_iter > 0) else None
    if st is not None:
        s1, s2, syx, W, wy, wyy = st
        mean = s1 / max(W, 1e-300)
        var = np.maximum((s2 - W * mean * mean) / max(W - 1.0, 1e-300), 0.0)
        ymean = wy / max(W, 1e-300)
    else:
        mean, var, W, ymean, _ = data.moments()
    std = np.sqrt(var)
    # mllib GradientDescent starts from all-zero weights, intercept included (the L-BFGS
    # path's log-odds / mean start is a Spark ML LogisticRegression convention, not mllib's)
    b0 = float(init_intercept) if (fit_intercept and init_intercept is not None) else 0.0
    sgd = DeviceSGD(data, loss, reg, fit_intercept, step_size, standardization, std, elastic_net=alpha,
                    mini_batch_fraction=frac, seed=seed, init_intercept=b0)
    setup_s = time.time() - t0
    done = 0
    if last is not None and last[1]["x"].shape[0] == data.d + (1 if fit_intercept else 0):
        done = int(last[0])
        sgd.set_state(last[1]["x"], done)
    elif st is not None:
        first = _first_step_out(loss, b0, s1, syx, W, wy, wyy)
        if first is not None:
            sgd.apply_first_step(*first, W)
    converged = False
    while sgd.t < max_iter:
        progress.iteration(sgd.t, max_iter)
        sgd.step()
        if (tol > 0 or ckpt is not None) and sgd.t % check_every == 0:
            h = sgd.loss_hist[max(0, sgd.t - 2):sgd.t].cpu().numpy()
            if ckpt is not None and ckpt.due(sgd.t):
                ckpt.save(sgd.t, {"x": sgd.state()})
            if tol > 0 and len(h) == 2 and abs(h[0] - h[1]) / max(abs(h[1]), 1e-12) < tol:
                converged = True
                break
    if ckpt is not None:
        ckpt.clear()
    res = sgd.result()
    res.converged = converged
    res.seconds = time.time() - t0
    res.setup_seconds = setup_s
    res.passes = data.passes
    return res


def fit_glm(data: GlmData, loss: str, reg=0.0, alpha=0.0, fit_intercept=True, standardization=True,
            max_iter=100, tol=1e-6, solver="auto", step_size=1.0, mini_batch_fraction=1.0, seed=0,
            init_intercept=None, ckpt=None) -> GlmResult:
    if solver in ("sgd", "gd") and isinstance(data, GlmData):
        return fit_sgd(data, loss, reg, alpha, fit_intercept, standardization, max_iter, tol, step_size,
                       mini_batch_fraction, seed, init_intercept, ckpt)
    t0 = time.time()
    mean, var, W, ymean, yvar = data.moments()
    std = np.sqrt(var)
    obj = GlmObjective(data, loss, reg, alpha, fit_intercept, standardization, std)
    d = data.d
    x0 = np.zeros(d + (1 if fit_intercept else 0))
    if fit_intercept:
        if init_intercept is not None:
            x0[-1] = init_intercept
        elif loss == "logistic" and 0 < ymean < 1:
            x0[-1] = math.log(ymean / (1 - ymean))
        elif loss == "squared":
            x0[-1] = ymean
    done = 0
    last = ckpt.latest() if ckpt is not None else None
    if last is not None and last[1]["x"].shape == x0.shape:
        done, x0 = last[0], last[1]["x"]            # warm restart from the checkpointed iterate

    def save(it, x, f):
        if ckpt is not None and ckpt.due(done + it):
            ckpt.save(done + it, {"x": np.asarray(x)})
    left = max(max_iter - done, 0)
    if solver in ("sgd", "gd"):
        res = _sgd(obj, x0, left, step_size, mini_batch_fraction, seed, tol)
    elif reg * alpha > 0:
        l1 = np.concatenate([obj.pen1, [0.0]]) if fit_intercept else obj.pen1
        r = optim.owlqn(obj.smooth, x0, l1, max_iter=left, tol=tol, callback=save)
        res = GlmResult(r.x, 0.0, r.history, done + r.iterations, r.converged)
    else:
        r = optim.lbfgs(obj.smooth, x0, max_iter=left, tol=tol, callback=save)
        res = GlmResult(r.x, 0.0, r.history, done + r.iterations, r.converged)
    if ckpt is not None:
        ckpt.clear()                     # finished: a later fit must not resume from this run
    bt, b = obj.split(res.coef)
    res.coef = bt * obj.inv_std
    res.intercept = float(b)
    res.seconds = time.time() - t0
    res.passes = data.passes
    return res


def _sgd(obj: GlmObjective, x0, max_iter, step, frac, seed, tol) -> GlmResult:
    """Host-driven minibatch SGD for CSR rows (Spark mllib GradientDescent: step/sqrt(t)
    schedule, per-iteration Bernoulli sample of ``frac`` keyed on (seed, t, global row) --
    the same draw as the device path)."""
    x = x0.copy()
    hist = []
    for t in range(1, max_iter + 1):
        progress.iteration(t - 1, max_iter)
        obj.data.sample_state = (int(seed), float(frac), t)
        f, g = obj.smooth(x)
        hist.append(f)
        x = x - (step / math.sqrt(t)) * g
        if len(hist) > 1 and abs(hist[-2] - hist[-1]) / max(abs(hist[-1]), 1e-12) < tol * 1e-3:
            break
    obj.data.sample_state = None
    return GlmResult(x, 0.0, hist, len(hist), False)


class DeviceSGD:
    """Device-resident gradient-descent stepper (no host sync per step).

    One ``step()`` = one fused pass over every local row (resident + lineage; with
    ``mini_batch_fraction < 1`` an in-kernel Bernoulli mask keyed on (seed, t, global row)),
    one all-reduce of a (D+3) fp64 vector, and an on-device update
    b~ <- prox_l1(b~ - eta_t (grad/W + l2 * b~)), eta_t = stepSize / sqrt(t), where W is
    the (sampled) weight sum -- mllib GradientDescent with its Squared-L2 / L1 updaters.
    This is the ``solver='sgd'`` path of LogisticRegression / LinearSVC / LinearRegression.

    Launch structure: after two eager steps a step is captured into HIP graphs.  With one
    rank the whole step (pass, update) is one graph; with several ranks the pass and the
    update are two graphs around the RCCL all-reduce, which runs eagerly on the same stream
    (stream-ordered, no host sync) -- the collective is never captured, so graph replay
    never depends on RCCL's capture support.
    """

    def __init__(self, data: GlmData, loss: str = "logistic", reg: float = 0.0, fit_intercept=True,
                 step_size: float = 1.0, standardization: bool = True, std: np.ndarray | None = None,
                 elastic_net: float = 0.0, mini_batch_fraction: float = 1.0, seed: int = 0,
                 init_intercept: float = 0.0):
        self.data, self.loss = data, LOSS_ID[loss]
        dev = data.device
        dpad = data.ws.dpad if data.kernel else data.ld
        self.dpad = dpad
        inv = np.ones(data.d) if std is None else np.where(std > 0, 1.0 / np.where(std > 0, std, 1.0), 0.0)
        self.inv_std = torch.zeros(dpad, dtype=torch.float64, device=dev)
        self.inv_std[: data.d] = torch.from_numpy(inv).to(dev)
        a = float(elastic_net)
        l2, l1 = float(reg) * (1.0 - a), float(reg) * a
        # penalties on the standardised coefficients b~ (standardization=true) or on b
        self.l2 = l2 if standardization else 0.0
        self.l2v = (l2 * self.inv_std ** 2) if not standardization else None
        self.l1 = l1 if standardization else 0.0
        self.l1v = (l1 * self.inv_std) if (not standardization and l1 > 0) else None
        self.bt = torch.zeros(dpad, dtype=torch.float64, device=dev)      # standardised coefficients
        self.b = torch.full((1,), float(init_intercept) if fit_intercept else 0.0, dtype=torch.float64, device=dev)
        # kernel operand: effective fp32 coefficients followed by the intercept
        self.coef_eff = torch.zeros(dpad + 1, dtype=torch.float32, device=dev)
        self.coef_eff[dpad] = float(self.b[0])
        self.fi = fit_intercept
        self.step_size = float(step_size)
        self.fraction = float(mini_batch_fraction)
        G.sample_threshold(self.fraction)
        self.sample = (int(seed), self.fraction) if self.fraction < 1.0 else None
        self.t = 0
        self.loss_hist = torch.zeros(1024, dtype=torch.float64, device=dev)
        self.t_dev = torch.zeros(1, dtype=torch.int64, device=dev)      # device step counter
        self._graphs = None
        self._graph_failed = False
        self._eager_steps = 0
        self._first_buf = None
        self.passes = 0

    # ---------------------------------------------------------------- state
    def state(self) -> np.ndarray:
        """[b~ (d) | intercept] on the host (checkpoint format of fit_glm)."""
        x = self.bt[: self.data.d].cpu().numpy()
        return np.concatenate([x, self.b.cpu().numpy()]) if self.fi else x

    def set_state(self, x: np.ndarray, t: int) -> None:
        d = self.data.d
        self.bt.zero_()
        self.bt[:d] = torch.from_numpy(np.asarray(x[:d], dtype=np.float64)).to(self.bt.device)
        if self.fi:
            self.b.fill_(float(x[d]))
        self.coef_eff[: self.dpad].copy_((self.bt * self.inv_std).to(torch.float32))
        self.coef_eff[self.dpad:].copy_(self.b.to(torch.float32))
        self.t = int(t)
        self.t_dev.fill_(int(t))
        self._ensure_hist()
        self._graphs = None

    def _ensure_hist(self):
        if self.t > self.loss_hist.shape[0]:
            n = self.loss_hist.shape[0]
            while n < self.t:
                n *= 2
            self.loss_hist = torch.cat([self.loss_hist, torch.zeros(n - self.loss_hist.shape[0],
                                                                     dtype=torch.float64, device=self.loss_hist.device)])
            self._graphs = None

    # ---------------------------------------------------------------- steps
    def apply_first_step(self, grad: np.ndarray, sum_r: float, loss_sum: float, W: float) -> None:
        """Iteration 1 from an already-reduced pass result at the initial iterate (the fused
        summarizer pass, fit_sgd): only the update runs."""
        out = torch.zeros(self.dpad + 3, dtype=torch.float64)
        out[: self.data.d] = torch.from_numpy(np.asarray(grad, dtype=np.float64))
        out[self.dpad:] = torch.tensor([sum_r, loss_sum, W], dtype=torch.float64)
        self._first_buf = out.to(self.bt.device)
        self.t += 1
        self._ensure_hist()
        self._update(self._first_buf)

    @traced("sgd.step")
    def step(self):
        """One iteration, stream-ordered on the device: pass -> all-reduce -> update."""
        self.t += 1
        self._ensure_hist()
        d = self.data
        self.passes += 1
        if d.kernel and self._graphs is not None:
            gp, gu = self._graphs
            gp.replay()
            if gu is not None:
                d.comm.all_reduce(self.data.ws.out)
                gu.replay()
            d.passes += 1
            return
        out = self._pass()
        d.comm.all_reduce(out)
        self._update(out)
        if d.kernel:
            self._eager_steps += 1
            self._maybe_capture()

    def _pass(self):
        if self.data.kernel:
            return self.data.pass_device(self.coef_eff, None, self.loss, t_dev=self.t_dev, sample=self.sample)
        return self.data.pass_torch(self.coef_eff[: self.dpad], float(self.b.item()), self.loss, it=self.t,
                                    sample=self.sample)

    def _update(self, out: torch.Tensor):
        if self.data.kernel:
            N.check(N.kernels().o3s_glm_sgd_update_dev(
                out.data_ptr(), self.dpad, self.bt.data_ptr(), self.b.data_ptr(), self.inv_std.data_ptr(),
                N.ptr(self.l2v), self.l2, N.ptr(self.l1v), self.l1, self.step_size, int(self.fi),
                self.coef_eff.data_ptr(), self.loss_hist.data_ptr(), int(self.loss_hist.shape[0]),
                self.t_dev.data_ptr(), torch.cuda.current_stream(self.data.device).cuda_stream), "glm_sgd_update")
            return
        eta = self.step_size / math.sqrt(self.t)
        W = out[self.dpad + 2]
        invW = torch.where(W > 0, 1.0 / W, torch.zeros_like(W))
        g = out[: self.dpad] * self.inv_std * invW
        g = g + (self.l2v if self.l2v is not None else self.l2) * self.bt
        v = self.bt - eta * g
        if self.l1v is not None or self.l1 > 0:
            sh = eta * (self.l1v if self.l1v is not None else self.l1)
            v = torch.sign(v) * torch.clamp(v.abs() - sh, min=0.0)
        self.bt.copy_(v)
        if self.fi:
            self.b -= eta * out[self.dpad] * invW
        self.coef_eff[: self.dpad].copy_((self.bt * self.inv_std).to(torch.float32))
        self.coef_eff[self.dpad:].copy_(self.b.to(torch.float32))
        self.loss_hist[self.t - 1:self.t].copy_(out[self.dpad + 1:self.dpad + 2] * invW)
        self.t_dev.fill_(self.t)

    # Steps whose pass streams more than this many bytes per rank are not captured: their
    # GPU time (>= ~40 us) already hides the host's launch sequence (the host runs ahead,
    # nothing in a step syncs), while capturing + instantiating costs ~12 ms of idle GPU
    # once per fit at 1B x 256 (rocprofv3 timeline, profiles/bench_fit_timeline_r3.json).
    GRAPH_MAX_BYTES = int(os.environ.get("O3S_SGD_GRAPH_MAX_BYTES", str(256 << 20)))

    def _maybe_capture(self):
        from ..runtime import faults
        mode = os.environ.get("O3S_SGD_GRAPH", "1")
        if self._graphs is not None or self._graph_failed or mode == "0" or self._eager_steps < 2:
            return
        if faults.launch_blocking():
            return
        d = self.data
        if d.spill is not None:               # host-streamed rows: copies + events stay eager
            return
        if mode != "force" and d.n_local * d.ld * 2 > self.GRAPH_MAX_BYTES:
            return
        if d.comm.world_size > 1 and mode != "all":
            # multi-rank: pass and update graphs around an eager RCCL all-reduce are opt-in
            # (O3S_SGD_GRAPH=all) until exercised on a multi-GPU RCCL group
            return
        try:
            if d.comm.world_size == 1:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    out = self._pass()
                    self._update(out)
                self._graphs = (g, None)
            else:
                gp, gu = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(gp):
                    out = self._pass()
                with torch.cuda.graph(gu):
                    self._update(out)
                self._graphs = (gp, gu)
            d.passes -= 1                    # the capture recorded, it did not run
        except Exception as e:  # noqa: BLE001 - fall back to eager launches
            log.warning("SGD step graph capture failed (%s); continuing eagerly", e)
            self._graph_failed = True
            self._graphs = None

    def result(self) -> GlmResult:
        coef = (self.bt * self.inv_std)[: self.data.d].cpu().numpy()
        hist = [float(x) for x in self.loss_hist[: self.t].cpu()]
        return GlmResult(coef, float(self.b.item()), hist, self.t, False, 0.0, self.data.passes)


# ------------------------------------------------------------------ multinomial
def _class_weights(yl: torch.Tensor, w: torch.Tensor | None, K: int) -> torch.Tensor:
    """fp64 per-class weight sums.  Integer bincount (LDS histogram) when unweighted; one
    masked reduction per class for few classes (a fp64-weighted bincount is a global-atomic
    histogram: 0.3 s for 20M rows into 10 bins on MI355X); index_add for many classes."""
    if w is None:
        return torch.bincount(yl, minlength=K)[:K].to(torch.float64)
    w64 = w.to(torch.float64)
    if K <= 64:
        return torch.stack([torch.where(yl == k, w64, 0.0).sum() for k in range(K)])
    return torch.zeros(K, dtype=torch.float64, device=yl.device).index_add_(0, yl, w64)


def fit_multinomial(comm, X: torch.Tensor, y: torch.Tensor, sw, num_classes: int, reg=0.0, alpha=0.0,
                    fit_intercept=True, standardization=True, max_iter=100, tol=1e-6, chunk=1 << 21):
    """Softmax regression (Spark 'multinomial' family).

    GPU, bf16 features, d <= 256, K <= 32: every objective/gradient evaluation is ONE
    fused pass (``glm_softmax_kernel``: margins and gradient on MFMA, X read once);
    otherwise chunked GEMMs.  Column moments: ``glm_colstats_kernel`` (bf16) or fp32
    chunks accumulated in fp64; class weights by bincount."""
    dev = X.device
    n, D = X.shape
    K = num_classes
    Xf_dtype = torch.float32 if X.is_cuda else torch.float64
    yl = y.to(dev).long()
    w = torch.ones(n, dtype=Xf_dtype, device=dev) if sw is None else sw.to(dev, Xf_dtype)
    fused = G.softmax_kernel_ok(X, K) and os.environ.get("O3S_SOFTMAX_KERNEL", "1") == "1"
    # moments
    if X.is_cuda and X.dtype == torch.bfloat16 and X.stride(1) == 1 and X.stride(0) % 8 == 0:
        base = torch.as_strided(X, (n, X.stride(0)), (X.stride(0), 1))     # the padded rows (zeros beyond d)
        cs = G.glm_colstats(base, None if sw is None else w.float().contiguous())
        ldp = X.stride(0)
        s1, s2 = cs[:D], cs[ldp:ldp + D]
    else:
        s1 = torch.zeros(D, dtype=torch.float64, device=dev)
        s2 = torch.zeros(D, dtype=torch.float64, device=dev)
        for a in range(0, n, chunk):
            Xc = X[a:a + chunk].to(torch.float64)
            wc = w[a:a + chunk].to(torch.float64)
            s1 += wc @ Xc
            s2 += wc @ (Xc * Xc)
    cnt = _class_weights(yl, None if sw is None else w, K)
    st = torch.cat([s1, s2, cnt])
    comm.all_reduce(st)
    st = st.cpu().numpy()
    W = st[2 * D:].sum()
    mean = st[:D] / W
    var = np.maximum((st[D:2 * D] - W * mean ** 2) / max(W - 1, 1e-300), 0)
    std = np.sqrt(var)
    inv = np.where(std > 0, 1.0 / np.where(std > 0, std, 1.0), 0.0)
    inv_t = torch.from_numpy(inv).to(dev, Xf_dtype)
    l2 = reg * (1 - alpha)
    pen2 = np.full(D, l2) if standardization else l2 * inv ** 2
    pen1 = np.full(D, reg * alpha) if standardization else reg * alpha * inv
    prior = st[2 * D:] / W

    y32 = yl.to(torch.int32).contiguous() if fused else None
    sw32 = None if (sw is None or not fused) else w.float().contiguous()

    def fg(x):
        Bt = x[: D * K].reshape(K, D)
        b = x[D * K:] if fit_intercept else np.zeros(K)
        if fused:
            Gk, gbk, lk = G.softmax_pass(X, y32, sw32, torch.from_numpy(Bt * inv[None, :]).to(dev, torch.float32),
                                         torch.from_numpy(b).to(dev, torch.float32))
            buf = torch.cat([Gk.T.reshape(-1), gbk, lk.reshape(1)])
            return _mn_finish(buf, Bt)
        Weff = torch.from_numpy(Bt.T * inv[:, None]).to(dev, Xf_dtype)      # [D, K]
        bt = torch.from_numpy(b).to(dev, Xf_dtype)
        G_ = torch.zeros((D, K), dtype=torch.float64, device=dev)
        gb = torch.zeros(K, dtype=torch.float64, device=dev)
        loss = torch.zeros(1, dtype=torch.float64, device=dev)
        for a in range(0, n, chunk):
            Xc = X[a:a + chunk].to(Xf_dtype)
            M = Xc @ Weff + bt
            lse = torch.logsumexp(M, dim=1)
            yc = yl[a:a + chunk]
            wc = w[a:a + chunk]
            loss += (wc * (lse - M.gather(1, yc[:, None]).squeeze(1))).to(torch.float64).sum()
            P = torch.softmax(M, dim=1)
            P[torch.arange(P.shape[0], device=dev), yc] -= 1.0
            R = P * wc[:, None]
            G_ += (Xc.T @ R).to(torch.float64)
            gb += R.sum(0).to(torch.float64)
        return _mn_finish(torch.cat([G_.reshape(-1), gb, loss]), Bt)

    def _mn_finish(buf, Bt):
        comm.all_reduce(buf)
        buf = buf.cpu().numpy()
        Gm = buf[: D * K].reshape(D, K).T * inv[None, :] / W     # [K, D]
        f = buf[-1] / W + 0.5 * float(np.sum(pen2[None, :] * Bt * Bt))
        Gm = Gm + pen2[None, :] * Bt
        g = Gm.reshape(-1)
        if fit_intercept:
            g = np.concatenate([g, buf[D * K:D * K + K] / W])
        return f, g

    x0 = np.zeros(D * K + (K if fit_intercept else 0))
    if fit_intercept:
        lp = np.log(np.maximum(prior, 1e-300))
        x0[D * K:] = lp - lp.mean()
    if reg * alpha > 0:
        l1 = np.concatenate([np.tile(pen1, K), np.zeros(K if fit_intercept else 0)])
        r = optim.owlqn(fg, x0, l1, max_iter=max_iter, tol=tol)
    else:
        r = optim.lbfgs(fg, x0, max_iter=max_iter, tol=tol)
    Bt = r.x[: D * K].reshape(K, D)
    B = Bt * inv[None, :]
    b = r.x[D * K:] if fit_intercept else np.zeros(K)
    if fit_intercept:
        b = b - b.mean()   # Spark centres the intercepts (identifiability)
    if reg == 0:
        B = B - B.mean(0, keepdims=True)
    return B, b, r
