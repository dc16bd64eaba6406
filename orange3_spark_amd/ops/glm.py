"""GLM streaming ops: fused gradient/loss pass, margins, synthetic row generation.

GPU tensors dispatch to ``csrc/glm.hip``; CPU tensors use the PyTorch reference
implementations below (fp64 math), which also serve as the numerics oracle in the
tests (kernel vs plain fp32/fp64 PyTorch of the same op).

Loss ids match the kernel: 0 logistic (y in {0,1}), 1 hinge (y in {0,1}, LinearSVC),
2 squared (LinearRegression).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _native as N

LOSS_LOGISTIC, LOSS_HINGE, LOSS_SQUARED = 0, 1, 2
_MASK = 0xFFFFFFFF


def padded_width(d: int) -> int:
    """Row stride (elements) used for bf16 feature matrices: multiple of 8 (16 B)."""
    return max(8, (d + 7) // 8 * 8)


def layout(ld: int) -> tuple[int, int]:
    """(dpad, pstride) of the gradient kernel for row stride ``ld`` (mirrors o3s_glm_layout)."""
    nch = ld // 8
    lpr = 4
    while lpr < nch and lpr < 64:
        lpr <<= 1
    cpl = 1
    if nch > 64:
        need = (nch + 63) // 64
        cpl = 2
        while cpl < need:
            cpl <<= 1
    if cpl > 16:
        raise ValueError(f"feature dimension {ld} too large for the fused GLM kernel")
    dpad = lpr * cpl * 8
    return dpad, dpad + 4


# --------------------------------------------------------------------------- hashing
def _fmix32(h: torch.Tensor) -> torch.Tensor:
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _MASK
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _MASK
    return h ^ (h >> 16)


def row_keys(seed: int, rows: torch.Tensor) -> torch.Tensor:
    lo = rows & _MASK
    hi = rows >> 32
    inner = (lo * 0x9E3779B1 + hi * 0x7FEB352D + 0x165667B1) & _MASK
    return _fmix32((seed & _MASK) ^ _fmix32(inner))


def _mix24(h: torch.Tensor) -> torch.Tensor:
    """Torch twin of csrc/glm.hip ``mix24`` (bijective; v_mad_u32_u24 steps + xorshifts)."""
    h = h ^ (h >> 16)
    h = ((h & 0xFFFFFF) * 0xED5AD4 + h) & _MASK
    h = h ^ (h >> 15)
    return ((h & 0xFFFFFF) * 0x2C1B3C + h) & _MASK


def feat_keys(seed: int, rows: torch.Tensor) -> torch.Tensor:
    """Per-row feature keys (csrc/glm.hip ``feat_key``); labels use :func:`row_keys`."""
    lo = rows & _MASK
    hi = rows >> 32
    k = _mix24((lo + ((seed * 0x9E3779B1) & _MASK)) & _MASK)
    return _mix24(k ^ (((hi & 0xFFFFFF) * 0x7FEB35 + 0x165667) & _MASK))


def synth_features_torch(fk: torch.Tensor, ld: int, d: int) -> torch.Tensor:
    """bf16 [n, ld] features for feature keys ``fk`` (int64 [n], :func:`feat_keys`).

    Word i = mix24(fk + i*0x9E3779) gives features 4i..4i+3 (byte q -> column 4i+q) as
    (2b - 255)/256: 256 symmetric levels in (-1, 1), exact in bf16 (csrc/glm.hip
    ``synth_chunk``).  All ``ld`` columns are generated (synthetic widths are rounded up to
    a multiple of 8; the ground-truth weights of columns >= d are zero, so those are pure
    noise features).
    """
    n = fk.shape[0]
    words = torch.arange(ld // 4, dtype=torch.int64, device=fk.device)
    h = _mix24((fk[:, None] + words[None, :] * 0x9E3779) & _MASK)
    shifts = torch.arange(4, dtype=torch.int64, device=fk.device) * 8
    b = (h[:, :, None] >> shifts) & 0xFF
    return ((2 * b - 255).to(torch.float32) * (1.0 / 256.0)).reshape(n, ld).to(torch.bfloat16)


def synth_labels_torch(rk: torch.Tensor, margin_true: torch.Tensor) -> torch.Tensor:
    u = (_fmix32(rk ^ 0xA511E9B3) >> 8).to(torch.float32) * (1.0 / 16777216.0)
    return (u < torch.sigmoid(margin_true.to(torch.float32))).to(torch.float32)


def synth_truth(seed: int, d: int, ld: int | None = None) -> tuple[torch.Tensor, float]:
    """Ground-truth separating hyperplane for synthetic classification data."""
    ld = ld or padded_width(d)
    rng = np.random.default_rng(seed ^ 0x5EED)
    w = np.zeros(ld, dtype=np.float32)
    # features are U[-1,1) (var 1/3): scale so the true margin has std ~2
    w[:d] = rng.standard_normal(d).astype(np.float32) * np.float32(np.sqrt(12.0 / max(d, 1)))
    b = float(rng.standard_normal() * 0.25)
    return torch.from_numpy(w), b


def synth_glm(n: int, d: int, seed: int, row0: int = 0, device="cpu", ld: int | None = None,
              wtrue: torch.Tensor | None = None, btrue: float | None = None):
    """Materialise synthetic rows [row0, row0+n): (X bf16 [n, ld], y f32 [n])."""
    ld = ld or padded_width(d)
    if wtrue is None:
        wtrue, btrue = synth_truth(seed, d, ld)
    device = torch.device(device)
    X = torch.empty((n, ld), dtype=torch.bfloat16, device=device)
    y = torch.empty((n,), dtype=torch.float32, device=device)
    if n == 0:
        return X, y
    if device.type == "cuda":
        lib = N.kernels()
        wt = wtrue.to(device=device, dtype=torch.float32).contiguous()
        grid = N.grid_for(device, n, 256)
        N.check(lib.o3s_synth_glm(X.data_ptr(), ld, n, y.data_ptr(), seed & _MASK, row0,
                                  wt.data_ptr(), float(btrue), grid, N.stream_of(X)), "synth_glm")
        return X, y
    step = 1 << 16
    for s in range(0, n, step):
        e = min(n, s + step)
        rows = torch.arange(row0 + s, row0 + e, dtype=torch.int64)
        rk = row_keys(seed, rows)
        xs = synth_features_torch(feat_keys(seed, rows), ld, d)
        X[s:e] = xs
        y[s:e] = synth_labels_torch(rk, xs.float() @ wtrue.float() + btrue)
    return X, y


# --------------------------------------------------------------------------- gradient
def _loss_terms(m: torch.Tensor, y: torch.Tensor, w: torch.Tensor, loss: int):
    if loss == LOSS_LOGISTIC:
        r = (torch.sigmoid(m) - y) * w
        l = w * (torch.nn.functional.softplus(m) - y * m)
    elif loss == LOSS_HINGE:
        s = 2.0 * y - 1.0
        mg = 1.0 - s * m
        act = (mg > 0).to(m.dtype)
        r = -s * w * act
        l = w * mg * act
    else:
        e = m - y
        r = e * w
        l = 0.5 * w * e * e
    return r, l


def glm_grad_torch(X, y, sw, coef, intercept, loss: int) -> torch.Tensor:
    """fp64 reference: [grad (ld) | sum r | loss | weight sum]."""
    Xd = X.to(torch.float64)
    m = Xd @ coef.to(torch.float64)[: X.shape[1]] + float(intercept)
    yd = y.to(torch.float64)
    w = torch.ones_like(yd) if sw is None else sw.to(torch.float64)
    r, l = _loss_terms(m, yd, w, loss)
    g = Xd.T @ r
    return torch.cat([g, torch.stack([r.sum(), l.sum(), w.sum()])])


class GlmWorkspace:
    """Per-device scratch for the gradient pass (partial slabs + fp64 result)."""

    def __init__(self, device: torch.device, ld: int, grid: int | None = None):
        self.device = torch.device(device)
        self.ld = ld
        self.dpad, self.pstride = layout(ld)
        self.grid = grid or (N.num_cus(self.device) * 8 if self.device.type == "cuda" else 1)
        self.partial = torch.empty(self.grid * self.pstride, dtype=torch.float32, device=self.device)
        self.out = torch.empty(self.dpad + 3, dtype=torch.float64, device=self.device)


def glm_grad(X: torch.Tensor, y: torch.Tensor, sw: torch.Tensor | None, coef: torch.Tensor,
             intercept: float | None, loss: int, ws: GlmWorkspace | None = None,
             accumulate: bool = False) -> torch.Tensor:
    """Fused margin -> loss -> X^T r pass.  Returns fp64 [grad (dpad) | sum r | loss | wsum].

    ``coef`` is fp32 with at least ``ld`` entries (padded columns ignored).  With
    ``intercept=None`` it must be the device operand itself: dpad coefficients followed
    by the intercept (what DeviceSGD keeps on the GPU, so no host sync is needed).  The
    returned tensor aliases the workspace buffer when one is given; ``accumulate`` adds
    into it instead of overwriting.
    """
    ld = X.shape[1]
    if X.is_cuda:
        if X.dtype != torch.bfloat16 or not X.is_contiguous():
            raise TypeError("GPU GLM pass expects a contiguous bf16 feature matrix")
        ws = ws or GlmWorkspace(X.device, ld)
        cf = _coef_buf(coef, ws.dpad, X.device, intercept=intercept)
        lib = N.kernels()
        N.check(lib.o3s_glm_grad(loss, 0, X.data_ptr(), ld, X.shape[0], y.data_ptr(),
                                 N.ptr(sw), cf.data_ptr(), 0, 0, None, 0.0,
                                 ws.partial.data_ptr(), ws.grid, ws.out.data_ptr(), int(accumulate),
                                 N.stream_of(X)), "glm_grad")
        return ws.out
    if intercept is None:
        intercept = float(coef[-1])
    dpad, _ = layout(ld)
    ref = glm_grad_torch(X, y, sw, coef.to(torch.float64)[:ld], intercept, loss)
    out = torch.zeros(dpad + 3, dtype=torch.float64)
    out[:ld] = ref[:ld]
    out[dpad:] = ref[ld:]
    return out


def glm_grad_synth(n: int, ld: int, d: int, seed: int, row0: int, wtrue: torch.Tensor,
                   btrue: float, coef: torch.Tensor, intercept: float | None, loss: int,
                   ws: GlmWorkspace, accumulate: bool = False) -> torch.Tensor:
    """Gradient over synthetic rows regenerated in-kernel (lineage recompute)."""
    if ws.device.type == "cuda":
        cf = _coef_buf(coef, ws.dpad, ws.device, intercept=intercept)
        wt = _coef_buf(wtrue, ws.dpad, ws.device, slot=1, intercept=0.0)
        lib = N.kernels()
        N.check(lib.o3s_glm_grad(loss, 1, None, ld, n, None, None, cf.data_ptr(),
                                 seed & _MASK, row0, wt.data_ptr(), float(btrue),
                                 ws.partial.data_ptr(), ws.grid, ws.out.data_ptr(), int(accumulate),
                                 torch.cuda.current_stream(ws.device).cuda_stream), "glm_grad_synth")
        return ws.out
    X, y = synth_glm(n, d, seed, row0, "cpu", ld, wtrue, btrue)
    out = glm_grad(X, y, None, coef, intercept, loss)
    if accumulate and ws is not None and getattr(ws, "out", None) is not None:
        ws.out += out
        return ws.out
    return out


# waves/SIMD the mixed kernel is register-allocated for (2 or 3; tools/sweep_glm_mixed.sh)
MIX_WAVES = int(os.environ.get("O3S_GLM_MIX_WAVES", "3"))
# waves/SIMD the fused summarizer kernel is compiled for (2: no spill, 3: 6-VGPR spill)
STATS_WAVES = int(os.environ.get("O3S_GLM_STATS_WAVES", "2"))
# rows per launch slice of a mixed pass (csrc/glm.hip o3s_glm_grad_mixed ``splits``): long
# passes restart their grid-stride walk every this many rows, at most 16 slices
MIX_SLICE_ROWS = int(os.environ.get("O3S_GLM_MIX_SLICE_ROWS", str(64 << 20)))


def mix_splits(n_rows: int) -> int:
    return max(1, min(16, n_rows // max(1, MIX_SLICE_ROWS)))


def sample_threshold(fraction: float) -> int:
    """miniBatchFraction -> the kernels' 24-bit keep threshold (>= 2^24: keep every row)."""
    f = float(fraction)
    if not 0.0 < f <= 1.0:
        raise ValueError(f"miniBatchFraction must be in (0, 1], got {fraction}")
    return 1 << 24 if f >= 1.0 else max(1, int(round(f * (1 << 24))))


def sample_key(seed: int, it: int) -> int:
    """Torch/host twin of csrc/glm.hip ``sample_key`` (per-iteration sampling key)."""
    t = torch.tensor([(int(it) * 0x9E3779B1 + 0x7F4A7C15) & _MASK], dtype=torch.int64)
    return int(_fmix32((int(seed) & _MASK) ^ _fmix32(t))[0])


def sample_mask(seed: int, it: int, grows: torch.Tensor, fraction: float) -> torch.Tensor:
    """Rows kept by iteration ``it``'s mini-batch (bool per global row index): the same
    draw as the GLM kernels' ``RowSampler``, so CPU and GPU paths select identical sets."""
    thr = sample_threshold(fraction)
    if thr >= 1 << 24:
        return torch.ones(grows.shape[0], dtype=torch.bool, device=grows.device)
    return (row_keys(sample_key(seed, it), grows.to(torch.int64)) >> 8) < thr


def glm_grad_mixed(X: torch.Tensor, y: torch.Tensor, sw: torch.Tensor | None, n_lin: int, d: int,
                   seed: int, row0: int, coef: torch.Tensor, intercept: float | None, loss: int,
                   ws: GlmWorkspace, res_row0: int = 0, t_dev: torch.Tensor | None = None,
                   sample_seed: int = 0, fraction: float = 1.0) -> torch.Tensor:
    """Resident rows of ``X`` plus ``n_lin`` lineage rows (global rows ``row0..``) in ONE
    launch (csrc/glm.hip ``glm_grad_mixed_kernel``): memory-bound and VALU-bound tiles
    are interleaved inside every wave so both resources stay busy.  ``y``/``sw`` are the
    materialised label/weight columns of all ``X.shape[0] + n_lin`` rows.  Overwrites
    ``ws.out``.

    ``fraction < 1`` keeps each row with that probability (mini-batch SGD), keyed on
    (``sample_seed``, iteration ``t_dev[0] + 1`` -- 1 when ``t_dev`` is None, global row:
    ``res_row0 + i`` for resident row i, ``row0 + j`` for lineage row j)."""
    ld = X.shape[1]
    nr = X.shape[0]
    if y.shape[0] != nr + n_lin or (sw is not None and sw.shape[0] != nr + n_lin):
        raise ValueError("label / weight columns must cover the resident and lineage rows")
    thr = sample_threshold(fraction)
    if ws.device.type != "cuda":
        Xl, _ = synth_glm(n_lin, d, seed, row0, "cpu", ld, torch.zeros(ld), 0.0)
        w = sw
        if thr < 1 << 24:
            it = int(t_dev[0]) + 1 if t_dev is not None else 1
            grows = torch.cat([torch.arange(res_row0, res_row0 + nr), torch.arange(row0, row0 + n_lin)])
            keep = sample_mask(sample_seed, it, grows, fraction).to(torch.float64)
            w = keep if sw is None else sw.to(torch.float64) * keep
        return glm_grad(torch.cat([X, Xl]), y, w, coef, intercept, loss)
    if X.dtype != torch.bfloat16 or not X.is_contiguous() or not y.is_contiguous():
        raise TypeError("GPU GLM pass expects a contiguous bf16 feature matrix")
    cf = _coef_buf(coef, ws.dpad, ws.device, intercept=intercept)
    N.check(N.kernels().o3s_glm_grad_mixed(loss, X.data_ptr(), ld, nr, y.data_ptr(), N.ptr(sw),
                                           cf.data_ptr(), seed & _MASK, row0, n_lin, ws.partial.data_ptr(),
                                           ws.grid, ws.out.data_ptr(), MIX_WAVES, int(res_row0),
                                           N.ptr(t_dev), int(sample_seed) & _MASK, thr, mix_splits(nr + n_lin),
                                           N.stream_of(X)),
            "glm_grad_mixed")
    return ws.out


def glm_stats_mixed(X: torch.Tensor, y: torch.Tensor, sw: torch.Tensor | None, n_lin: int, d: int,
                    seed: int, row0: int, grid: int | None = None) -> torch.Tensor | None:
    """Summarizer pass fused with the first gradient (csrc/glm.hip ``glm_stats_mixed_kernel``)
    over the resident rows of ``X`` and ``n_lin`` lineage rows: fp64 [s1 (dpad) | s2 (dpad) |
    syx (dpad) | sum w | sum w y | sum w y^2] with s1 = sum w x, s2 = sum w x^2, syx =
    sum w y x.  Returns None when the layout has no fused instantiation (ld > 2048)."""
    ld = X.shape[1]
    nr = X.shape[0]
    dpad, _ = layout(ld)
    if y.shape[0] != nr + n_lin or (sw is not None and sw.shape[0] != nr + n_lin):
        raise ValueError("label / weight columns must cover the resident and lineage rows")
    if X.device.type != "cuda":
        return glm_stats_torch(X, y, sw, n_lin, d, seed, row0)
    grid = grid or N.num_cus(X.device) * 16   # 16 blocks per CU: 45.9 vs 47.3 ms at 8 (profiles/glm_stats_unweighted_r3.json)
    pstride = 3 * dpad + 4
    partial = torch.empty(grid * pstride, dtype=torch.float32, device=X.device)
    out = torch.empty(3 * dpad + 3, dtype=torch.float64, device=X.device)
    rc = N.kernels().o3s_glm_stats_mixed(X.data_ptr(), ld, nr, y.data_ptr(), N.ptr(sw), seed & _MASK, row0,
                                         n_lin, partial.data_ptr(), grid, out.data_ptr(), STATS_WAVES, N.stream_of(X))
    if rc == -2:
        return None
    N.check(rc, "glm_stats_mixed")
    return out


def glm_stats_torch(X, y, sw, n_lin=0, d=None, seed=0, row0=0) -> torch.Tensor:
    """fp64 reference of :func:`glm_stats_mixed`."""
    ld = X.shape[1]
    dpad, _ = layout(ld)
    if n_lin:
        Xl, _ = synth_glm(n_lin, d or ld, seed, row0, "cpu", ld, torch.zeros(ld), 0.0)
        X = torch.cat([X.cpu(), Xl])
    Xd = X.to(torch.float64).cpu()
    yd = y.to(torch.float64).cpu()
    w = torch.ones_like(yd) if sw is None else sw.to(torch.float64).cpu()
    out = torch.zeros(3 * dpad + 3, dtype=torch.float64)
    out[:ld] = w @ Xd
    out[dpad:dpad + ld] = w @ (Xd * Xd)
    out[2 * dpad:2 * dpad + ld] = (w * yd) @ Xd
    out[3 * dpad:] = torch.stack([w.sum(), (w * yd).sum(), (w * yd * yd).sum()])
    return out


_COEF_CACHE: dict = {}


def _coef_buf(coef: torch.Tensor, dpad: int, device, slot: int = 0,
              intercept: float | None = 0.0) -> torch.Tensor:
    """Kernel operand: fp32 [dpad coefficients (zero padded) | intercept] on ``device``.

    ``intercept=None`` means ``coef`` already is such an operand and is used as is.
    """
    if intercept is None:
        if coef.shape[0] != dpad + 1 or coef.dtype != torch.float32 or coef.device != torch.device(device):
            raise ValueError("coef operand must be fp32 [dpad + 1] on the pass device")
        return coef
    key = (str(device), dpad, slot)
    buf = _COEF_CACHE.get(key)
    if buf is None:
        buf = torch.zeros(dpad + 1, dtype=torch.float32, device=device)
        _COEF_CACHE[key] = buf
    k = min(coef.shape[0], dpad)
    buf[:k].copy_(coef[:k], non_blocking=True)
    if k < dpad:
        buf[k:dpad].zero_()
    buf[dpad] = float(intercept)
    return buf


def glm_margin(X: torch.Tensor, coef: torch.Tensor, intercept: float) -> torch.Tensor:
    """margins = X . coef + intercept (fp32 [n])."""
    ld = X.shape[1]
    if X.is_cuda and X.dtype == torch.bfloat16 and X.is_contiguous():
        dpad, _ = layout(ld)
        cf = torch.zeros(dpad, dtype=torch.float32, device=X.device)
        k = min(coef.shape[0], dpad)
        cf[:k] = coef[:k].to(X.device, torch.float32)
        out = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
        lib = N.kernels()
        grid = N.grid_for(X.device, X.shape[0], 64)
        N.check(lib.o3s_glm_margin(X.data_ptr(), ld, X.shape[0], cf.data_ptr(), float(intercept),
                                   out.data_ptr(), grid, N.stream_of(X)), "glm_margin")
        return out
    c = coef.to(X.device, torch.float64)[:ld]
    return (X.to(torch.float64) @ c + float(intercept)).to(torch.float32)


# --------------------------------------------------------------------------- multinomial
def softmax_kernel_ok(X: torch.Tensor, K: int) -> bool:
    return (X.is_cuda and X.dtype == torch.bfloat16 and X.dim() == 2 and X.stride(1) == 1
            and X.stride(0) % 8 == 0 and 1 <= X.shape[1] <= 256 and 1 <= K <= 32)


def softmax_pass(X: torch.Tensor, y: torch.Tensor, sw: torch.Tensor | None, W: torch.Tensor, b: torch.Tensor):
    """One fused multinomial pass over the rows of X (``glm_softmax_kernel``, csrc/glm.hip).

    X bf16 [n, d] (row stride a multiple of 8), y int32 labels, sw fp32 weights or None,
    W fp32 [K, d] effective coefficients, b fp32 [K].  Returns fp64 (G [K, d] = sum_i
    w_i (p_i - onehot(y_i)) x_i^T, sum_i w_i (p_i - onehot(y_i)) [K], sum_i w_i (lse_i -
    m_{i, y_i}))."""
    n, d = X.shape
    K = W.shape[0]
    dev = X.device
    D = 32 * (-(-d // 32))
    Wp = torch.zeros((32, D), dtype=torch.float32, device=dev)
    Wp[:K, :d] = W
    hi = Wp.to(torch.bfloat16)
    r1 = Wp - hi.float()
    mid = r1.to(torch.bfloat16)
    lo = (r1 - mid.float()).to(torch.bfloat16)
    Wsp = torch.stack([hi, mid, lo]).contiguous()
    bp = torch.zeros(32, dtype=torch.float32, device=dev)
    bp[:K] = b
    grid = N.num_cus(dev)
    pstride = 32 * D + 33
    partial = torch.empty(grid * 4 * pstride, dtype=torch.float32, device=dev)
    out = torch.empty(pstride, dtype=torch.float64, device=dev)
    yi = y if y.dtype == torch.int32 else y.to(torch.int32)
    N.check(N.kernels().o3s_glm_softmax(X.data_ptr(), n, X.stride(0), d, yi.contiguous().data_ptr(),
                                        N.ptr(None if sw is None else sw.float().contiguous()),
                                        Wsp.data_ptr(), bp.data_ptr(), K, partial.data_ptr(), grid,
                                        out.data_ptr(), N.stream_of(X)), "glm_softmax")
    return out[: 32 * D].view(32, D)[:K, :d], out[32 * D:32 * D + K], out[32 * D + 32]


def softmax_pass_torch(X, y, sw, W, b):
    """fp64 reference of :func:`softmax_pass`."""
    Xd = X.to(torch.float64)
    M = Xd @ W.to(torch.float64).T + b.to(torch.float64)
    lse = torch.logsumexp(M, 1)
    w = torch.ones(X.shape[0], dtype=torch.float64, device=X.device) if sw is None else sw.to(torch.float64)
    yl = y.long()
    P = torch.exp(M - lse[:, None])
    P[torch.arange(X.shape[0], device=X.device), yl] -= 1.0
    R = P * w[:, None]
    return R.T @ Xd, R.sum(0), (w * (lse - M.gather(1, yl[:, None]).squeeze(1))).sum()


# --------------------------------------------------------------------------- moments
def _colstats_out(ld: int, device, grid: int):
    dpad, _ = layout(ld)
    partial = torch.empty(grid * (2 * dpad + 2), dtype=torch.float32, device=device)
    out = torch.empty(2 * dpad + 1, dtype=torch.float64, device=device)
    return dpad, partial, out


def glm_colstats(X: torch.Tensor, sw: torch.Tensor | None = None) -> torch.Tensor:
    """fp64 [sum w x (ld) | sum w x^2 (ld) | sum w] over the rows of X."""
    ld = X.shape[1]
    if X.is_cuda and X.dtype == torch.bfloat16 and X.is_contiguous():
        grid = N.num_cus(X.device) * 4
        dpad, partial, out = _colstats_out(ld, X.device, grid)
        N.check(N.kernels().o3s_glm_colstats(0, X.data_ptr(), ld, X.shape[0], N.ptr(sw), 0, 0,
                                             partial.data_ptr(), grid, out.data_ptr(), N.stream_of(X)),
                "glm_colstats")
        return torch.cat([out[:ld], out[dpad:dpad + ld], out[2 * dpad:]])
    Xd = X.to(torch.float64)
    w = torch.ones(X.shape[0], dtype=torch.float64, device=X.device) if sw is None else sw.to(torch.float64)
    return torch.cat([w @ Xd, w @ (Xd * Xd), w.sum().reshape(1)])


def glm_colstats_synth(n: int, ld: int, d: int, seed: int, row0: int, device) -> torch.Tensor:
    device = torch.device(device)
    if device.type == "cuda":
        grid = N.num_cus(device) * 4
        dpad, partial, out = _colstats_out(ld, device, grid)
        N.check(N.kernels().o3s_glm_colstats(1, None, ld, n, None, seed & _MASK, row0, partial.data_ptr(), grid,
                                             out.data_ptr(), torch.cuda.current_stream(device).cuda_stream),
                "glm_colstats_synth")
        return torch.cat([out[:ld], out[dpad:dpad + ld], out[2 * dpad:]])
    X, _ = synth_glm(n, d, seed, row0, "cpu", ld, torch.zeros(ld), 0.0)
    return glm_colstats(X)
