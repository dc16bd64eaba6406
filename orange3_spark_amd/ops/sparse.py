"""Sparse (CSR) GLM passes: gfx950 kernels (csrc/sparse.hip) with PyTorch references.

``SparseRows`` keeps this rank's CSR rows plus a CSC copy built once (for X^T r) and the
column-piece plan of the gradient kernel; every pass is deterministic (fixed-order slab
and piece sums, no atomics)."""
from __future__ import annotations

import torch

from . import _native as N


class SparseRows:
    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, d: int):
        dev = values.device
        self.d = int(d)
        self.n = int(indptr.numel() - 1)
        self.indptr = indptr.to(dev, torch.int64).contiguous()
        self.idx = indices.to(dev, torch.int32).contiguous()
        self.val = values.to(dev, torch.float32).contiguous()
        self.device = dev
        self.kernel = dev.type == "cuda"
        self._csc = False
        if self.kernel:
            self.grid = max(1, min(N.num_cus(dev) * 8, (self.n + 31) // 32))
            self.slab = torch.empty(self.grid * 3, dtype=torch.float32, device=dev)

    def _build_csc(self):
        """CSC copy + gradient piece plan, built on first use (a transform needs neither)."""
        if self._csc:
            return
        dev = self.device
        nnz = int(self.val.numel())
        row_of = torch.repeat_interleave(torch.arange(self.n, device=dev, dtype=torch.int32),
                                         self.indptr[1:] - self.indptr[:-1])
        order = torch.argsort(self.idx.to(torch.int64), stable=True)   # CSC = entries sorted by column
        self.csc_rows = row_of[order].contiguous()
        self.csc_val = self.val[order].contiguous()
        cnt = torch.bincount(self.idx.to(torch.int64), minlength=self.d) if nnz else \
            torch.zeros(self.d, dtype=torch.int64, device=dev)
        self.col_ptr = torch.zeros(self.d + 1, dtype=torch.int64, device=dev)
        self.col_ptr[1:] = torch.cumsum(cnt, 0)
        if self.kernel:
            P = int(N.kernels().o3s_csc_piece())
            npc = (cnt + P - 1) // P                                     # pieces per column
            self.col_pieces = torch.zeros(self.d + 1, dtype=torch.int64, device=dev)
            self.col_pieces[1:] = torch.cumsum(npc, 0)
            self.npieces = int(self.col_pieces[-1])
            pcol = torch.repeat_interleave(torch.arange(self.d, device=dev), npc)
            k = torch.arange(self.npieces, device=dev) - self.col_pieces[:-1][pcol]
            self.plo = (self.col_ptr[:-1][pcol] + k * P).contiguous()
            self.pcnt = torch.minimum(torch.full_like(self.plo, P), self.col_ptr[1:][pcol] - self.plo).to(
                torch.int32).contiguous()
            self.psum = torch.empty(max(self.npieces, 1), dtype=torch.float32, device=dev)
        self._csc = True

    # ------------------------------------------------------------------ column sums
    def colsum(self, r: torch.Tensor | None, square: bool = False) -> torch.Tensor:
        """fp64 [d]: sum_i r_i x_ij (x_ij^2 if square; r None = 1)."""
        self._build_csc()
        out = torch.empty(self.d, dtype=torch.float64, device=self.device)
        if self.kernel:
            rr = None if r is None else r.to(torch.float32).contiguous()
            N.check(N.kernels().o3s_csc_colsum(self.plo.data_ptr(), self.pcnt.data_ptr(), self.npieces,
                                               self.col_pieces.data_ptr(), self.d, self.csc_rows.data_ptr(),
                                               self.csc_val.data_ptr(), N.ptr(rr), int(square),
                                               self.psum.data_ptr(), out.data_ptr(), N.stream_of(out)),
                    "csc_colsum")
            return out
        v = self.csc_val.to(torch.float64)
        v = v * v if square else v
        if r is not None:
            v = v * r.to(torch.float64)[self.csc_rows.long()]
        out.zero_()
        col = torch.repeat_interleave(torch.arange(self.d, device=self.device), self.col_ptr[1:] - self.col_ptr[:-1])
        return out.index_add_(0, col, v)

    # ------------------------------------------------------------------ margins / residuals
    def margins(self, coef: torch.Tensor, intercept: float) -> torch.Tensor:
        """fp32 [n]: x_i . coef + intercept."""
        if self.kernel:
            c = coef.to(self.device, torch.float32).contiguous()
            out = torch.empty(self.n, dtype=torch.float32, device=self.device)
            N.check(N.kernels().o3s_csr_glm(-1, self.indptr.data_ptr(), self.idx.data_ptr(), self.val.data_ptr(), self.n,
                                            c.data_ptr(), float(intercept), None, None, out.data_ptr(), None,
                                            self.grid, N.stream_of(out)), "csr_margin")
            return out
        return self._margins_f64(coef, intercept).float()

    def _margins_f64(self, coef, intercept):
        """CPU reference (fp64)."""
        c = coef.to(self.device, torch.float64)
        row = torch.repeat_interleave(torch.arange(self.n, device=self.device), self.indptr[1:] - self.indptr[:-1])
        m = torch.zeros(self.n, dtype=torch.float64, device=self.device)
        m.index_add_(0, row, self.val.to(torch.float64) * c[self.idx.long()])
        return m + float(intercept)

    def loss_grad(self, coef: torch.Tensor, intercept: float, loss: int, y: torch.Tensor,
                  w: torch.Tensor | None) -> torch.Tensor:
        """fp64 [grad (d) | sum r | loss | weight sum] of this rank's rows."""
        if not self.kernel:
            from .glm import _loss_terms
            m = self._margins_f64(coef, intercept)
            yd = y.to(torch.float64)
            wd = torch.ones_like(yd) if w is None else w.to(torch.float64)
            r, l = _loss_terms(m, yd, wd, loss)
            g = self.colsum(r)
            return torch.cat([g, torch.stack([r.sum(), l.sum(), wd.sum()])])
        c = coef.to(self.device, torch.float32).contiguous()
        r = torch.empty(self.n, dtype=torch.float32, device=self.device)
        yf = y.to(torch.float32).contiguous()
        wf = None if w is None else w.to(torch.float32).contiguous()
        N.check(N.kernels().o3s_csr_glm(int(loss), self.indptr.data_ptr(), self.idx.data_ptr(), self.val.data_ptr(),
                                        self.n, c.data_ptr(), float(intercept), yf.data_ptr(), N.ptr(wf),
                                        r.data_ptr(), self.slab.data_ptr(), self.grid, N.stream_of(r)), "csr_glm")
        g = self.colsum(r)
        tail = self.slab.view(self.grid, 3).to(torch.float64).sum(0)
        return torch.cat([g, tail])
