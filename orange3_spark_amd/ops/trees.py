"""Tree histogram op: gfx950 kernel (csrc/trees.hip) with a PyTorch reference."""
from __future__ import annotations

import torch

from . import _native as N


def hist_kernel_ok(bins: torch.Tensor, B: int, S: int) -> bool:
    if not bins.is_cuda or bins.dtype != torch.uint8:
        return False
    F = bins.shape[1]
    fp = 4
    while fp < F and fp < 64:
        fp <<= 1
    return N.kernels().o3s_tree_hist_lds(fp, B, S) > 0


def node_hist(bins: torch.Tensor, order: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None,
              seg_lo: torch.Tensor, seg_hi: torch.Tensor, seg_node: torch.Tensor, n_nodes: int, B: int, S: int,
              cls: bool, chunk: int = 1 << 17) -> torch.Tensor:
    """Histograms [n_nodes, F, B, S] (fp32) of rows order[lo:hi] for each segment -> node.

    Segments are split into work items of <= ``chunk`` rows; the kernel writes one slab row
    per item and the rows are summed per node in item order (deterministic)."""
    F = bins.shape[1]
    dev = bins.device
    out = torch.zeros((n_nodes, F * B * S), dtype=torch.float32, device=dev)
    if seg_lo.numel() == 0:
        return out.view(n_nodes, F, B, S)
    lens = (seg_hi - seg_lo).clamp_min(0)
    nchunks = (lens + chunk - 1) // chunk
    nchunks = torch.where(lens > 0, nchunks, torch.zeros_like(nchunks))
    seg_id = torch.repeat_interleave(torch.arange(seg_lo.numel(), device=dev), nchunks)
    first = torch.cumsum(nchunks, 0) - nchunks
    k = torch.arange(seg_id.numel(), device=dev) - first[seg_id]
    it_lo = (seg_lo[seg_id] + k * chunk).to(torch.int64).contiguous()
    it_hi = torch.minimum(it_lo + chunk, seg_hi[seg_id].to(torch.int64)).contiguous()
    it_node = seg_node[seg_id].to(torch.int64)
    n_items = int(it_lo.numel())
    if n_items == 0:
        return out.view(n_nodes, F, B, S)
    if hist_kernel_ok(bins, B, S):
        slab = torch.empty((n_items, F * B * S), dtype=torch.float32, device=dev)
        yf = y.to(torch.float32).contiguous()
        wf = None if w is None else w.to(torch.float32).contiguous()
        N.check(N.kernels().o3s_tree_hist(bins.data_ptr(), bins.shape[0], F, B, S, int(cls),
                                          order.data_ptr(), yf.data_ptr(), N.ptr(wf), it_lo.data_ptr(),
                                          it_hi.data_ptr(), n_items, slab.data_ptr(), N.stream_of(bins)),
                "tree_hist")
        out.index_add_(0, it_node, slab)
        return out.view(n_nodes, F, B, S)
    # reference path (CPU / oversize bins): direct scatter-add per segment
    return hist_torch(bins, order, y, w, seg_lo, seg_hi, seg_node, n_nodes, B, S, cls)


def hist_torch(bins, order, y, w, seg_lo, seg_hi, seg_node, n_nodes, B, S, cls):
    F = bins.shape[1]
    dev = bins.device
    out = torch.zeros(n_nodes * F * B * S, dtype=torch.float64, device=dev)
    lens = (seg_hi - seg_lo).clamp_min(0)
    if int(lens.sum()) == 0:
        return out.view(n_nodes, F, B, S).float()
    pos = torch.cat([torch.arange(int(a), int(b), device=dev) for a, b in zip(seg_lo.tolist(), seg_hi.tolist())])
    node = torch.repeat_interleave(seg_node.to(dev), lens)
    rows = order[pos].long()
    bb = bins[rows].long()                                  # [m, F]
    yy = y[rows].to(torch.float64)
    ww = torch.ones_like(yy) if w is None else w[rows].to(torch.float64)
    fidx = torch.arange(F, device=dev)[None, :]
    base = ((node[:, None] * F + fidx) * B + bb) * S        # [m, F]
    if cls:
        idx = base + yy.long()[:, None]
        out.index_add_(0, idx.reshape(-1), ww[:, None].expand(-1, F).reshape(-1))
    else:
        for s, v in enumerate((ww, ww * yy, ww * yy * yy)):
            out.index_add_(0, (base + s).reshape(-1), v[:, None].expand(-1, F).reshape(-1))
    return out.view(n_nodes, F, B, S).float()
