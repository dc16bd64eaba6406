"""Tree histogram op: gfx950 kernel (csrc/trees.hip) with a PyTorch reference."""
from __future__ import annotations

import torch

from . import _native as N


def hist_kernel_ok(bins: torch.Tensor, B: int, S: int, cls: bool) -> bool:
    if not bins.is_cuda or bins.dtype != torch.uint8:
        return False
    F = bins.shape[1]
    fp = 4
    while fp < F and fp < 64:
        fp <<= 1
    return N.kernels().o3s_tree_hist_lds(fp, B, S, int(cls)) > 0


def _items(seg_lo: torch.Tensor, seg_hi: torch.Tensor, chunk: int):
    """Split segments into work items of <= chunk rows: (it_lo, it_hi, it_seg)."""
    dev = seg_lo.device
    lens = (seg_hi - seg_lo).clamp_min(0)
    nchunks = (lens + chunk - 1) // chunk
    nchunks = torch.where(lens > 0, nchunks, torch.zeros_like(nchunks))
    seg_id = torch.repeat_interleave(torch.arange(seg_lo.numel(), device=dev), nchunks)
    first = torch.cumsum(nchunks, 0) - nchunks
    k = torch.arange(seg_id.numel(), device=dev) - first[seg_id]
    it_lo = (seg_lo[seg_id] + k * chunk).to(torch.int64).contiguous()
    it_hi = torch.minimum(it_lo + chunk, seg_hi[seg_id].to(torch.int64)).contiguous()
    return it_lo, it_hi, seg_id, first


def feature_major(bins: torch.Tensor) -> torch.Tensor | None:
    """[F, n] copy of the binned matrix for the partition's per-row feature reads (GPU;
    LDS-tiled ``u8_transpose_kernel``, F % 4 == 0, else torch's strided copy)."""
    if not bins.is_cuda:
        return None
    n, F = bins.shape
    if F % 4 != 0 or not bins.is_contiguous():
        return bins.t().contiguous()
    out = torch.empty((F, n), dtype=torch.uint8, device=bins.device)
    N.check(N.kernels().o3s_u8_transpose(bins.data_ptr(), n, F, out.data_ptr(), N.stream_of(bins)), "u8_transpose")
    return out


def partition(bins: torch.Tensor, order: torch.Tensor, s_lo: torch.Tensor, s_hi: torch.Tensor,
              s_feat: torch.Tensor, s_bin: torch.Tensor, chunk: int = 1 << 14, bins_t: torch.Tensor | None = None):
    """Stable split of every segment [s_lo, s_hi) of ``order`` into rows with
    bins[row, feat] <= bin (first) and the rest.  Returns (new_order, nleft per segment).

    GPU: two passes of ``tree_part_*_kernel`` over work items (count, then scatter to
    destinations computed by small scans here); CPU: the PyTorch reference."""
    if not (bins.is_cuda and order.dtype == torch.int32):
        return partition_torch(bins, order, s_lo, s_hi, s_feat, s_bin)
    dev = bins.device
    F = bins.shape[1]
    nseg = s_lo.numel()
    it_lo, it_hi, it_seg, first_item = _items(s_lo, s_hi, chunk)
    n_items = int(it_lo.numel())
    new_order = order.clone()
    if n_items == 0:
        return new_order, torch.zeros(nseg, dtype=torch.int64, device=dev)
    it_feat = s_feat[it_seg].to(torch.int32).contiguous()
    it_bin = s_bin[it_seg].to(torch.int32).contiguous()
    it_left = torch.empty(n_items, dtype=torch.int64, device=dev)
    flags = torch.empty(order.shape[0], dtype=torch.uint8, device=dev)
    lib = N.kernels()
    st = N.stream_of(bins)
    src, rs, cs = (bins_t, 1, bins.shape[0]) if bins_t is not None else (bins, F, 1)
    N.check(lib.o3s_tree_partition(src.data_ptr(), rs, cs, order.data_ptr(), None, it_lo.data_ptr(), it_hi.data_ptr(),
                                   it_feat.data_ptr(), it_bin.data_ptr(), it_left.data_ptr(), None, None,
                                   flags.data_ptr(), n_items, 0, st), "tree_part_count")
    it_right = (it_hi - it_lo) - it_left
    nleft = torch.zeros(nseg, dtype=torch.int64, device=dev).index_add_(0, it_seg, it_left)
    cl = torch.cumsum(it_left, 0) - it_left                    # global exclusive prefixes
    cr = torch.cumsum(it_right, 0) - it_right
    f = first_item[it_seg]                                     # first item of each item's segment
    dst_left = (s_lo[it_seg] + cl - cl[f]).contiguous()
    dst_right = (s_lo[it_seg] + nleft[it_seg] + cr - cr[f]).contiguous()
    N.check(lib.o3s_tree_partition(src.data_ptr(), rs, cs, order.data_ptr(), new_order.data_ptr(), it_lo.data_ptr(),
                                   it_hi.data_ptr(), it_feat.data_ptr(), it_bin.data_ptr(), None,
                                   dst_left.data_ptr(), dst_right.data_ptr(), flags.data_ptr(), n_items, 1, st),
            "tree_part_scatter")
    return new_order, nleft


def partition_torch(bins, order, s_lo, s_hi, s_feat, s_bin):
    dev = bins.device
    F = bins.shape[1]
    lens = s_hi - s_lo
    total = int(lens.sum())
    sid = torch.repeat_interleave(torch.arange(s_lo.numel(), device=dev), lens)
    first = torch.cumsum(lens, 0) - lens
    pos = s_lo[sid] + (torch.arange(total, device=dev) - first[sid])
    rows = order[pos].long()
    bvals = bins.view(-1)[rows * F + s_feat[sid]]
    go_left = bvals.to(torch.int64) <= s_bin[sid]
    gl = go_left.to(torch.int64)
    cl = torch.cumsum(gl, 0)
    nleft = torch.zeros(s_lo.numel(), dtype=torch.int64, device=dev).index_add_(0, sid, gl)
    if total == 0:
        return order.clone(), nleft
    cl_before = cl[first.clamp_max(total - 1)] - gl[first.clamp_max(total - 1)]
    lrank = cl - cl_before[sid]                            # inclusive rank among lefts
    rel = torch.arange(total, device=dev) - first[sid]
    rrank = rel + 1 - lrank
    newpos = torch.where(go_left, s_lo[sid] + lrank - 1, s_lo[sid] + nleft[sid] + rrank - 1)
    new_order = order.clone()
    new_order[newpos] = order[pos]
    return new_order, nleft


def node_hist(bins: torch.Tensor, order: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None,
              seg_lo: torch.Tensor, seg_hi: torch.Tensor, seg_node: torch.Tensor, n_nodes: int, B: int, S: int,
              cls: bool, chunk: int = 1 << 13) -> torch.Tensor:
    """Histograms [n_nodes, F, B, S] (fp64) of rows order[lo:hi] for each segment -> node.

    Classification: per-bin weighted class counts.  Regression (S = 3): per-bin sums of
    w and w*y; the node's sum of w*y^2 sits in (feature 0, bin 0, stat 2) -- variance
    split gains need only the first two, the node impurity the third.

    Segments are split into work items of <= ``chunk`` rows; the kernel writes one fp32
    slab row per item (exact for integer weights: <= 8192 rows per item) and the slab rows
    of each segment are summed in fp64, in item order, by ``slab_range_sum_kernel``
    (two fixed-shape stages), so the result is bitwise reproducible and bins past 2^24
    weight keep full precision -- which histogram subtraction (sibling = parent - child)
    relies on."""
    F = bins.shape[1]
    dev = bins.device
    out = torch.zeros((n_nodes, F * B * S), dtype=torch.float64, device=dev)
    if seg_lo.numel() == 0:
        return out.view(n_nodes, F, B, S)
    it_lo, it_hi, seg_id, first = _items(seg_lo, seg_hi, chunk)
    n_items = int(it_lo.numel())
    if n_items == 0:
        return out.view(n_nodes, F, B, S)
    if hist_kernel_ok(bins, B, S, cls):
        C = F * B * S
        slab = torch.empty((n_items, C), dtype=torch.float32, device=dev)
        yf = y.to(torch.float32).contiguous()
        wf = None if w is None else w.to(torch.float32).contiguous()
        lib = N.kernels()
        st = N.stream_of(bins)
        N.check(lib.o3s_tree_hist(bins.data_ptr(), bins.shape[0], F, B, S, int(cls),
                                  order.data_ptr(), yf.data_ptr(), N.ptr(wf), it_lo.data_ptr(),
                                  it_hi.data_ptr(), n_items, slab.data_ptr(), st), "tree_hist")
        seg_sum = _ordered_segment_sums(lib, st, slab, seg_lo, seg_hi, first, chunk)
        out.index_add_(0, seg_node.to(torch.int64), seg_sum)    # one segment per node in the engine
        return out.view(n_nodes, F, B, S)
    # reference path (CPU / oversize bins): direct scatter-add per segment
    return hist_torch(bins, order, y, w, seg_lo, seg_hi, seg_node, n_nodes, B, S, cls)


_RUN = 64      # slab rows per first-stage partial


def _ordered_segment_sums(lib, st, slab, seg_lo, seg_hi, first, chunk):
    """[nseg, C] fp64: sum of each segment's slab rows (items of a segment are contiguous
    from ``first[s]``) in a fixed order -- runs of <= 64 items, then the runs in order."""
    dev = slab.device
    C = slab.shape[1]
    nseg = seg_lo.numel()
    lens = (seg_hi - seg_lo).clamp_min(0)
    n_it = torch.where(lens > 0, (lens + chunk - 1) // chunk, torch.zeros_like(lens)).to(torch.int64)
    n_run = (n_it + _RUN - 1) // _RUN
    run_seg = torch.repeat_interleave(torch.arange(nseg, device=dev), n_run)
    run_first = torch.cumsum(n_run, 0) - n_run
    k = torch.arange(run_seg.numel(), device=dev) - run_first[run_seg]
    r_lo = (first.to(torch.int64)[run_seg] + k * _RUN).contiguous()
    r_cnt = torch.minimum(torch.full_like(r_lo, _RUN), first.to(torch.int64)[run_seg] + n_it[run_seg] - r_lo).contiguous()
    runs = torch.empty((run_seg.numel(), C), dtype=torch.float64, device=dev)
    out = torch.zeros((nseg, C), dtype=torch.float64, device=dev)
    for a in range(0, runs.shape[0], 65535):
        b = min(a + 65535, runs.shape[0])
        N.check(lib.o3s_slab_range_sum(slab.data_ptr(), 0, C, r_lo[a:b].data_ptr(), r_cnt[a:b].data_ptr(), b - a,
                                       runs[a:].data_ptr(), st), "slab_range_sum")
    run_first = run_first.contiguous()
    n_run = n_run.contiguous()
    for a in range(0, nseg, 65535):
        b = min(a + 65535, nseg)
        N.check(lib.o3s_slab_range_sum(runs.data_ptr(), 1, C, run_first[a:b].data_ptr(), n_run[a:b].data_ptr(), b - a,
                                       out[a:].data_ptr(), st), "slab_range_sum")
    return out


def hist_torch(bins, order, y, w, seg_lo, seg_hi, seg_node, n_nodes, B, S, cls):
    F = bins.shape[1]
    dev = bins.device
    out = torch.zeros(n_nodes * F * B * S, dtype=torch.float64, device=dev)
    lens = (seg_hi - seg_lo).clamp_min(0)
    if int(lens.sum()) == 0:
        return out.view(n_nodes, F, B, S)
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
        for s, v in enumerate((ww, ww * yy)):
            out.index_add_(0, (base + s).reshape(-1), v[:, None].expand(-1, F).reshape(-1))
        # sum of w*y^2 is a node total (the split gain needs only w and w*y per bin),
        # stored in (feature 0, bin 0) like the kernel does; rows are grouped by segment,
        # so per-segment totals come from one prefix sum (no contended atomics)
        cs = torch.cumsum(ww * yy * yy, 0)
        ends = torch.cumsum(lens, 0)
        seg_tot = cs[(ends - 1).clamp_min(0)] - torch.where(ends - lens > 0, cs[(ends - lens - 1).clamp_min(0)],
                                                             torch.zeros_like(ends, dtype=cs.dtype))
        seg_tot = torch.where(lens > 0, seg_tot, torch.zeros_like(seg_tot))
        out.index_add_(0, seg_node.to(dev).long() * F * B * S + 2, seg_tot)
    return out.view(n_nodes, F, B, S)
