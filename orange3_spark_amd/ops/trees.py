"""Tree histogram op: gfx950 kernel (csrc/trees.hip) with a PyTorch reference."""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _native as N


def _host(x):
    """int64 numpy view of a small index array given as numpy or a (device) tensor."""
    import numpy as np
    if isinstance(x, torch.Tensor):
        return x.detach().to("cpu", torch.int64).numpy()
    return np.asarray(x, dtype=np.int64)


def _dev(x, dev):
    return x.to(dev) if isinstance(x, torch.Tensor) else N.upload(_host(x), dev)


def hist_kernel_ok(bins: torch.Tensor, B: int, S: int, cls: bool) -> bool:
    if not bins.is_cuda or bins.dtype != torch.uint8:
        return False
    F = bins.shape[1]
    fp = 4
    while fp < F and fp < 64:
        fp <<= 1
    return N.kernels().o3s_tree_hist_lds(fp, B, S, int(cls)) > 0


# row-major bins -> the feature-major copy written in the same pass by the binning kernel
# (models/trees.bin_features), so feature_major() needs no second pass over the matrix.
# Kept as an attribute of the bins tensor itself: it lives exactly as long as the bins (a
# WeakKeyDictionary keyed by tensors compares keys with Tensor.__eq__ on hash collisions).
def remember_feature_major(bins: torch.Tensor, bins_t: torch.Tensor) -> None:
    bins._o3s_feature_major = bins_t


def feature_major(bins: torch.Tensor) -> torch.Tensor | None:
    """[F, n] copy of the binned matrix for the partition's per-row feature reads (GPU;
    the binning kernel's own feature-major output when it wrote one, else the LDS-tiled
    ``u8_transpose_kernel``, F % 4 == 0, or torch's strided copy)."""
    if not bins.is_cuda:
        return None
    fm = getattr(bins, "_o3s_feature_major", None)
    if fm is not None:
        return fm
    n, F = bins.shape
    if F % 4 != 0 or not bins.is_contiguous():
        return bins.t().contiguous()
    out = torch.empty((F, n), dtype=torch.uint8, device=bins.device)
    N.check(N.kernels().o3s_u8_transpose(bins.data_ptr(), n, F, out.data_ptr(), N.stream_of(bins)), "u8_transpose")
    return out


PART_CHUNK = int(os.environ.get("O3S_PART_CHUNK", str(1 << 14)))   # rows per partition work item


def partition(bins: torch.Tensor, order: torch.Tensor, s_lo: torch.Tensor, s_hi: torch.Tensor,
              s_feat: torch.Tensor, s_bin: torch.Tensor, chunk: int | None = None, bins_t: torch.Tensor | None = None,
              out: torch.Tensor | None = None, payload=(), payload_out=()):
    """Stable split of every segment [s_lo, s_hi) of ``order`` into rows with
    bins[row, feat] <= bin (first) and the rest.  Returns (new_order, nleft per segment).

    ``out`` (GPU): write the split segments into this buffer and leave every other
    position of it untouched (ping-pong buffers of a caller that no longer needs the
    rows outside the split segments); default: a full copy of ``order`` first.

    ``payload`` (<= 2 fp32 arrays in POSITION order, e.g. y and w): moved with the rows
    into the matching ``payload_out`` buffers (same rule as ``out``: positions outside
    the split segments are not written).

    GPU: two passes of ``tree_part_*_kernel`` over work items (count, then scatter to
    destinations from ``tree_part_dest_kernel``); CPU: the PyTorch reference."""
    payload, payload_out = tuple(payload), tuple(payload_out)
    chunk = chunk or PART_CHUNK
    if len(payload) != len(payload_out) or len(payload) > 2:
        raise ValueError("payload / payload_out mismatch")
    if not (bins.is_cuda and order.dtype == torch.int32):
        dv = bins.device
        return partition_torch(bins, order, _dev(s_lo, dv), _dev(s_hi, dv), _dev(s_feat, dv), _dev(s_bin, dv),
                               out=out, payload=payload, payload_out=payload_out)
    import numpy as np
    dev = bins.device
    F = bins.shape[1]
    # work items planned on the host (segment bounds are tiny) and uploaded in one copy
    lo, hi = _host(s_lo), _host(s_hi)
    nseg = len(lo)
    n_it = (np.maximum(hi - lo, 0) + chunk - 1) // chunk
    first = np.cumsum(n_it) - n_it
    n_items = int(n_it.sum())
    new_order = order.clone() if out is None else out
    if n_items == 0:
        return new_order, torch.zeros(nseg, dtype=torch.int64, device=dev)
    seg_of = np.repeat(np.arange(nseg), n_it)
    it_lo_h = lo[seg_of] + (np.arange(n_items) - first[seg_of]) * chunk
    it_hi_h = np.minimum(it_lo_h + chunk, hi[seg_of])
    seg_first = np.append(first, n_items)
    fb = np.concatenate([_host(s_feat).astype(np.int32)[seg_of], _host(s_bin).astype(np.int32)[seg_of]])
    i64, i32 = N.upload_many(dev, np.concatenate([it_lo_h, it_hi_h, seg_first, lo]).astype(np.int64), fb)
    it_lo, it_hi = i64[:n_items], i64[n_items:2 * n_items]
    seg_first_d, seg_lo_d = i64[2 * n_items:2 * n_items + nseg + 1], i64[2 * n_items + nseg + 1:]
    it_feat, it_bin = i32[:n_items], i32[n_items:]
    work = torch.empty(3 * n_items + nseg, dtype=torch.int64, device=dev)
    it_left, dst_left, dst_right = work[:n_items], work[n_items:2 * n_items], work[2 * n_items:3 * n_items]
    nleft = work[3 * n_items:]
    flags = torch.empty(order.shape[0], dtype=torch.uint8, device=dev)
    lib = N.kernels()
    st = N.stream_of(bins)
    src, rs, cs = (bins_t, 1, bins.shape[0]) if bins_t is not None else (bins, F, 1)
    N.check(lib.o3s_tree_partition(src.data_ptr(), rs, cs, order.data_ptr(), None, it_lo.data_ptr(), it_hi.data_ptr(),
                                   it_feat.data_ptr(), it_bin.data_ptr(), it_left.data_ptr(), None, None,
                                   flags.data_ptr(), n_items, 0, None, None, None, None, st), "tree_part_count")
    N.check(lib.o3s_tree_part_dest(it_lo.data_ptr(), it_hi.data_ptr(), it_left.data_ptr(), seg_first_d.data_ptr(),
                                   seg_lo_d.data_ptr(), nseg, dst_left.data_ptr(), dst_right.data_ptr(),
                                   nleft.data_ptr(), st), "tree_part_dest")
    pl = [None] * 4
    for q, (a, b) in enumerate(zip(payload, payload_out)):
        if a.dtype != torch.float32 or b.dtype != torch.float32 or a.numel() != order.numel() \
                or b.numel() != order.numel() or not (a.is_contiguous() and b.is_contiguous()):
            raise ValueError("payloads must be contiguous fp32 arrays of the order's length")
        pl[2 * q], pl[2 * q + 1] = a.data_ptr(), b.data_ptr()
    N.check(lib.o3s_tree_partition(src.data_ptr(), rs, cs, order.data_ptr(), new_order.data_ptr(), it_lo.data_ptr(),
                                   it_hi.data_ptr(), it_feat.data_ptr(), it_bin.data_ptr(), None,
                                   dst_left.data_ptr(), dst_right.data_ptr(), flags.data_ptr(), n_items, 1, *pl, st),
            "tree_part_scatter")
    return new_order, nleft


def final_level(bins: torch.Tensor, order: torch.Tensor, s_lo, s_hi, s_feat, s_bin, vl, vr, y: torch.Tensor,
                w: torch.Tensor | None, acc: torch.Tensor | None, need_y2: bool,
                bins_t: torch.Tensor | None = None, chunk: int = 1 << 14):
    """Last split level of a tree: rows of every splitting segment are routed by its
    split; ``acc`` (fp64 [n], boosting) gets the left / right child's leaf value per row
    (``vl`` / ``vr`` per segment) and, with ``need_y2``, the children's sums of w*y^2
    (fp64 [nseg, 2]: left, right; y / w in position order) are returned, else None.

    GPU: ``tree_final_level_kernel`` + ordered fp64 range sums; CPU: torch."""
    lo, hi = _host(s_lo), _host(s_hi)
    nseg = len(lo)
    dev = bins.device
    vl = np.asarray(vl, dtype=np.float64)
    vr = np.asarray(vr, dtype=np.float64)
    if nseg == 0:
        return torch.zeros((0, 2), dtype=torch.float64, device=dev) if need_y2 else None
    if not (bins.is_cuda and order.dtype == torch.int32):
        F = bins.shape[1]
        lens = np.maximum(hi - lo, 0)
        sid = np.repeat(np.arange(nseg), lens)
        pos = torch.from_numpy(np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]) if lens.sum()
                               else np.zeros(0, dtype=np.int64)).to(dev)
        rows = order[pos].long()
        fe = torch.from_numpy(_host(s_feat)[sid]).to(dev)
        bb = torch.from_numpy(_host(s_bin)[sid]).to(dev)
        left = bins.view(-1)[rows * F + fe].to(torch.int64) <= bb
        sid_t = torch.from_numpy(sid).to(dev)
        if acc is not None:
            v = torch.where(left, torch.from_numpy(vl[sid]).to(dev), torch.from_numpy(vr[sid]).to(dev))
            acc.index_add_(0, rows.to(acc.device), v.to(acc.dtype))
        if not need_y2:
            return None
        yy = y[pos].to(torch.float64)
        ww = torch.ones_like(yy) if w is None else w[pos].to(torch.float64)
        out = torch.zeros((nseg, 2), dtype=torch.float64, device=dev)
        out.view(-1).index_add_(0, sid_t * 2 + (~left).long(), ww * yy * yy)
        return out
    n_it = (np.maximum(hi - lo, 0) + chunk - 1) // chunk
    first = np.cumsum(n_it) - n_it
    n_items = int(n_it.sum())
    if n_items == 0:
        return torch.zeros((nseg, 2), dtype=torch.float64, device=dev) if need_y2 else None
    seg_of = np.repeat(np.arange(nseg), n_it)
    it_lo = lo[seg_of] + (np.arange(n_items) - first[seg_of]) * chunk
    it_hi = np.minimum(it_lo + chunk, hi[seg_of])
    fb = np.concatenate([_host(s_feat).astype(np.int32)[seg_of], _host(s_bin).astype(np.int32)[seg_of]])
    r_lo, r_cnt = first, n_it
    i64, i32, f64 = N.upload_many(dev, np.concatenate([it_lo, it_hi, r_lo, r_cnt]).astype(np.int64), fb,
                                  np.concatenate([vl[seg_of], vr[seg_of]]))
    part = torch.empty((n_items, 2), dtype=torch.float32, device=dev) if need_y2 else None
    yf = y.to(torch.float32).contiguous() if need_y2 else None
    wf = None if (w is None or not need_y2) else w.to(torch.float32).contiguous()
    src, rs, cs = (bins_t, 1, bins.shape[0]) if bins_t is not None else (bins, bins.shape[1], 1)
    lib = N.kernels()
    st = N.stream_of(bins)
    N.check(lib.o3s_tree_final_level(src.data_ptr(), rs, cs, order.data_ptr(), i64[:n_items].data_ptr(),
                                     i64[n_items:2 * n_items].data_ptr(), i32[:n_items].data_ptr(),
                                     i32[n_items:].data_ptr(), f64[:n_items].data_ptr(), f64[n_items:].data_ptr(),
                                     N.ptr(yf), N.ptr(wf), N.ptr(acc), N.ptr(part), n_items, st), "tree_final_level")
    if not need_y2:
        return None
    out = torch.empty((nseg, 2), dtype=torch.float64, device=dev)
    rl, rc = i64[2 * n_items:2 * n_items + nseg], i64[2 * n_items + nseg:]
    for a in range(0, nseg, 65535):                           # item partials summed per segment, in order
        b = min(a + 65535, nseg)
        N.check(lib.o3s_slab_range_sum(part.data_ptr(), 0, 2, rl[a:].data_ptr(), rc[a:].data_ptr(), b - a,
                                       out[a:].data_ptr(), st), "slab_range_sum")
    return out


def leaf_apply(order: torch.Tensor, seg_lo: torch.Tensor, seg_hi: torch.Tensor, seg_val: torch.Tensor,
               acc: torch.Tensor, chunk: int = 1 << 14) -> None:
    """acc[order[p]] += seg_val[s] for every position p of segment s (fp64 acc).

    GPU: ``tree_leaf_apply_kernel`` over <= chunk-row items planned on the host; CPU: torch."""
    import numpy as np
    if len(seg_lo) == 0:
        return
    dev = acc.device
    lo, hi = _host(seg_lo), _host(seg_hi)
    val = seg_val.detach().to("cpu", torch.float64).numpy() if isinstance(seg_val, torch.Tensor) \
        else np.asarray(seg_val, dtype=np.float64)
    lens = np.maximum(hi - lo, 0)
    if not (acc.is_cuda and order.dtype == torch.int32 and acc.dtype == torch.float64):
        if lens.sum() == 0:
            return
        pos = torch.from_numpy(np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)])).to(order.device)
        v = torch.from_numpy(np.repeat(val, lens)).to(acc.device, acc.dtype)
        acc.index_add_(0, order[pos].long().to(acc.device), v)
        return
    n_it = (lens + chunk - 1) // chunk
    first = np.cumsum(n_it) - n_it
    n_items = int(n_it.sum())
    if n_items == 0:
        return
    seg_of = np.repeat(np.arange(len(lo)), n_it)
    it_lo = lo[seg_of] + (np.arange(n_items) - first[seg_of]) * chunk
    it_hi = np.minimum(it_lo + chunk, hi[seg_of])
    i64, fv = N.upload_many(dev, np.concatenate([it_lo, it_hi]).astype(np.int64),
                            np.ascontiguousarray(val[seg_of], dtype=np.float64))
    N.check(N.kernels().o3s_tree_leaf_apply(order.data_ptr(), i64[:n_items].data_ptr(), i64[n_items:].data_ptr(),
                                            fv.data_ptr(), n_items, acc.data_ptr(), N.stream_of(acc)),
            "tree_leaf_apply")


_KINDS = {"variance": 0, "gini": 1, "entropy": 2}
_GBT_LOSS = {"logistic": 0, "squared": 1, "absolute": 2}


def gbt_point_loss(loss: str, yy: torch.Tensor, Fm: torch.Tensor) -> torch.Tensor:
    """Spark GBT per-row loss (logistic: 2*log(1 + e^{-2yF}), evaluated stably)."""
    if loss == "logistic":
        z = -2.0 * yy * Fm
        return 2.0 * torch.where(z > 0, z + torch.log1p(torch.exp(-z)), torch.log1p(torch.exp(z)))
    if loss == "squared":
        return (yy - Fm) ** 2
    return (yy - Fm).abs()


def gbt_residual(loss: str, yy: torch.Tensor, Fm: torch.Tensor) -> torch.Tensor:
    """Pseudo-residuals (negative loss gradients) the next tree is fit to."""
    if loss == "logistic":
        return 4.0 * yy / (1.0 + torch.exp(2.0 * yy * Fm))
    if loss == "squared":
        return 2.0 * (yy - Fm)
    return torch.sign(yy - Fm)


def gbt_grad_loss(loss: str, yy: torch.Tensor, Fm: torch.Tensor, w: torch.Tensor | None, w_val: torch.Tensor | None,
                  target: torch.Tensor | None = None) -> torch.Tensor:
    """One boosting epilogue pass: returns fp64 [sum loss*w, sum w, sum loss*w_val,
    sum w_val] over the local rows and (``target`` given, fp32) writes the residuals of
    the next tree into it.  GPU: ``gbt_grad_loss_kernel`` (one fused pass, fixed-grid
    partial sums); CPU: the torch reference."""
    n = yy.shape[0]
    dev = yy.device
    if yy.is_cuda and n > 0:
        f64 = [None if t is None else t.to(torch.float64).contiguous() for t in (yy, Fm, w, w_val)]
        nb = int(min(2048, max(1, (n + 255) // 256)))
        part = torch.empty((nb, 4), dtype=torch.float64, device=dev)
        if target is not None and (target.dtype != torch.float32 or target.numel() != n or not target.is_contiguous()):
            raise ValueError("target must be a contiguous fp32 [n] tensor")
        N.check(N.kernels().o3s_gbt_grad_loss(*(N.ptr(t) for t in f64), n, _GBT_LOSS[loss], N.ptr(target),
                                              part.data_ptr(), nb, N.stream_of(yy)), "gbt_grad_loss")
        return part.sum(0)
    pl = gbt_point_loss(loss, yy.double(), Fm.double())
    wt = torch.ones_like(pl) if w is None else w.double()
    out = [(pl * wt).sum(), wt.sum()]
    if w_val is not None:
        out += [(pl * w_val.double()).sum(), w_val.double().sum()]
    else:
        out += [torch.zeros((), dtype=torch.float64, device=dev)] * 2
    if target is not None:
        target.copy_(gbt_residual(loss, yy.double(), Fm.double()))
    return torch.stack(out)


LEAF_PASS_MAX_DEPTH = 10            # 2^D per-leaf y^2 columns per wave fit the kernel's LDS


def tree_node_arrays(feature: np.ndarray, split_bin: np.ndarray, value: np.ndarray, scale: float):
    """Heap-ordered tree -> (node_fb int32 [nodes]: feature | bin << 16 for internal
    nodes, -1 for leaves / absent; node_val fp64 [nodes]: leaf value * scale)."""
    fe = np.asarray(feature, dtype=np.int64)
    fb = np.where(fe >= 0, fe | (np.asarray(split_bin, dtype=np.int64) << 16), -1).astype(np.int32)
    return fb, np.asarray(value, dtype=np.float64).reshape(len(fe), -1)[:, 0] * float(scale)


LEAF_BLOCKS_PER_CU = int(os.environ.get("O3S_LEAF_BLOCKS", "4"))     # gbt_leaf_pass_kernel grid (A/B 4 / 8 / 16: 12.2 / 12.6 / 13.5 ms per tree)


def gbt_leaf_pass(bins: torch.Tensor, feature, split_bin, value, scale: float, depth: int, loss: str,
                  yy: torch.Tensor, Fm: torch.Tensor, wt: torch.Tensor | None, wd: torch.Tensor | None,
                  wv: torch.Tensor | None, first: bool, target: torch.Tensor | None, need_y2: bool):
    """The GBT tree epilogue in ONE pass over the rows in row order (``gbt_leaf_pass_kernel``):
    every row walks the finished tree on its bins, ``Fm += scale * value(leaf)``, the loss
    partials of the updated ensemble [sum l*wd, sum wd, sum l*wv, sum wv] (fp64 [4]) are
    returned, ``target`` (fp32, optional) receives the next tree's residuals, and with
    ``need_y2`` the sums of wt*y^2 of the leaves at depth ``depth`` (fp64 [2^depth], y =
    the residual this tree was fit to: yy for the first tree, else the loss gradient at
    the pre-update Fm) -- the last level's children impurities.  CPU: torch."""
    n, F = bins.shape
    dev = bins.device
    fb, val = tree_node_arrays(feature, split_bin, value, scale)
    nodes = len(fb)
    L = 1 << depth
    if bins.is_cuda and n > 0:
        f64 = [None if t is None else t.to(torch.float64).contiguous() for t in (wd, wv)]
        wt32 = None if wt is None else wt.to(torch.float32).contiguous()
        if target is not None and (target.dtype != torch.float32 or target.numel() != n or not target.is_contiguous()):
            raise ValueError("target must be a contiguous fp32 [n] tensor")
        if not (yy.dtype == torch.float64 and Fm.dtype == torch.float64 and yy.is_contiguous() and Fm.is_contiguous()):
            raise ValueError("yy / Fm must be contiguous fp64")
        grid = int(max(1, min(N.num_cus(dev) * LEAF_BLOCKS_PER_CU, (n + 255) // 256)))
        part = torch.empty((grid, 4), dtype=torch.float64, device=dev)
        slab = torch.empty((grid * 4, L), dtype=torch.float32, device=dev) if need_y2 else None   # a row per wave
        fb_d, val_d = N.upload_many(dev, fb, val)
        lib = N.kernels()
        N.check(lib.o3s_gbt_leaf_pass(bins.data_ptr(), n, F, fb_d.data_ptr(), nodes, val_d.data_ptr(), depth,
                                      yy.data_ptr(), Fm.data_ptr(), N.ptr(wt32), N.ptr(f64[0]), N.ptr(f64[1]),
                                      _GBT_LOSS[loss], int(first), N.ptr(target), part.data_ptr(), N.ptr(slab),
                                      grid, N.stream_of(Fm)), "gbt_leaf_pass")
        y2 = None
        if need_y2:
            y2 = torch.empty((1, L), dtype=torch.float64, device=dev)
            lo, cnt = N.upload_many(dev, np.zeros(1, np.int64), np.full(1, grid * 4, np.int64))
            N.check(lib.o3s_slab_range_sum(slab.data_ptr(), 0, L, lo.data_ptr(), cnt.data_ptr(), 1, y2.data_ptr(),
                                           N.stream_of(Fm)), "gbt_leaf_pass y2")
            y2 = y2[0]
        return part.sum(0), y2
    # torch reference: walk the tree, update, loss / residual, per-leaf y^2
    fb_t = torch.from_numpy(fb.astype(np.int64)).to(dev)
    node = torch.ones(n, dtype=torch.int64, device=dev)
    for _ in range(depth):
        code = fb_t[node]
        inner = code >= 0
        if not bool(inner.any()):
            break
        f = torch.where(inner, code & 0xFFFF, torch.zeros_like(code))
        sb = (code >> 16) & 0x7FFF
        b = bins.gather(1, f[:, None]).squeeze(1).to(torch.int64)
        node = torch.where(inner, 2 * node + (b > sb).to(torch.int64), node)
    Fo = Fm.clone()
    Fm += torch.from_numpy(val).to(dev)[node]
    out = gbt_grad_loss(loss, yy, Fm, wd, wv, target)
    y2 = None
    if need_y2:
        yo = yy.to(torch.float32) if first else gbt_residual(loss, yy.double(), Fo.double()).to(torch.float32)
        ww = torch.ones_like(yo) if wt is None else wt.to(torch.float32)
        v = (ww * yo * yo).to(torch.float64)
        at = node >= L
        y2 = torch.zeros(L, dtype=torch.float64, device=dev)
        y2.index_add_(0, (node[at] - L), v[at])
    return out, y2


def best_splits(H: torch.Tensor, nb: torch.Tensor, fmask, kind: str, min_inst: float, min_w: float,
                min_wfrac: float, min_w_node=None) -> torch.Tensor:
    """Per-node best split of histograms H [k, F, B, S] (fp64, GPU) in ONE launch of
    ``tree_split_kernel``.  Returns the fp64 bundle [idx | gain | impurity | weight |
    wL | wR | values (k x V)] (V = S for classification, 1 for variance).

    ``fmask`` (numpy bool [k, F] or None): features each node may split on (forests);
    ``min_wfrac`` > 0: the minimum child weight is that fraction of the node's weight
    (the root level), else ``min_w``; ``min_w_node`` (numpy [k]) overrides both per node."""
    k, F, B, S = H.shape
    dev = H.device
    Hc = H.to(torch.float64).contiguous()
    nb32 = nb.to(dev, torch.int32).contiguous()
    fm = None if fmask is None else N.upload(np.asarray(fmask, dtype=np.uint8), dev)
    V = 1 if kind == "variance" else S
    mwn = None if min_w_node is None else N.upload(np.asarray(min_w_node, dtype=np.float64), dev)
    out = torch.empty(6 * k + k * V, dtype=torch.float64, device=dev)
    N.check(N.kernels().o3s_tree_split(Hc.data_ptr(), k, F, B, S, _KINDS[kind], nb32.data_ptr(), N.ptr(fm),
                                       float(min_inst), float(min_w), float(min_wfrac),
                                       N.ptr(mwn), out.data_ptr(),
                                       N.stream_of(Hc)), "tree_split")
    return out


def partition_torch(bins, order, s_lo, s_hi, s_feat, s_bin, out=None, payload=(), payload_out=()):
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
    new_order = order.clone() if out is None else out
    if total == 0:
        return new_order, nleft
    cl_before = cl[first.clamp_max(total - 1)] - gl[first.clamp_max(total - 1)]
    lrank = cl - cl_before[sid]                            # inclusive rank among lefts
    rel = torch.arange(total, device=dev) - first[sid]
    rrank = rel + 1 - lrank
    newpos = torch.where(go_left, s_lo[sid] + lrank - 1, s_lo[sid] + nleft[sid] + rrank - 1)
    new_order[newpos] = order[pos]
    for a, b in zip(payload, payload_out):
        b[newpos] = a[pos]
    return new_order, nleft


def node_hist(bins: torch.Tensor, order: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None,
              seg_lo: torch.Tensor, seg_hi: torch.Tensor, seg_node: torch.Tensor, n_nodes: int, B: int, S: int,
              cls: bool, chunk: int | None = None, ypos: bool = False) -> torch.Tensor:
    """Histograms [n_nodes, F, B, S] (fp64) of rows order[lo:hi] for each segment -> node.

    ``ypos``: y / w are in position order (y[p] is the label of row order[p], kept so
    by moving them through ``partition(payload=...)``): they stream contiguously.

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
    chunk = chunk or HIST_CHUNK
    if len(seg_lo) == 0:
        return torch.zeros((n_nodes, F, B, S), dtype=torch.float64, device=dev)
    if not hist_kernel_ok(bins, B, S, cls):
        # reference path (CPU / oversize bins): direct scatter-add per segment
        return hist_torch(bins, order, y, w, _dev(seg_lo, dev), _dev(seg_hi, dev), _dev(seg_node, dev), n_nodes,
                          B, S, cls, ypos=ypos)
    plan = _HistPlan(seg_lo, seg_hi, seg_node, chunk, dev)
    if plan.n_items == 0:
        return torch.zeros((n_nodes, F, B, S), dtype=torch.float64, device=dev)
    C = F * B * S
    slab = torch.empty((plan.n_items, C), dtype=torch.float32, device=dev)
    yf = y.to(torch.float32).contiguous()
    wf = None if w is None else w.to(torch.float32).contiguous()
    lib = N.kernels()
    st = N.stream_of(bins)
    N.check(lib.o3s_tree_hist(bins.data_ptr(), bins.shape[0], F, B, S, int(cls), order.data_ptr(), yf.data_ptr(),
                              N.ptr(wf), plan.it_lo.data_ptr(), plan.it_hi.data_ptr(), plan.n_items,
                              slab.data_ptr(), int(bool(ypos)), st), "tree_hist")
    # ordered fp64 sums: runs of <= 64 item rows, then each segment's runs in order
    runs = torch.empty((plan.n_runs, C), dtype=torch.float64, device=dev)
    for a in range(0, plan.n_runs, 65535):
        b = min(a + 65535, plan.n_runs)
        N.check(lib.o3s_slab_range_sum(slab.data_ptr(), 0, C, plan.r_lo[a:].data_ptr(), plan.r_cnt[a:].data_ptr(),
                                       b - a, runs[a:].data_ptr(), st), "slab_range_sum")
    nseg = plan.nseg
    seg_sum = torch.empty((nseg, C), dtype=torch.float64, device=dev)
    for a in range(0, nseg, 65535):
        b = min(a + 65535, nseg)
        N.check(lib.o3s_slab_range_sum(runs.data_ptr(), 1, C, plan.s_run0[a:].data_ptr(), plan.s_nrun[a:].data_ptr(),
                                       b - a, seg_sum[a:].data_ptr(), st), "slab_range_sum")
    if plan.identity and nseg == n_nodes:                 # the engine: segment i is node i
        return seg_sum.view(n_nodes, F, B, S)
    out = torch.zeros((n_nodes, C), dtype=torch.float64, device=dev)
    out.index_add_(0, plan.seg_node, seg_sum)
    return out.view(n_nodes, F, B, S)


def sibling_hists(Hs: torch.Tensor, parent: torch.Tensor, small_right, cls: bool) -> torch.Tensor:
    """Level histograms [2P, F, B, S] from the scanned smaller children Hs [P] and the
    parents [P]: node 2p + small_right[p] is Hs[p], its sibling parent[p] - Hs[p] with
    the rounding residue of fractional weights cleaned (class counts / weights clamped
    at 0, REG w*y zeroed where w <= 0, the node's w*y^2 clamped at 0).

    GPU: ``tree_sibling_kernel`` (one pass); CPU: torch."""
    P = Hs.shape[0]
    sr = np.asarray(small_right, dtype=np.uint8)
    if Hs.is_cuda and P > 0:
        Hs_c, par = Hs.contiguous(), parent.contiguous()
        H = torch.empty((2 * P,) + tuple(Hs.shape[1:]), dtype=torch.float64, device=Hs.device)
        srd = N.upload(sr, Hs.device)
        _, F, B, S = Hs.shape
        N.check(N.kernels().o3s_tree_sibling(Hs_c.data_ptr(), par.data_ptr(), srd.data_ptr(), P, F * B, S, int(cls),
                                             H.data_ptr(), N.stream_of(Hs)), "tree_sibling")
        return H
    sib = parent - Hs
    if cls:
        sib.clamp_min_(0.0)
    else:
        y2 = sib[:, 0, 0, 2].clamp_min(0.0)
        empty = sib[..., 0] <= 0.0
        sib[..., :2] = torch.where(empty[..., None], torch.zeros_like(sib[..., :2]), sib[..., :2])
        sib[:, 0, 0, 2] = y2
    H = torch.empty((2 * P,) + tuple(Hs.shape[1:]), dtype=torch.float64, device=Hs.device)
    pick = torch.from_numpy(2 * np.arange(P) + sr.astype(np.int64)).to(Hs.device)
    H[pick] = Hs
    H[pick ^ 1] = sib
    return H


_RUN = 64      # slab rows per first-stage partial
# rows per histogram work item: with the LDS-DMA row stage 16384 is best on the 500M x 64
# depth-8 config (s/tree 0.1253 / 0.1195 / 0.1169 / 0.1173 at 4096 / 8192 / 16384 / 32768,
# profiles/kernel_experiments_r6.json); O3S_HIST_CHUNK overrides for A/B runs
HIST_CHUNK = int(os.environ.get("O3S_HIST_CHUNK", str(1 << 14)))


class _HistPlan:
    """Work items (<= chunk rows of one segment) and their fixed-order reduction runs,
    planned on the host from the (small) segment bounds and uploaded in ONE copy --
    instead of a dozen tiny device ops and syncs per tree level."""

    def __init__(self, seg_lo, seg_hi, seg_node, chunk: int, dev):
        import numpy as np
        lo, hi, nd = _host(seg_lo), _host(seg_hi), _host(seg_node)
        lens = np.maximum(hi - lo, 0)
        n_it = (lens + chunk - 1) // chunk
        first = np.cumsum(n_it) - n_it
        self.nseg = len(lo)
        self.n_items = int(n_it.sum())
        seg_of = np.repeat(np.arange(self.nseg), n_it)
        k = np.arange(self.n_items) - first[seg_of]
        it_lo = lo[seg_of] + k * chunk
        it_hi = np.minimum(it_lo + chunk, hi[seg_of])
        n_run = (n_it + _RUN - 1) // _RUN
        run0 = np.cumsum(n_run) - n_run
        self.n_runs = int(n_run.sum())
        rseg = np.repeat(np.arange(self.nseg), n_run)
        kr = np.arange(self.n_runs) - run0[rseg]
        r_lo = first[rseg] + kr * _RUN
        r_cnt = np.minimum(_RUN, first[rseg] + n_it[rseg] - r_lo)
        parts = [it_lo, it_hi, r_lo, r_cnt, run0, n_run, nd]
        buf = N.upload(np.concatenate(parts).astype(np.int64), dev)
        views, off = [], 0
        for p in parts:
            views.append(buf[off: off + len(p)])
            off += len(p)
        self.it_lo, self.it_hi, self.r_lo, self.r_cnt, self.s_run0, self.s_nrun, self.seg_node = views
        self.identity = bool(np.array_equal(nd, np.arange(self.nseg)))


def hist_torch(bins, order, y, w, seg_lo, seg_hi, seg_node, n_nodes, B, S, cls, ypos=False):
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
    at = pos if ypos else rows
    yy = y[at].to(torch.float64)
    ww = torch.ones_like(yy) if w is None else w[at].to(torch.float64)
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
