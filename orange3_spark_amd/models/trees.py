"""Decision-tree engine (DecisionTree / RandomForest / GBT), level-wise, row-sharded.

Replaces MLlib's RandomForest.run / GradientBoostedTrees.boost (reached through the
Classification/Regression widgets, orangecontrib/spark/base/spark_ml_estimator.py:22).

Pipeline per tree, per level (every rank):
  1. ``ops.trees.node_hist``: LDS-privatised histogram kernel over this rank's rows,
     which are kept grouped by node in a permutation (``order``), one slab row per work
     item, summed per node in a fixed order;
  2. ONE all-reduce of the level's [nodes, F, bins, stats] histogram (<= 3 MB at depth 8,
     64 features, 32 bins) over RCCL;
  3. best split per node on device (replicated; Spark impurity/gain semantics, bins
     from approximate quantiles, ``minInstancesPerNode``, ``minInfoGain``, per-node
     feature subsets for forests);
  4. stable re-partition of ``order`` into the children (cumsum ranks, no sort).
Node numbering follows Spark (root = 1, children 2i / 2i+1).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import _native as N
from ..ops import sampling
from ..ops import trees as T
from ..runtime.tracing import trace
from ..runtime import progress


# ----------------------------------------------------------------------------- binning
def find_splits(comm, X, max_bins: int, seed: int = 0, sample: int | None = None) -> list:
    """Per-feature candidate thresholds from a global sample (Spark findSplitsBySorting:
    few distinct values -> midpoints, else approximate quantiles).  ``X``: a [n, F] tensor,
    or a ``frame.spill.RowBlocks`` (MEMORY_AND_DISK rows: only the sampled rows are
    fetched)."""
    from ..frame.spill import RowBlocks
    n_local = X.shape[0]
    n = comm.sum_scalar(int(n_local))
    want = sample or max(max_bins * max_bins, 10000)
    frac = min(1.0, want / max(n, 1))
    sizes = comm.all_gather_object(int(n_local))
    off = sum(sizes[: comm.rank])
    dev = X.device
    rows = torch.arange(off, off + n_local, dtype=torch.int64, device=dev)
    m = sampling.bernoulli_mask(rows, seed + 17, frac)
    if isinstance(X, RowBlocks):
        S = X.rows(torch.nonzero(m).reshape(-1)).to(torch.float64)
    else:
        S = X[m].to(torch.float64)
    S = comm.all_gather_v(S) if comm.world_size > 1 else S
    S = S.cpu().numpy()
    splits = []
    for f in range(X.shape[1]):
        v = S[:, f]
        v = v[~np.isnan(v)]
        u = np.unique(v)
        if len(u) <= 1:
            splits.append(np.zeros(0))
        elif len(u) <= max_bins - 1:
            splits.append((u[:-1] + u[1:]) / 2.0)
        else:
            qs = np.quantile(v, np.linspace(0, 1, max_bins + 1)[1:-1], method="linear")
            splits.append(np.unique(qs))
    return splits


def _thresholds(splits: list, F: int, device):
    T_ = max((len(s) for s in splits), default=0) + 1
    Tp = 1 << max(0, (T_ - 1).bit_length())
    if Tp > 256 or 4 * F * (Tp + 1) + F * 68 > 160 * 1024:      # thresholds + the [F][64] bin tile
        return None, Tp
    th = np.full((F, Tp), np.inf, dtype=np.float32)
    for f, s in enumerate(splits):
        th[f, :len(s)] = np.asarray(s, dtype=np.float32)
    return torch.from_numpy(th).to(device), Tp


def _bin_block_kernel(X: torch.Tensor, tht, Tp, out: torch.Tensor, out_t: torch.Tensor | None, ldt: int) -> None:
    n, F = X.shape
    N.check(N.kernels().o3s_bin_features2(X.data_ptr(), int(X.dtype == torch.bfloat16), n, X.stride(0), F,
                                          tht.data_ptr(), Tp, out.data_ptr(), N.ptr(out_t), ldt, N.stream_of(X)),
            "bin_features")


def _bin_block_torch(X: torch.Tensor, splits: list, out: torch.Tensor) -> None:
    if X.dtype == torch.bfloat16:
        X = X.float()
    step = 1 << 22
    for f in range(X.shape[1]):
        t = torch.as_tensor(splits[f], dtype=X.dtype if X.is_floating_point() else torch.float64, device=X.device)
        for a in range(0, X.shape[0], step):
            col = X[a:a + step, f].contiguous()
            out[a:a + step, f] = torch.bucketize(col.to(t.dtype), t, right=False).to(torch.uint8) if t.numel() \
                else torch.zeros_like(col, dtype=torch.uint8)


def bin_features(X, splits: list) -> torch.Tensor:
    """uint8 [n, F]: bin = #thresholds < value (value <= t_0 -> bin 0).

    GPU fp32 / bf16: one pass of ``bin_features_kernel`` (all thresholds in LDS, branchless
    search per element) that also writes the feature-major copy the partition reads
    (``ops.trees.feature_major`` returns it); otherwise per-feature ``torch.bucketize``.
    ``X`` may be a ``frame.spill.RowBlocks``: the resident rows and every host-streamed
    chunk are binned as they arrive into one resident uint8 matrix (the fp/bf16 features
    never need to fit in device memory together)."""
    from ..frame.spill import RowBlocks
    n, F = X.shape
    dev = X.device
    out = torch.empty((n, F), dtype=torch.uint8, device=dev)
    tht, Tp = _thresholds(splits, F, dev) if dev.type == "cuda" else (None, 0)
    out_t = torch.empty((F, n), dtype=torch.uint8, device=dev) if tht is not None and n > 0 else None

    def block(Xb: torch.Tensor, a: int) -> None:
        m = Xb.shape[0]
        if m == 0:
            return
        if tht is not None and Xb.dtype in (torch.float32, torch.bfloat16) and Xb.stride(1) == 1:
            _bin_block_kernel(Xb, tht, Tp, out[a:a + m], out_t[:, a:] if out_t is not None else None, n)
        else:
            _bin_block_torch(Xb, splits, out[a:a + m])
            if out_t is not None:
                out_t[:, a:a + m] = out[a:a + m].t()
    if isinstance(X, RowBlocks):
        X.run(block)
    else:
        block(X, 0)
    if out_t is not None:
        T.remember_feature_major(out, out_t)
    return out


# ----------------------------------------------------------------------------- impurity
def _sibling(parent: torch.Tensor, child: torch.Tensor, cls: bool) -> torch.Tensor:
    """Histogram of the scanned child's sibling, parent - child ([P, F, B, S] fp64).

    Both operands are exact ordered fp64 sums, but with fractional weights the
    difference can still leave rounding residue in bins the sibling does not populate;
    it is cleaned so such a bin reads as empty: weights / class counts are clamped at 0
    and REG bins whose weight is not positive get zero w*y.  The REG node total of w*y^2
    (feature 0, bin 0, stat 2) is only clamped at 0."""
    sib = parent - child
    if cls:
        return sib.clamp_min_(0.0)
    y2 = sib[:, 0, 0, 2].clamp_min(0.0)
    empty = sib[..., 0] <= 0.0
    sib[..., :2] = torch.where(empty[..., None], torch.zeros_like(sib[..., :2]), sib[..., :2])
    sib[:, 0, 0, 2] = y2
    return sib


def _impurity(stats: torch.Tensor, kind: str) -> tuple[torch.Tensor, torch.Tensor]:
    """stats [..., S] -> (impurity, weight)."""
    if kind == "variance":
        w = stats[..., 0]
        mean = stats[..., 1] / w.clamp_min(1e-300)
        imp = (stats[..., 2] / w.clamp_min(1e-300) - mean * mean).clamp_min(0.0)
        return torch.where(w > 0, imp, torch.zeros_like(imp)), w
    w = stats.sum(-1)
    p = stats / w.clamp_min(1e-300)[..., None]
    if kind == "gini":
        imp = 1.0 - (p * p).sum(-1)
    elif kind == "entropy":
        imp = -(torch.where(p > 0, p * torch.log2(p.clamp_min(1e-300)), torch.zeros_like(p))).sum(-1)
    else:
        raise ValueError(kind)
    return torch.where(w > 0, imp, torch.zeros_like(imp)), w


def _split_bundle_torch(H, kind, cls, nb, bin_ids, fm, min_inst, min_w, min_wfrac, min_w_node=None):
    """Reference of ``tree_split_kernel``: the per-node decision bundle (fp64
    [idx | gain | impurity | weight | wL | wR | values]) from histograms [k, F, B, S]."""
    k = H.shape[0]
    dev = H.device
    tot = H[:, 0].sum(1)                                   # [k, S] node stats (feature 0 bins)
    imp_p, w_p = _impurity(tot, kind)
    vals = (tot / w_p.clamp_min(1e-300)[:, None]) if cls else (tot[:, 1] / w_p.clamp_min(1e-300))[:, None]
    # split search: cumulative stats over bins (left = bins <= j)
    cum = H.cumsum(2)                                      # [k, F, B, S]
    left = cum[:, :, :-1]
    right = tot[:, None, None, :] - left
    W = w_p[:, None, None].clamp_min(1e-300)
    if cls:
        iL, wL = _impurity(left, kind)
        iR, wR = _impurity(right, kind)
        g = imp_p[:, None, None] - (wL / W) * iL - (wR / W) * iR
    else:
        # variance gain from (w, w*y) only: (SyL^2/wL + SyR^2/wR - Sy^2/W) / W
        wL, wR = left[..., 0], right[..., 0]
        sL, sR = left[..., 1], right[..., 1]
        sP = tot[:, 1][:, None, None]
        g = (sL * sL / wL.clamp_min(1e-300) + sR * sR / wR.clamp_min(1e-300) - sP * sP / W) / W
    ok = (wL >= min_inst) & (wR >= min_inst)
    if min_w_node is not None:
        mw = torch.as_tensor(np.asarray(min_w_node, dtype=np.float64), device=dev)[:, None, None]
    else:
        mw = (min_wfrac * w_p)[:, None, None] if min_wfrac > 0.0 else torch.full_like(W, min_w)
    ok &= (mw <= 0.0) | ((wL >= mw) & (wR >= mw))
    ok &= bin_ids[None, None, :] < nb[None, :, None]
    if fm is not None:
        ok &= torch.from_numpy(fm).to(dev)[:, :, None]
    g = torch.where(ok, g, torch.full_like(g, -math.inf))
    best = g.reshape(k, -1).max(1)
    # global child weights at the chosen split decide which child the next level scans
    wl_best = wL.reshape(k, -1).gather(1, best.indices[:, None])[:, 0]
    wr_best = wR.reshape(k, -1).gather(1, best.indices[:, None])[:, 0]
    return torch.cat([best.indices.to(torch.float64), best.values, imp_p, w_p, wl_best, wr_best, vals.reshape(-1)])


@dataclass
class Tree:
    """Flat tree: arrays indexed by Spark node id (1-based; 0 unused)."""
    feature: np.ndarray          # split feature (-1 = leaf)
    threshold: np.ndarray        # split threshold (value <= thr -> left)
    split_bin: np.ndarray
    value: np.ndarray            # [nodes, V]: mean (regression) or class distribution
    impurity: np.ndarray
    gain: np.ndarray
    count: np.ndarray            # weighted instance count
    num_features: int = 0

    @property
    def depth(self) -> int:
        ids = np.nonzero(self.count > 0)[0]
        return int(math.floor(math.log2(ids.max()))) if ids.size else 0

    @property
    def numNodes(self) -> int:
        return int(np.sum(self.count > 0))

    def leaf_of(self, X: torch.Tensor) -> torch.Tensor:
        """Spark node id of the leaf for each row of raw features X (device traversal)."""
        dev = X.device
        feat = torch.from_numpy(self.feature).to(dev)
        thr = torch.from_numpy(self.threshold).to(dev, torch.float64)
        node = torch.ones(X.shape[0], dtype=torch.int64, device=dev)
        for _ in range(self.depth + 1):
            f = feat[node]
            leaf = f < 0
            if bool(leaf.all()):
                break
            xv = X.gather(1, f.clamp_min(0)[:, None]).squeeze(1).to(torch.float64)
            nxt = torch.where(xv <= thr[node], 2 * node, 2 * node + 1)
            node = torch.where(leaf, node, nxt)
        return node

    def is_leaf(self, nid: int) -> bool:
        return bool(self.feature[nid] < 0 or 2 * nid >= len(self.feature) or self.count[2 * nid] == 0)

    def leaf_index_map(self) -> np.ndarray:
        """heap node id -> Spark leaf index (leaves numbered 0..numLeaves-1 in preorder,
        i.e. left to right, as ``leafCol`` / ``predictLeaf`` report them); -1 elsewhere."""
        out = -np.ones(len(self.feature), dtype=np.int64)
        nxt, stack = 0, [1]
        while stack:
            nid = stack.pop()
            if self.is_leaf(nid):
                out[nid], nxt = nxt, nxt + 1
            else:
                stack += [2 * nid + 1, 2 * nid]                 # left subtree first
        return out

    def leaf_index(self, X: torch.Tensor) -> torch.Tensor:
        """Preorder leaf index of each row (int64, device of X)."""
        return torch.from_numpy(self.leaf_index_map()).to(X.device)[self.leaf_of(X)]

    def predict_value(self, X: torch.Tensor) -> torch.Tensor:
        v = torch.from_numpy(self.value).to(X.device)
        return v[self.leaf_of(X)]

    def feature_importance(self) -> np.ndarray:
        imp = np.zeros(self.num_features)
        for i in np.nonzero(self.feature >= 0)[0]:
            imp[self.feature[i]] += self.gain[i] * self.count[i]
        s = imp.sum()
        return imp / s if s > 0 else imp


class TreeBuilder:
    """Grows trees over this rank's binned rows (collectives keep ranks in lockstep).

    Several trees grow TOGETHER (random forests: one tree per entry of ``w`` when it is a
    list of per-tree weight vectors, e.g. bootstrap counts): every tree owns a block of
    the position space ([t*n, (t+1)*n) of one row permutation, with its labels and
    weights moved alongside), so each level is ONE histogram launch, ONE all-reduce, ONE
    split launch and ONE partition for all trees -- Spark's "several trees per pass"
    (RandomForest.run groups nodes of all trees into one aggregation), without the
    per-tree launch and synchronisation overhead."""

    hist_subtraction = True         # False: scan every node at every level (reference path)
    batch_trees = True              # False: forests grow one tree at a time (reference path)
    final_from_parent = True        # False: the last level is histogrammed like any other (reference path)
    # GBT (fit_gbt): no per-row work at all while growing -- no leaf_apply of finished
    # segments, no routing pass at the last level; the caller runs ONE fused row-order
    # pass afterwards (ops/trees.gbt_leaf_pass) that applies every leaf and returns the
    # last level's w*y^2 sums for complete_final()
    defer_leaves = False

    def __init__(self, comm, bins: torch.Tensor, splits: list, y: torch.Tensor, w,
                 impurity: str, num_classes: int, max_depth: int = 5, min_instances: float = 1.0,
                 min_info_gain: float = 0.0, feature_fraction: float = 1.0, seed=0,
                 max_bins: int = 32, bins_t: torch.Tensor | None = None, min_weight_fraction: float = 0.0,
                 own_y: bool = False):
        self.comm, self.bins, self.splits = comm, bins, splits
        self.min_wfrac = float(min_weight_fraction)      # Spark minWeightFractionPerNode
        self.bins_t = bins_t if bins_t is not None else T.feature_major(bins)
        self.y = y
        self.ws = list(w) if isinstance(w, (list, tuple)) else [w]
        self.seeds = list(seed) if isinstance(seed, (list, tuple)) else [seed] * len(self.ws)
        if len(self.seeds) != len(self.ws):
            raise ValueError("one seed per tree")
        self.own_y = own_y               # y is a scratch fp32 buffer the build may overwrite
        self.kind = impurity
        self.cls = impurity in ("gini", "entropy")
        self.S = num_classes if self.cls else 3
        self.B = max(2, max(len(s) for s in splits) + 1) if splits else 2
        self.max_depth, self.min_inst, self.min_gain = max_depth, min_instances, min_info_gain
        self.ffrac = feature_fraction
        self.F = bins.shape[1]
        self.pending_y2 = None           # defer_leaves: (node ids [P, 2], w [P, 2], w*y [P, 2]) of the last level

    def build(self, leaf_acc: torch.Tensor | None = None, leaf_scale: float = 1.0):
        """Grow the (single) tree.  Returns (tree, None).

        ``leaf_acc`` (fp64 [n], boosting): every segment adds ``leaf_scale * value(leaf)``
        to leaf_acc[row] of its rows the moment it becomes a leaf
        (``tree_leaf_apply_kernel``)."""
        if len(self.ws) != 1:
            raise ValueError("build() grows one tree; use build_many()")
        return self._grow(leaf_acc, leaf_scale)[0], None

    def build_many(self) -> list:
        """Grow one tree per weight vector, in batches that keep positions in int32 and
        the per-batch row permutations within a quarter of free device memory."""
        n = max(1, self.bins.shape[0])
        tb = max(1, min(len(self.ws), (2 ** 31 - 1) // n))
        if self.bins.is_cuda:
            free, _ = torch.cuda.mem_get_info(self.bins.device)
            tb = max(1, min(tb, int(0.25 * free) // (26 * n)))
        trees, ws, seeds = [], self.ws, self.seeds
        for a in range(0, len(ws), tb):
            self.ws, self.seeds = ws[a:a + tb], seeds[a:a + tb]
            try:
                with progress.sub_range(a / len(ws), min(len(ws), a + tb) / len(ws)):
                    trees += self._grow(None, 1.0)
            finally:
                self.ws, self.seeds = ws, seeds
        return trees

    def _grow(self, leaf_acc, leaf_scale):
        dev = self.bins.device
        n = self.bins.shape[0]
        Tn = len(self.ws)
        F, B, S = self.F, self.B, self.S
        V = S if self.cls else 1
        max_nodes = 2 ** (self.max_depth + 1)
        feature = -np.ones((Tn, max_nodes), dtype=np.int64)
        threshold = np.zeros((Tn, max_nodes))
        split_bin = np.zeros((Tn, max_nodes), dtype=np.int64)
        value = np.zeros((Tn, max_nodes, V))
        impurity = np.zeros((Tn, max_nodes))
        gain = np.zeros((Tn, max_nodes))
        count = np.zeros((Tn, max_nodes))
        # one row permutation per tree, tree t at positions [t*n, (t+1)*n); labels and
        # weights travel with the rows in POSITION order (yp[p] belongs to row order[p]),
        # so the histogram kernel streams them instead of gathering a line per row
        order = torch.arange(n, dtype=torch.int32, device=dev)
        if Tn > 1:
            order = order.repeat(Tn)
        yp = self.y.to(torch.float32).contiguous()
        if Tn > 1:
            yp = yp.repeat(Tn)
        elif not (self.own_y and yp is self.y):
            yp = yp.clone()
        if all(w_ is None for w_ in self.ws):
            wp = None
        else:
            wp = torch.cat([torch.ones(n, dtype=torch.float32, device=dev) if w_ is None
                            else w_.to(dev, torch.float32).reshape(-1) for w_ in self.ws]).contiguous()
        # ping-pong buffers on the GPU: rows of finished leaves are never read again, so a
        # partition writes only the split segments into the spare buffers (no full copy)
        pingpong = order.is_cuda
        spare = torch.empty_like(order) if pingpong else None
        y_sp = torch.empty_like(yp) if pingpong else None
        w_sp = torch.empty_like(wp) if (pingpong and wp is not None) else None
        # segment bounds live on the HOST (a few hundred int64s): per level there are two
        # device->host copies (the split decisions, then the left counts of the partition)
        seg_lo = np.arange(Tn, dtype=np.int64) * n
        seg_hi = seg_lo + n
        seg_tree = np.arange(Tn, dtype=np.int64)
        seg_nid = np.ones(Tn, dtype=np.int64)
        rngs = [np.random.default_rng(sd) for sd in self.seeds]
        nb = torch.tensor([len(s_) for s_ in self.splits], device=dev)
        bin_ids = torch.arange(B - 1, device=dev)
        root_w = np.zeros(Tn)
        # histogram subtraction: below the root only the globally smaller child of each
        # split is scanned; its sibling is parent - smaller (histograms are additive), which
        # at least halves the rows the hist kernel touches per level and the all-reduce size
        parent_H = None                                           # [P, F, B, S] fp64, global
        small_right = None                                        # [P] bool (host): right child smaller
        for depth in range(self.max_depth + 1):
            progress.iteration(depth, self.max_depth + 1)
            k = len(seg_nid)
            if k == 0:
                break
            with trace("tree.hist"):
                if parent_H is None or not self.hist_subtraction:
                    H = T.node_hist(self.bins, order, yp, wp, seg_lo, seg_hi, np.arange(k), k, B, S, self.cls,
                                    ypos=True)
                    H = H.to(torch.float64).contiguous()
                    self.comm.all_reduce(H)                       # [k, F, B, S]
                else:
                    P = k // 2                                    # segments come as (left, right) pairs
                    pick_h = 2 * np.arange(P) + small_right.astype(np.int64)
                    Hs = T.node_hist(self.bins, order, yp, wp, seg_lo[pick_h], seg_hi[pick_h],
                                     np.arange(P), P, B, S, self.cls, ypos=True)
                    Hs = Hs.to(torch.float64).contiguous()
                    self.comm.all_reduce(Hs)
                    H = T.sibling_hists(Hs, parent_H, small_right, self.cls)
            with trace("tree.split"):
                fm = None
                if self.ffrac < 1.0:
                    m = max(1, int(math.ceil(self.ffrac * F)))
                    fm = np.zeros((k, F), dtype=bool)
                    for t in np.unique(seg_tree):                     # each tree draws from its own stream:
                        rows_t = np.nonzero(seg_tree == t)[0]         # m of F features per node, uniformly
                        keys = rngs[t].random((len(rows_t), F))
                        pick = np.argpartition(keys, m - 1, axis=1)[:, :m] if m < F else \
                            np.broadcast_to(np.arange(F), (len(rows_t), F))
                        fm[rows_t[:, None], pick] = True
                # min child weight: at the root a fraction of its total weight (Spark
                # minWeightFractionPerNode), below it the absolute value that gave, per tree
                mw_frac = self.min_wfrac if depth == 0 else 0.0
                mw_node = (self.min_wfrac * root_w[seg_tree]) if (depth > 0 and self.min_wfrac > 0.0) else None
                if H.is_cuda:
                    bundle_t = T.best_splits(H, nb, fm, self.kind, self.min_inst, 0.0, mw_frac, mw_node)
                else:
                    bundle_t = _split_bundle_torch(H, self.kind, self.cls, nb, bin_ids, fm, self.min_inst, 0.0,
                                                   mw_frac, mw_node)
                # ONE device->host copy of every per-node decision input
                bundle = bundle_t.cpu().numpy()
                bi = bundle[:k].astype(np.int64)
                bg, imp_np, w_np, wl_np, wr_np = (bundle[q * k:(q + 1) * k] for q in range(1, 6))
                vals_np = bundle[6 * k:].reshape(k, V)
                if depth == 0:
                    root_w = w_np.copy()
                bf, bb = bi // (B - 1), bi % (B - 1)
                do_split = (bg > self.min_gain) & (bg > 0) & np.isfinite(bg) & (depth < self.max_depth)
            old_order = order
            is_leaf = ~do_split                                # segments that end here
            if do_split.any() and depth == self.max_depth - 1 and self.final_from_parent:
                # children are at maxDepth, i.e. leaves: their stats come from the parent's
                # histogram (left = bins <= split bin of the split feature, right = rest) and
                # one routing pass applies the leaf values / sums the REG w*y^2 -- no
                # partition, no histogram and no split search for the last level
                with trace("tree.final_level"):
                    self._final_level(H, do_split, bf, bb, bg, seg_lo, seg_hi, seg_tree, seg_nid, order, yp, wp,
                                      leaf_acc, leaf_scale, value, impurity, count, feature, split_bin, threshold,
                                      gain)
                do_split = np.zeros_like(do_split)            # nothing left to grow
            if do_split.any():
                # the partition is launched first: the tree bookkeeping and the leaf
                # updates below run on the host while it executes
                with trace("tree.partition"):
                    st, sn = seg_tree[do_split], seg_nid[do_split]
                    s_lo, s_hi = seg_lo[do_split], seg_hi[do_split]
                    pay = (yp,) if wp is None else (yp, wp)
                    if pingpong:
                        pout = (y_sp,) if wp is None else (y_sp, w_sp)
                        new_order, nleft = T.partition(self.bins, order, s_lo, s_hi, bf[do_split], bb[do_split],
                                                       bins_t=self.bins_t, out=spare, payload=pay, payload_out=pout)
                        spare, order = order, new_order
                        y_sp, yp = yp, y_sp
                        w_sp, wp = wp, w_sp
                    else:
                        pout = tuple(t.clone() for t in pay)
                        order, nleft = T.partition(self.bins, order, s_lo, s_hi, bf[do_split], bb[do_split],
                                                   bins_t=self.bins_t, payload=pay, payload_out=pout)
                        yp, wp = pout[0], (pout[1] if len(pout) > 1 else None)
                    # integer gather (a boolean mask index would sync on the device-side nonzero)
                    parent_H = H.index_select(0, N.upload(np.nonzero(do_split)[0], dev))
                    small_right = (wr_np < wl_np)[do_split]
            value[seg_tree, seg_nid] = vals_np
            impurity[seg_tree, seg_nid] = imp_np
            count[seg_tree, seg_nid] = w_np
            if leaf_acc is not None and is_leaf.any() and not self.defer_leaves:
                with trace("tree.leaf_apply"):          # finished segments: rows in the pre-split order
                    lf = is_leaf
                    T.leaf_apply(old_order, seg_lo[lf], seg_hi[lf], value[seg_tree[lf], seg_nid[lf], 0] * leaf_scale,
                                 leaf_acc)
            if not do_split.any():
                break
            with trace("tree.partition"):
                feature[st, sn] = bf[do_split]
                split_bin[st, sn] = bb[do_split]
                threshold[st, sn] = [float(self.splits[f_][b_]) for f_, b_ in zip(bf[do_split], bb[do_split])]
                gain[st, sn] = bg[do_split]
                mid = s_lo + nleft.cpu().numpy().astype(np.int64)
                seg_lo = np.stack([s_lo, mid], 1).reshape(-1)
                seg_hi = np.stack([mid, s_hi], 1).reshape(-1)
                seg_tree = np.repeat(st, 2)
                seg_nid = np.stack([2 * sn, 2 * sn + 1], 1).reshape(-1)
            # empty local segments still participate (other ranks may have rows there)
        return [Tree(feature[t], threshold[t], split_bin[t], value[t], impurity[t], gain[t], count[t], F)
                for t in range(Tn)]

    def _final_level(self, H, do_split, bf, bb, bg, seg_lo, seg_hi, seg_tree, seg_nid, order, yp, wp, leaf_acc,
                     leaf_scale, value, impurity, count, feature, split_bin, threshold, gain):
        dev = H.device
        idx = np.nonzero(do_split)[0]
        P = len(idx)
        st, sn = seg_tree[idx], seg_nid[idx]
        feature[st, sn] = bf[idx]
        split_bin[st, sn] = bb[idx]
        threshold[st, sn] = [float(self.splits[f_][b_]) for f_, b_ in zip(bf[idx], bb[idx])]
        gain[st, sn] = bg[idx]
        idx_d, bf_d, bb_d = (N.upload(a.astype(np.int64), dev) for a in (idx, bf[idx], bb[idx]))
        Hp = H.index_select(0, idx_d)                                        # [P, F, B, S]
        ar = torch.arange(P, device=dev)
        left = Hp[ar, bf_d].cumsum(1)[ar, bb_d]                               # [P, S]
        tot = Hp[:, 0].sum(1)                                                 # node totals (feature 0)
        child = torch.stack([left, tot - left], 1).cpu().numpy()              # [P, 2, S]
        w_ch = child[..., :].sum(-1) if self.cls else child[..., 0]
        V = self.S if self.cls else 1
        if self.cls:
            vals = child / np.maximum(w_ch, 1e-300)[..., None]
        else:
            vals = (child[..., 1] / np.maximum(w_ch, 1e-300))[..., None]
        s_lo, s_hi = seg_lo[idx], seg_hi[idx]
        if self.defer_leaves:            # rows are routed (and y^2 summed) by the caller's leaf pass
            for side in (0, 1):
                nid = 2 * sn + side
                value[st, nid] = vals[:, side].reshape(P, V)
                count[st, nid] = w_ch[:, side]
            if not self.cls:
                self.pending_y2 = (np.stack([2 * sn, 2 * sn + 1], 1), child[..., 0], child[..., 1])
            else:
                imp, _ = _impurity(torch.from_numpy(child), self.kind)
                for side in (0, 1):
                    impurity[st, 2 * sn + side] = imp.numpy()[:, side]
            return
        y2 = T.final_level(self.bins, order, s_lo, s_hi, bf[idx], bb[idx], vals[:, 0, 0] * leaf_scale,
                           vals[:, 1, 0] * leaf_scale, yp, wp, leaf_acc, need_y2=not self.cls,
                           bins_t=self.bins_t) if (leaf_acc is not None or not self.cls) else None
        if self.cls:
            imp, _ = _impurity(torch.from_numpy(child), self.kind)
        else:
            y2 = y2.contiguous()
            self.comm.all_reduce(y2)
            stats = np.concatenate([child[..., :2], y2.cpu().numpy()[..., None]], -1)   # [P, 2, 3]
            imp, _ = _impurity(torch.from_numpy(stats), self.kind)
        imp = imp.numpy()
        for side in (0, 1):
            nid = 2 * sn + side
            value[st, nid] = vals[:, side].reshape(P, V)
            impurity[st, nid] = imp[:, side]
            count[st, nid] = w_ch[:, side]


    def complete_final(self, tree: "Tree", y2_leaves) -> None:
        """defer_leaves: the impurities of the last level's children from the leaf pass's
        per-leaf sums of w*y^2 (fp64 [2^maxDepth], all ranks reduced)."""
        if self.pending_y2 is None:
            return
        nid, w, wy = self.pending_y2
        y2 = np.asarray(y2_leaves, dtype=np.float64)[nid - (1 << self.max_depth)]
        stats = np.stack([w, wy, y2], -1)                                  # [P, 2, 3]
        imp, _ = _impurity(torch.from_numpy(stats), self.kind)
        tree.impurity[nid] = imp.numpy()
        self.pending_y2 = None


# ----------------------------------------------------------------------------- ensembles
@dataclass
class Ensemble:
    trees: list
    weights: list
    kind: str                         # "gbt" | "rf" | "dt"
    num_classes: int = 0
    losses: list = field(default_factory=list)


def subsample_weights(n_local, rows: torch.Tensor, rate: float, seed: int, bootstrap: bool) -> torch.Tensor | None:
    if bootstrap:
        return sampling.poisson_counts(rows, seed, rate).to(torch.float32)
    if rate < 1.0:
        return sampling.bernoulli_mask(rows, seed, rate).to(torch.float32)
    return None


GBT_FUSED_EPILOGUE = True      # False: per-level leaf_apply + last-level routing + gbt_grad_loss (reference path)


def fit_gbt(comm, bins, splits, y: torch.Tensor, w, loss: str = "logistic", max_iter: int = 20,
            step: float = 0.1, max_depth: int = 5, min_instances: float = 1.0, min_info_gain: float = 0.0,
            subsampling_rate: float = 1.0, seed: int = 0, feature_fraction: float = 1.0, rows=None,
            classification: bool = True, validation: torch.Tensor | None = None, validation_tol: float = 0.01,
            min_weight_fraction: float = 0.0) -> Ensemble:
    """Spark GradientBoostedTrees.boost: tree 0 fit on (scaled) labels with weight 1, then
    trees on pseudo-residuals with weight ``step``.

    ``validation`` (bool per local row, Spark's ``validationIndicatorCol``): those rows get
    weight 0 in every tree and, after each tree, the weighted mean validation loss is
    all-reduced; boosting stops once it improves by less than
    ``validation_tol * max(error, 0.01)`` and the ensemble is cut back to the best
    iteration (Spark runWithValidation semantics)."""
    dev = bins.device
    bins_t = T.feature_major(bins)                    # shared by every tree of the ensemble
    yy = y.to(torch.float64)
    if classification:
        yy = 2.0 * yy - 1.0
    wd = None if w is None else w.to(torch.float64)           # None: unit training weights
    w_val = None
    if validation is not None:
        vmask = validation.to(dev, torch.bool)
        wd0 = torch.ones_like(yy) if wd is None else wd
        w_val = torch.where(vmask, wd0, torch.zeros_like(wd0))
        wd = torch.where(vmask, torch.zeros_like(wd0), wd0)
        w = wd.float()
    Fm = torch.zeros_like(yy)
    fused = GBT_FUSED_EPILOGUE and max_depth <= T.LEAF_PASS_MAX_DEPTH and bins.dtype == torch.uint8
    trees, weights, losses = [], [], []
    best_err, best_m = math.inf, 0
    target = yy.to(torch.float32)                            # tree 0 fits the (scaled) labels
    for m in range(max_iter):
        progress.iteration(m, max_iter)
        sw = w
        if subsampling_rate < 1.0 and rows is not None:
            sub = subsample_weights(None, rows, subsampling_rate, seed + m, False)
            sw = sub if w is None else w * sub
        tb = TreeBuilder(comm, bins, splits, target, sw, "variance", 1, max_depth, min_instances,
                         min_info_gain, feature_fraction, seed + m, bins_t=bins_t,
                         min_weight_fraction=min_weight_fraction, own_y=True)
        tb.defer_leaves = fused
        wt = 1.0 if m == 0 else step
        with progress.sub_range(m / max_iter, (m + 1) / max_iter):
            tree, _ = tb.build(leaf_acc=Fm, leaf_scale=wt)      # Fm += wt * leaf value, per row
        with trace("gbt.update"):
            trees.append(tree)
            weights.append(wt)
            if fused:
                # ONE row-order pass: every row walks the tree (Fm += wt * leaf), the loss of the
                # updated ensemble, the next tree's residuals (into the target buffer: the build
                # is done with it) and the last level's w*y^2 sums
                nxt = target if m + 1 < max_iter else None
                need_y2 = tb.pending_y2 is not None
                buf, y2 = T.gbt_leaf_pass(bins, tree.feature, tree.split_bin, tree.value, wt, max_depth, loss, yy, Fm,
                                          sw, wd, w_val, m == 0, nxt, need_y2)
                if need_y2:
                    both = torch.cat([buf, y2]).contiguous()
                    comm.all_reduce(both)
                    buf = both[:4]
                    tb.complete_final(tree, both[4:].cpu().numpy())
                else:
                    comm.all_reduce(buf)
                target = nxt
            else:
                # one fused pass: this iteration's (validation) loss and the next tree's residuals
                target = torch.empty_like(target) if m + 1 < max_iter else None
                buf = T.gbt_grad_loss(loss, yy, Fm, wd, w_val, target)
                comm.all_reduce(buf)
            sums = buf.cpu().numpy()
            losses.append(float(sums[0] / max(sums[1], 1e-300)))
        if validation is not None:
            err = float(sums[2] / max(sums[3], 1e-300))
            if m == 0:
                best_err, best_m = err, 1
            elif best_err - err < validation_tol * max(err, 0.01):
                break
            elif err < best_err:
                best_err, best_m = err, m + 1
    if validation is not None:
        trees, weights, losses = trees[:best_m], weights[:best_m], losses[:best_m]
    return Ensemble(trees, weights, "gbt", 2 if classification else 0, losses)


def fit_forest(comm, bins, splits, y, w, num_trees: int, impurity: str, num_classes: int, max_depth: int,
               min_instances: float, min_info_gain: float, subsampling_rate: float, feature_fraction: float,
               seed: int, rows: torch.Tensor, bootstrap: bool, min_weight_fraction: float = 0.0) -> Ensemble:
    """Random forest: every tree's bootstrap (Poisson) or subsample weights, then all
    trees grown together level by level (``TreeBuilder.build_many``)."""
    ws = []
    with trace("forest.weights"):
        if rows.is_cuda and (bootstrap or subsampling_rate < 1.0):
            # every tree's bootstrap / subsample weights in one kernel (same draws)
            seeds = np.array([(seed * 7919 + t) & 0xFFFFFFFF for t in range(num_trees)], dtype=np.uint32)
            table = sampling.poisson_table(subsampling_rate, rows.device) if bootstrap else None
            wf = None if w is None else w.to(rows.device, torch.float32).contiguous()
            out = torch.empty((num_trees, rows.shape[0]), dtype=torch.float32, device=rows.device)
            r64 = rows.to(torch.int64).contiguous()
            N.check(N.kernels().o3s_forest_weights(r64.data_ptr(), r64.shape[0],
                                                   N.upload(seeds.view(np.int32), rows.device).data_ptr(),
                                                   num_trees, N.ptr(table), 0 if table is None else table.numel(),
                                                   float(subsampling_rate), N.ptr(wf), out.data_ptr(),
                                                   N.stream_of(out)), "forest_weights")
            ws = list(out)
        else:
            for t in range(num_trees):
                sw = subsample_weights(None, rows, subsampling_rate, seed * 7919 + t, bootstrap)
                if w is not None:
                    sw = w if sw is None else w * sw
                ws.append(sw)
    tb = TreeBuilder(comm, bins, splits, y, ws, impurity, num_classes, max_depth, min_instances,
                     min_info_gain, feature_fraction, [seed + 31 * t for t in range(num_trees)],
                     bins_t=T.feature_major(bins), min_weight_fraction=min_weight_fraction)
    trees = tb.build_many() if TreeBuilder.batch_trees else \
        [TreeBuilder(comm, bins, splits, y, ws[t], impurity, num_classes, max_depth, min_instances,
                     min_info_gain, feature_fraction, seed + 31 * t, bins_t=tb.bins_t,
                     min_weight_fraction=min_weight_fraction).build()[0] for t in range(num_trees)]
    return Ensemble(trees, [1.0] * num_trees, "rf", num_classes)


def feature_fraction_for(strategy: str, F: int, classification: bool, num_trees: int) -> float:
    s = str(strategy).lower()
    if s == "auto":
        s = "all" if num_trees == 1 else ("sqrt" if classification else "onethird")
    if s == "all":
        return 1.0
    if s == "sqrt":
        return math.ceil(math.sqrt(F)) / F
    if s == "log2":
        return max(1, math.ceil(math.log2(F))) / F
    if s == "onethird":
        return math.ceil(F / 3.0) / F
    try:
        v = float(s)
    except ValueError:
        raise ValueError(f"invalid featureSubsetStrategy {strategy}")
    if v >= 1.0 and float(v).is_integer() and "." not in s:
        return min(1.0, v / F)
    return v
