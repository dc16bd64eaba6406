"""Property-based tests (hypothesis) of the pure building blocks whose edge cases are
shard and segment boundaries: GuiParam coercion, the stable level
partition, work-item planning, leaf application, per-row sampling keys and Spark's
preorder leaf numbering."""
import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from orange3_spark_amd.ops import sampling
from orange3_spark_amd.ops import trees as T
from orangecontrib.spark_amd.utils.gui_param import coerce

SET = settings(max_examples=60, deadline=None)


@SET
@given(st.integers(-10**12, 10**12))
def test_coerce_integer_literals(i):
    v = coerce(str(i))
    assert v == i and type(v) is int


@SET
@given(st.floats(allow_nan=False, allow_infinity=False, width=64))
def test_coerce_float_literals(f):
    v = coerce(repr(f))
    assert isinstance(v, (int, float)) and v == f


@SET
@given(st.text(alphabet="abcxyz_", min_size=1, max_size=12))
def test_coerce_text_stays_text(s):
    assert coerce(s) == (s if s not in ("None",) else None)


@SET
@given(st.lists(st.integers(0, 40), min_size=1, max_size=8), st.integers(0, 2**31 - 1))
def test_partition_is_stable_and_complete(seg_lens, seed):
    rng = np.random.default_rng(seed)
    n = int(sum(seg_lens)) + 3
    F = 3
    bins = torch.from_numpy(rng.integers(0, 8, (n, F)).astype(np.uint8))
    order = torch.from_numpy(rng.permutation(n).astype(np.int32))
    lo = np.concatenate([[0], np.cumsum(seg_lens)[:-1]]).astype(np.int64)
    hi = lo + np.asarray(seg_lens, dtype=np.int64)
    feat = rng.integers(0, F, len(seg_lens))
    b = rng.integers(0, 8, len(seg_lens))
    new, nleft = T.partition(bins, order, lo, hi, feat, b)
    o, nw = order.numpy(), new.numpy()
    for s_, (a, e) in enumerate(zip(lo, hi)):
        seg = o[a:e]
        go = bins.numpy()[seg, feat[s_]] <= b[s_]
        ref = np.concatenate([seg[go], seg[~go]])
        np.testing.assert_array_equal(nw[a:e], ref)
        assert int(nleft[s_]) == int(go.sum())
    np.testing.assert_array_equal(nw[hi[-1]:], o[hi[-1]:])          # rows outside every segment untouched


@SET
@given(st.lists(st.integers(0, 300), min_size=1, max_size=12), st.integers(1, 64))
def test_hist_plan_covers_every_row_once_in_order(seg_lens, chunk):
    lo = np.concatenate([[0], np.cumsum(seg_lens)[:-1]]).astype(np.int64)
    hi = lo + np.asarray(seg_lens, dtype=np.int64)
    p = T._HistPlan(lo, hi, np.arange(len(lo)), chunk, torch.device("cpu"))
    it_lo, it_hi = p.it_lo.numpy(), p.it_hi.numpy()
    assert np.all(it_hi - it_lo <= chunk) and np.all(it_hi > it_lo)
    covered = np.concatenate([np.arange(a, b) for a, b in zip(it_lo, it_hi)]) if p.n_items else np.zeros(0)
    np.testing.assert_array_equal(covered, np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]))
    # runs: each segment's items, in order, in runs of <= 64 (the fixed fp64 summation order)
    r_lo, r_cnt = p.r_lo.numpy(), p.r_cnt.numpy()
    s0, sn = p.s_run0.numpy(), p.s_nrun.numpy()
    first = 0
    for s_ in range(len(lo)):
        n_it = -(-int(hi[s_] - lo[s_]) // chunk)
        items = [i for r in range(s0[s_], s0[s_] + sn[s_]) for i in range(r_lo[r], r_lo[r] + r_cnt[r])]
        assert items == list(range(first, first + n_it)) and all(c <= 64 for c in r_cnt)
        first += n_it


@SET
@given(st.lists(st.integers(0, 50), min_size=1, max_size=6), st.integers(0, 2**31 - 1))
def test_leaf_apply_adds_each_rows_leaf_value(seg_lens, seed):
    rng = np.random.default_rng(seed)
    n = int(sum(seg_lens))
    order = torch.from_numpy(rng.permutation(n).astype(np.int32))
    lo = np.concatenate([[0], np.cumsum(seg_lens)[:-1]]).astype(np.int64)
    hi = lo + np.asarray(seg_lens, dtype=np.int64)
    val = rng.normal(size=len(lo))
    acc = torch.zeros(n, dtype=torch.float64)
    T.leaf_apply(order, lo, hi, val, acc)
    ref = np.zeros(n)
    for v, a, b in zip(val, lo, hi):
        ref[order.numpy()[a:b]] += v
    np.testing.assert_allclose(acc.numpy(), ref)


@SET
@given(st.integers(1, 5000), st.lists(st.integers(0, 5000), min_size=1, max_size=5), st.integers(0, 2**31 - 1),
       st.floats(0.0, 1.0))
def test_sampling_masks_are_shard_invariant(n, cuts, seed, frac):
    """Row keys are a pure function of (seed, global row): any sharding gives the same rows."""
    rows = torch.arange(n, dtype=torch.int64)
    full = sampling.bernoulli_mask(rows, seed, frac)
    bounds = sorted({0, n, *[c % (n + 1) for c in cuts]})
    parts = [sampling.bernoulli_mask(rows[a:b], seed, frac) for a, b in zip(bounds[:-1], bounds[1:])]
    assert torch.equal(torch.cat(parts), full)


@SET
@given(st.integers(0, 2**31 - 1), st.integers(1, 6))
def test_leaf_index_is_preorder_on_random_trees(seed, depth):
    from orange3_spark_amd.models.trees import Tree
    rng = np.random.default_rng(seed)
    size = 2 ** (depth + 1)
    feat = -np.ones(size, dtype=np.int64)
    cnt = np.zeros(size)

    def grow(nid, d):
        cnt[nid] = 1
        if d < depth and rng.uniform() < 0.7:
            feat[nid] = 0
            grow(2 * nid, d + 1)
            grow(2 * nid + 1, d + 1)
    grow(1, 0)
    t = Tree(feat, np.zeros(size), np.zeros(size, dtype=np.int64), np.zeros((size, 1)), np.zeros(size),
             np.zeros(size), cnt, 1)
    leaves = []

    def visit(nid):
        if t.is_leaf(nid):
            leaves.append(nid)
        else:
            visit(2 * nid)
            visit(2 * nid + 1)
    visit(1)
    m = t.leaf_index_map()
    assert [m[i] for i in leaves] == list(range(len(leaves)))
    assert int((m >= 0).sum()) == len(leaves)


if __name__ == "__main__":
    pytest.main([__file__])


@pytest.mark.gpu
def test_gpu_sampling_draws_bitwise_equal_cpu():
    """hash_uniform_kernel == the torch draws (uniform, Bernoulli mask, Poisson counts)."""
    from orange3_spark_amd.ops import sampling
    rows = torch.cat([torch.arange(0, 100_000), torch.arange(2 ** 33, 2 ** 33 + 1000)])
    g = rows.to("cuda")
    for seed, stream in ((0, 0), (12345, 7), (-3, 11), (2 ** 40 + 5, 1)):
        assert torch.equal(sampling.uniform(g, seed, stream).cpu(), sampling.uniform(rows, seed, stream))
    assert torch.equal(sampling.bernoulli_mask(g, 9, 0.37).cpu(), sampling.bernoulli_mask(rows, 9, 0.37))
    assert torch.equal(sampling.poisson_counts(g, 5, 1.0).cpu(), sampling.poisson_counts(rows, 5, 1.0))
