"""Trees: CPU path vs scikit-learn-level accuracy; GPU histogram kernel vs torch reference."""
import numpy as np
import pandas as pd
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.classification import (DecisionTreeClassifier, GBTClassifier, GBTClassificationModel,
                                                 RandomForestClassifier)
from orange3_spark_amd.ml.evaluation import BinaryClassificationEvaluator, RegressionEvaluator
from orange3_spark_amd.ml.regression import DecisionTreeRegressor, GBTRegressor, RandomForestRegressor


@pytest.fixture(scope="module")
def cpu():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _xor_data(s, n=4000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-1, 1, size=(n, 5))
    y = ((X[:, 0] > 0) ^ (X[:, 1] > 0.2)).astype(float)
    return s.createDataFrame(pd.DataFrame({"features": list(X), "label": y})), X, y


def test_decision_tree_learns_xor(cpu):
    df, X, y = _xor_data(cpu)
    m = DecisionTreeClassifier(maxDepth=3).fit(df)
    pred = m.transform(df).toPandas()["prediction"].values
    assert (pred == y).mean() > 0.97
    assert m.depth <= 3 and m.numNodes >= 5
    imp = m.featureImportances.toArray()
    assert imp[0] + imp[1] > 0.9


def test_random_forest_and_gbt(cpu):
    df, X, y = _xor_data(cpu, seed=1)
    rf = RandomForestClassifier(numTrees=10, maxDepth=4, seed=1).fit(df)
    acc = (rf.transform(df).toPandas()["prediction"].values == y).mean()
    assert acc > 0.9
    gbt = GBTClassifier(maxIter=10, maxDepth=3, seed=1).fit(df)
    out = gbt.transform(df)
    assert (out.toPandas()["prediction"].values == y).mean() > 0.95
    assert BinaryClassificationEvaluator().evaluate(out) > 0.97
    h = gbt.trainingLossHistory
    assert h[-1] < h[0]


def test_regressors(cpu):
    rng = np.random.default_rng(3)
    X = rng.uniform(-2, 2, size=(3000, 3))
    y = np.sin(X[:, 0]) * 2 + X[:, 1] ** 2
    df = cpu.createDataFrame(pd.DataFrame({"features": list(X), "label": y}))
    ev = RegressionEvaluator(metricName="r2")
    for est in (DecisionTreeRegressor(maxDepth=6), RandomForestRegressor(numTrees=8, maxDepth=6, seed=2),
                GBTRegressor(maxIter=20, maxDepth=4)):
        r2 = ev.evaluate(est.fit(df).transform(df))
        assert r2 > 0.85, (type(est).__name__, r2)


def test_gbt_save_load(cpu, tmp_path):
    df, X, y = _xor_data(cpu, n=500, seed=4)
    m = GBTClassifier(maxIter=3, maxDepth=2).fit(df)
    m.save(str(tmp_path / "gbt"))
    m2 = GBTClassificationModel.load(str(tmp_path / "gbt"))
    a = m.transform(df).toPandas()["probability"]
    b = m2.transform(df).toPandas()["probability"]
    assert np.allclose(np.stack(a.map(lambda v: v.toArray())), np.stack(b.map(lambda v: v.toArray())))


@pytest.mark.gpu
@pytest.mark.parametrize("F,B,S,cls", [(64, 32, 3, False), (10, 16, 3, False), (64, 32, 2, True), (100, 32, 4, True),
                                      (80, 32, 3, False), (96, 16, 2, True)])
def test_gpu_hist_matches_torch(gpu, F, B, S, cls):
    from orange3_spark_amd.ops import trees as T
    g = torch.Generator(device="cpu").manual_seed(F + B)
    n = 300_001
    bins = torch.randint(0, B, (n, F), generator=g, dtype=torch.uint8).to(gpu)
    y = (torch.randint(0, S, (n,), generator=g).float() if cls else torch.randn(n, generator=g)).to(gpu)
    w = torch.rand(n, generator=g).to(gpu)
    order = torch.randperm(n, generator=g).to(torch.int32).to(gpu)
    lo = torch.tensor([0, 1000, 200_000], device=gpu)
    hi = torch.tensor([1000, 200_000, n], device=gpu)
    nd = torch.tensor([0, 1, 2], device=gpu)
    a = T.node_hist(bins, order, y, w, lo, hi, nd, 3, B, S, cls, chunk=50_000)
    b = T.hist_torch(bins, order, y, w, lo, hi, nd, 3, B, S, cls)
    assert torch.allclose(a, b, rtol=1e-4, atol=1e-2)
    # position-ordered labels / weights (ypos): same histogram
    for ww in (w, None):
        ol = order.long()
        c = T.node_hist(bins, order, y[ol].contiguous(), None if ww is None else ww[ol].contiguous(), lo, hi, nd, 3,
                        B, S, cls, chunk=50_000, ypos=True)
        d = T.node_hist(bins, order, y, ww, lo, hi, nd, 3, B, S, cls, chunk=50_000)
        assert torch.equal(c, d)


@pytest.mark.gpu
def test_gpu_gbt_fit():
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.trees(400_000, 16, seed=1)
    m = GBTClassifier(maxIter=5, maxDepth=5).fit(df)
    auc = BinaryClassificationEvaluator().evaluate(m.transform(df))
    assert auc > 0.8


@pytest.mark.gpu
@pytest.mark.parametrize("feature_major", [False, True])
def test_gpu_partition_matches_torch(gpu, feature_major):
    from orange3_spark_amd.ops import trees as T
    g = torch.Generator().manual_seed(0)
    n, F = 200_003, 13
    bins = torch.randint(0, 32, (n, F), generator=g, dtype=torch.uint8)
    order = torch.randperm(n, generator=g).to(torch.int32)
    cuts = torch.tensor([0, 5, 70_000, 70_001, 150_000, n])           # includes 1-row and empty-ish segments
    s_lo, s_hi = cuts[:-1].clone(), cuts[1:].clone()
    s_feat = torch.randint(0, F, (s_lo.numel(),), generator=g)
    s_bin = torch.randint(0, 32, (s_lo.numel(),), generator=g)
    ref_o, ref_n = T.partition_torch(bins, order, s_lo, s_hi, s_feat, s_bin)
    bg = bins.to(gpu)
    got_o, got_n = T.partition(bg, order.to(gpu), s_lo.to(gpu), s_hi.to(gpu), s_feat.to(gpu),
                               s_bin.to(gpu), chunk=4096, bins_t=T.feature_major(bg) if feature_major else None)
    assert torch.equal(got_n.cpu(), ref_n)
    assert torch.equal(got_o.cpu(), ref_o)                             # stable -> identical permutation
    # payloads in position order move with their rows; positions outside the split
    # segments of the output buffers are left alone
    yv = torch.randn(n, generator=g)
    wv = torch.rand(n, generator=g)
    yp, wp = yv[order.long()].contiguous(), wv[order.long()].contiguous()
    outs = [torch.full((n,), -7.0, device=gpu) for _ in range(2)]
    o2 = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    sub = slice(1, 4)                                                  # split only segments 1..3
    T.partition(bg, order.to(gpu), s_lo[sub].to(gpu), s_hi[sub].to(gpu), s_feat[sub].to(gpu), s_bin[sub].to(gpu),
                chunk=4096, out=o2, payload=(yp.to(gpu), wp.to(gpu)), payload_out=outs)
    o2c = o2.cpu()
    inside = torch.zeros(n, dtype=torch.bool)
    inside[int(s_lo[1]):int(s_hi[3])] = True
    assert bool((o2c[~inside] == -1).all()) and bool((outs[0].cpu()[~inside] == -7.0).all())
    rows = o2c[inside].long()
    assert torch.equal(outs[0].cpu()[inside], yv[rows]) and torch.equal(outs[1].cpu()[inside], wv[rows])


@pytest.mark.parametrize("cls_model", ["dt_cls", "gbt_reg", "rf_cls"])
def test_hist_subtraction_matches_full_scan(cpu, cls_model):
    """Scanning only the smaller child per split (sibling = parent - child) grows the same
    trees as scanning every node."""
    from orange3_spark_amd.models.trees import TreeBuilder
    rng = np.random.default_rng(5)
    X = rng.uniform(-1, 1, size=(3000, 6))
    y = ((X[:, 0] > 0.1) ^ (X[:, 2] > -0.3)).astype(float)
    yr = np.round(X[:, 0] * 4 + X[:, 3] * 2 + rng.normal(size=3000))
    df = cpu.createDataFrame(pd.DataFrame({"features": list(X), "label": yr if cls_model == "gbt_reg" else y}))
    mk = {"dt_cls": lambda: DecisionTreeClassifier(maxDepth=6),
          "gbt_reg": lambda: GBTRegressor(maxDepth=5, maxIter=3),
          "rf_cls": lambda: RandomForestClassifier(numTrees=3, maxDepth=5, seed=2)}[cls_model]
    outs = []
    for flag in (True, False):
        TreeBuilder.hist_subtraction = flag
        try:
            outs.append(mk().fit(df).transform(df).toPandas()["prediction"].to_numpy())
        finally:
            TreeBuilder.hist_subtraction = True
    # same splits; GBT leaf values (real-valued residual sums) agree to rounding
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("cls", [False, True])
def test_gpu_hist_subtraction_exact_with_heavy_fractional_weights(gpu, cls):
    """Sibling = parent - child equals a direct scan of the sibling when weights are
    fractional and a bin's weight is past 2^24 (fp64 ordered slab sums), and
    the histogram is bitwise reproducible across launches."""
    from orange3_spark_amd.models.trees import _sibling
    from orange3_spark_amd.ops import trees as T
    g = torch.Generator().manual_seed(11)
    n, F, B = 400_003, 8, 16
    S = 3 if not cls else 2
    bins = torch.randint(0, B, (n, F), generator=g, dtype=torch.uint8)
    bins[: n // 2, 0] = 3                                           # one heavy bin in feature 0 ...
    bins[n // 2:, 0] %= 3                                           # ... that only the child populates
    y = (torch.randint(0, 2, (n,), generator=g).float() if cls else torch.randn(n, generator=g))
    w = 700.0 + torch.rand(n, generator=g) * 0.37                    # bin 3: ~1.4e8 > 2^24
    bins, y, w = bins.to(gpu), y.to(gpu), w.to(gpu)
    order = torch.arange(n, dtype=torch.int32, device=gpu)
    split = 8192 * 30                                               # item-aligned: child items = parent's first 30
    lo_p, hi_p = torch.tensor([0], device=gpu), torch.tensor([n], device=gpu)
    nd = torch.tensor([0], device=gpu)
    parent = T.node_hist(bins, order, y, w, lo_p, hi_p, nd, 1, B, S, cls)
    again = T.node_hist(bins, order, y, w, lo_p, hi_p, nd, 1, B, S, cls)
    assert parent.dtype == torch.float64 and torch.equal(parent, again)          # deterministic
    assert float(parent[0, 0, 3, :2].sum()) > 2 ** 24
    child = T.node_hist(bins, order, y, w, torch.tensor([0], device=gpu), torch.tensor([split], device=gpu),
                        nd, 1, B, S, cls)
    direct = T.node_hist(bins, order, y, w, torch.tensor([split], device=gpu), hi_p, nd, 1, B, S, cls)
    sib = _sibling(parent, child, cls)
    ref = T.hist_torch(bins, order, y, w, torch.tensor([split], device=gpu), hi_p, nd, 1, B, S, cls)
    torch.testing.assert_close(direct, ref, rtol=1e-6, atol=1.0)   # fp32 per-item partials, fp64 sums
    torch.testing.assert_close(sib, ref, rtol=1e-6, atol=1.0)
    assert bool((sib[0, 0, 3] == 0).all())                          # empty in the sibling: exactly empty
    assert bool((sib[..., 0] >= 0).all())


@pytest.mark.gpu
@pytest.mark.parametrize("n,F", [(1_000_003, 64), (4099, 12), (256, 68), (5, 4)])
def test_gpu_u8_transpose(gpu, n, F):
    from orange3_spark_amd.ops import trees as T
    b = torch.randint(0, 255, (n, F), dtype=torch.uint8, generator=torch.Generator().manual_seed(n)).to(gpu)
    assert torch.equal(T.feature_major(b).cpu(), b.cpu().t().contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("n,F,nb,bf16", [(100_003, 64, 32, False), (100_003, 64, 32, True), (2049, 16, 8, True),
                                         (100_000, 64, 32, True), (4098, 64, 32, False), (100_000, 128, 255, True),
                                         (5000, 7, 2, False), (777, 130, 255, False), (3, 1, 32, False),
                                         # the unrolled search-tree kernel at every depth it is built
                                         # for (16..256 bins) and 1, 2, 3, 5, 8 feature groups
                                         (50_001, 24, 16, True), (20_000, 8, 64, False), (65_537, 64, 64, True),
                                         (30_000, 40, 128, True), (10_007, 16, 256, False), (9_999, 40, 32, False)])
def test_gpu_bin_features_matches_bucketize(gpu, n, F, nb, bf16):
    """bin_features (vector kernel for F % 8 == 0: 8 features per lane, unrolled for the
    bin count when it has 16..256 bins; scalar kernel otherwise; fp32 or bf16 rows) ==
    torch.bucketize, and the feature-major copy the kernel writes == the transpose."""
    from orange3_spark_amd.models import trees as TR
    g = torch.Generator().manual_seed(F)
    X = torch.randn(n, F, generator=g)
    if bf16:
        X = X.to(torch.bfloat16).float()                          # exactly representable in bf16
    X[:, 0] = torch.round(X[:, 0] * 2) / 2                          # ties on thresholds
    splits = TR.find_splits(Session(SessionConf().set("o3s.device", "cpu")).comm, X, nb, 0)
    ref = torch.empty((n, F), dtype=torch.uint8)
    for f in range(F):
        t = torch.as_tensor(splits[f], dtype=torch.float32)
        ref[:, f] = torch.bucketize(X[:, f], t).to(torch.uint8) if t.numel() else 0
    got_d = TR.bin_features(X.to(gpu).to(torch.bfloat16) if bf16 else X.to(gpu), splits)
    got = got_d.cpu()
    assert torch.equal(got, ref)
    from orange3_spark_amd.ops import trees as T
    fm = getattr(got_d, "_o3s_feature_major", None)       # written by the binning kernel itself
    assert fm is not None and torch.equal(fm.cpu(), ref.t().contiguous())
    assert T.feature_major(got_d) is fm


def test_tree_models_predict_leaf_and_evaluate(cpu):
    df, X, y = _xor_data(cpu, n=1500, seed=3)
    rf = RandomForestClassifier(numTrees=4, maxDepth=4, seed=3).fit(df)
    leaves = rf.predictLeaf(X[0]).toArray()
    assert leaves.shape == (4,)
    for t, leaf in zip(rf._ens.trees, leaves):          # preorder leaf index in [0, numLeaves)
        m = t.leaf_index_map()
        n_leaves = int((m >= 0).sum())
        assert 0 <= leaf < n_leaves
        heap = int(t.leaf_of(torch.from_numpy(X[:1]))[0])
        assert m[heap] == leaf and t.feature[heap] < 0
    # leafCol: one preorder index per tree, matching predictLeaf row by row
    out = rf.copy({rf.leafCol: "leaf"}).transform(df).toPandas()
    got = np.stack(out["leaf"].map(lambda v: v.toArray()))
    np.testing.assert_array_equal(got[:5], np.stack([rf.predictLeaf(x).toArray() for x in X[:5]]))
    sm = rf.evaluate(df)
    pred = rf.transform(df).toPandas()["prediction"].to_numpy()
    assert abs(sm.accuracy - (pred == y).mean()) < 1e-12 and 0.5 < sm.areaUnderROC <= 1.0


def test_leaf_index_is_preorder():
    from orange3_spark_amd.models.trees import Tree
    # root 1 splits; 2 is a leaf; 3 splits into leaves 6, 7  -> preorder leaves 2, 6, 7
    size = 8
    feat = -np.ones(size, dtype=np.int64)
    feat[1], feat[3] = 0, 0
    cnt = np.zeros(size)
    cnt[[1, 2, 3, 6, 7]] = 1
    t = Tree(feat, np.zeros(size), np.zeros(size, dtype=np.int64), np.zeros((size, 1)), np.zeros(size),
             np.zeros(size), cnt, 1)
    m = t.leaf_index_map()
    assert (m[2], m[6], m[7]) == (0, 1, 2) and m[1] == -1 and m[3] == -1


def test_gbt_validation_indicator_stops_early(cpu):
    rng = np.random.default_rng(9)
    X = rng.uniform(-1, 1, size=(3000, 4))
    y = (X[:, 0] + 0.3 * rng.normal(size=3000) > 0).astype(float)
    val = rng.uniform(size=3000) < 0.3
    df = cpu.createDataFrame(pd.DataFrame({"features": list(X), "label": y, "isVal": val}))
    full = GBTClassifier(maxIter=40, maxDepth=3, stepSize=0.5).fit(df)
    es = GBTClassifier(maxIter=40, maxDepth=3, stepSize=0.5, validationIndicatorCol="isVal",
                       validationTol=0.01).fit(df)
    assert len(full.trees) == 40
    assert 1 <= len(es.trees) < 40                      # noisy label: validation loss plateaus early
    # training rows only: a fit on the train split alone grows the same first tree
    tr = cpu.createDataFrame(pd.DataFrame({"features": list(X[~val]), "label": y[~val]}))
    one = GBTClassifier(maxIter=1, maxDepth=3).fit(tr)
    np.testing.assert_allclose(es._ens.trees[0].value[:, 0], one._ens.trees[0].value[:, 0], atol=1e-9)


def test_min_weight_fraction_per_node(cpu):
    df, X, y = _xor_data(cpu, n=2000, seed=8)
    deep = DecisionTreeClassifier(maxDepth=8).fit(df)
    frac = DecisionTreeClassifier(maxDepth=8, minWeightFractionPerNode=0.2).fit(df)
    t = frac._ens.trees[0]
    leaves = [i for i in range(1, len(t.feature)) if t.count[i] > 0 and t.is_leaf(i)]
    assert min(t.count[i] for i in leaves) >= 0.2 * 2000 - 1e-9
    assert frac.numNodes < deep.numNodes
    with pytest.raises(ValueError):
        DecisionTreeClassifier(minWeightFractionPerNode=0.6).fit(df)


def test_partition_payload_torch():
    """CPU reference: payloads (position order) follow their rows through a partition."""
    from orange3_spark_amd.ops import trees as T
    g = torch.Generator().manual_seed(3)
    n, F = 1000, 5
    bins = torch.randint(0, 8, (n, F), generator=g, dtype=torch.uint8)
    order = torch.randperm(n, generator=g).to(torch.int32)
    yv = torch.randn(n, generator=g)
    yp = yv[order.long()].contiguous()
    lo, hi = torch.tensor([0, 400]), torch.tensor([400, n])
    out_y = yp.clone()
    new, _ = T.partition(bins, order, lo, hi, torch.tensor([1, 3]), torch.tensor([2, 5]), payload=(yp,),
                         payload_out=(out_y,))
    assert torch.equal(out_y, yv[new.long()])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,S", [("variance", 3), ("gini", 2), ("entropy", 5), ("gini", 12)])
def test_gpu_split_kernel_matches_torch(gpu, kind, S):
    """tree_split_kernel (one fused launch per level) == the torch split search."""
    from orange3_spark_amd.models.trees import _split_bundle_torch
    from orange3_spark_amd.ops import trees as T
    g = torch.Generator().manual_seed(S)
    k, F, B = 37, 20, 16
    H = torch.rand((k, F, B, S), generator=g, dtype=torch.float64) * 50
    if kind == "variance":
        H[..., 1] = torch.randn((k, F, B), generator=g, dtype=torch.float64) * 20
        H[..., 2] = 0.0
        H[:, 0, 0, 2] = 1e4
        H[:, 1:, :, :2] = H[:, :1, :, :2].expand(-1, F - 1, -1, -1)[:, :, torch.randperm(B, generator=g)]
    else:                                                             # every feature sees the node's rows
        H[:, 1:] = H[:, :1].expand(-1, F - 1, -1, -1)[:, :, torch.randperm(B, generator=g)]
    H[3] = 0.0                                                        # an empty node
    nb = torch.randint(1, B, (F,), generator=g)
    fm = (torch.rand((k, F), generator=g) < 0.5).numpy()
    bin_ids = torch.arange(B - 1)
    for fmask, mi, mw, mwf in ((None, 1.0, 0.0, 0.0), (fm, 30.0, 0.0, 0.0), (fm, 1.0, 0.0, 0.2), (None, 1.0, 90.0, 0.0)):
        ref = _split_bundle_torch(H, kind, kind != "variance", nb, bin_ids, fmask, mi, mw, mwf)
        got = T.best_splits(H.to(gpu), nb.to(gpu), fmask, kind, mi, mw, mwf).cpu()
        fin = torch.isfinite(ref[k:2 * k])
        assert torch.equal(fin, torch.isfinite(got[k:2 * k]))
        assert torch.equal(ref[:k][fin], got[:k][fin])                # same split (no exact ties here)
        torch.testing.assert_close(got[k:2 * k][fin], ref[k:2 * k][fin], rtol=1e-9, atol=1e-12)
        torch.testing.assert_close(got[2 * k:4 * k], ref[2 * k:4 * k], rtol=1e-12, atol=1e-12)
        torch.testing.assert_close(got[4 * k:6 * k][fin.repeat(2)], ref[4 * k:6 * k][fin.repeat(2)])
        torch.testing.assert_close(got[6 * k:], ref[6 * k:], rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("loss", ["logistic", "squared", "absolute"])
def test_gpu_gbt_grad_loss_matches_torch(gpu, loss):
    """gbt_grad_loss_kernel (fused loss sums + residuals) == the torch reference."""
    from orange3_spark_amd.ops import trees as T
    g = torch.Generator().manual_seed(7)
    n = 1_000_003
    yy = (torch.randint(0, 2, (n,), generator=g).double() * 2 - 1) if loss == "logistic" else \
        torch.randn(n, generator=g, dtype=torch.float64)
    Fm = torch.randn(n, generator=g, dtype=torch.float64) * 30            # large margins: stable loss needed
    w = torch.rand(n, generator=g, dtype=torch.float64)
    wv = torch.where(torch.rand(n, generator=g) < 0.2, w, torch.zeros_like(w))
    for ww, vv in ((None, None), (w, wv)):
        t_ref = torch.empty(n, dtype=torch.float32)
        ref = T.gbt_grad_loss(loss, yy, Fm, ww, vv, t_ref)
        t_got = torch.empty(n, dtype=torch.float32, device=gpu)
        got = T.gbt_grad_loss(loss, yy.to(gpu), Fm.to(gpu), None if ww is None else ww.to(gpu),
                              None if vv is None else vv.to(gpu), t_got).cpu()
        assert torch.isfinite(got).all()
        torch.testing.assert_close(got, ref, rtol=1e-10, atol=1e-8)
        torch.testing.assert_close(t_got.cpu(), t_ref, rtol=1e-6, atol=1e-6)


def _forest_batched_vs_sequential(session, dev_name):
    from orange3_spark_amd.models.trees import TreeBuilder
    rng = np.random.default_rng(9)
    X = rng.uniform(-1, 1, size=(4000, 7))
    y = ((X[:, 0] > 0.2) ^ (X[:, 3] > -0.1)).astype(float) + (X[:, 5] > 0.6)
    df = session.createDataFrame(pd.DataFrame({"features": list(X), "label": y}))
    outs = []
    for flag in (True, False):
        TreeBuilder.batch_trees = flag
        try:
            m = RandomForestClassifier(numTrees=6, maxDepth=5, seed=3, subsamplingRate=0.8,
                                       minWeightFractionPerNode=0.01).fit(df)
            outs.append((m.transform(df).toPandas()["probability"].map(lambda v: v.toArray()).tolist(),
                         [t.numNodes for t in m.trees]))
        finally:
            TreeBuilder.batch_trees = True
    np.testing.assert_allclose(np.array(outs[0][0]), np.array(outs[1][0]), rtol=1e-9, atol=1e-12)
    assert outs[0][1] == outs[1][1]


def test_forest_batched_equals_sequential(cpu):
    """Growing all trees of a forest together (one launch per level) builds the same
    trees as growing them one at a time (bootstrap, feature subsets, min weight fraction)."""
    _forest_batched_vs_sequential(cpu, "cpu")


@pytest.mark.gpu
def test_gpu_forest_batched_equals_sequential():
    s = Session(SessionConf().set("o3s.device", "cuda"))
    _forest_batched_vs_sequential(s, "cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("cls", [False, True])
def test_gpu_sibling_kernel_matches_torch(gpu, cls):
    """tree_sibling_kernel (level histogram assembly + residue cleaning) == torch path."""
    from orange3_spark_amd.ops import trees as T
    g = torch.Generator().manual_seed(4)
    P, F, B = 19, 9, 16
    S = 4 if cls else 3
    parent = torch.rand((P, F, B, S), generator=g, dtype=torch.float64) * 10
    Hs = parent * torch.rand((P, F, B, S), generator=g, dtype=torch.float64)
    Hs[0, 1, 2] = parent[0, 1, 2] + 1e-9                     # residue: sibling slightly negative
    if not cls:
        parent[:, 1:, :, 2] = 0.0
        Hs[:, 1:, :, 2] = 0.0
    sr = (torch.rand(P, generator=g) < 0.5).numpy()
    ref = T.sibling_hists(Hs, parent, sr, cls)
    got = T.sibling_hists(Hs.to(gpu), parent.to(gpu), sr, cls).cpu()
    assert torch.equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("bootstrap,rate", [(True, 1.0), (True, 0.7), (False, 0.6)])
def test_gpu_forest_weights_kernel_matches_sampling(gpu, bootstrap, rate, monkeypatch):
    """forest_weights_kernel draws bitwise the per-tree weights of the torch sampling path."""
    from orange3_spark_amd.models import trees as TR
    n = 100_003
    rows = torch.arange(5_000, 5_000 + n, dtype=torch.int64)
    w = torch.rand(n, generator=torch.Generator().manual_seed(1))
    ref = [TR.subsample_weights(None, rows, rate, 11 * 7919 + t, bootstrap) * w for t in range(3)]
    seen = {}

    class _Stop(Exception):
        pass

    def grab(self):
        seen["ws"] = [x.cpu() for x in self.ws]
        raise _Stop

    monkeypatch.setattr(TR.TreeBuilder, "build_many", grab)
    bins = torch.zeros((n, 2), dtype=torch.uint8, device=gpu)
    with pytest.raises(_Stop):
        TR.fit_forest(None, bins, [np.zeros(0), np.zeros(0)], torch.zeros(n, device=gpu), w.to(gpu), 3, "gini", 2,
                      3, 1.0, 0.0, rate, 1.0, 11, rows.to(gpu), bootstrap)
    for a, b in zip(seen["ws"], ref):
        assert torch.equal(a, b.float())


def _final_level_parity(session):
    from orange3_spark_amd.models.trees import TreeBuilder
    rng = np.random.default_rng(12)
    X = rng.uniform(-1, 1, size=(5000, 6))
    yc = ((X[:, 0] > 0.1) ^ (X[:, 2] > -0.3)).astype(float) + (X[:, 4] > 0.5)
    yr = np.sin(3 * X[:, 0]) + X[:, 1] * X[:, 3] + 0.1 * rng.normal(size=5000)
    w = rng.uniform(0.5, 2.0, size=5000)
    dfc = session.createDataFrame(pd.DataFrame({"features": list(X), "label": yc, "w": w}))
    dfr = session.createDataFrame(pd.DataFrame({"features": list(X), "label": yr, "w": w}))
    makers = [(dfr, lambda: GBTRegressor(maxDepth=4, maxIter=4, weightCol="w")),
              (dfc, lambda: DecisionTreeClassifier(maxDepth=5, impurity="entropy")),
              (dfc, lambda: RandomForestClassifier(numTrees=3, maxDepth=4, seed=2)),
              (dfr, lambda: RandomForestRegressor(numTrees=3, maxDepth=5, seed=4, weightCol="w"))]
    for df, mk in makers:
        outs = []
        for flag in (True, False):
            TreeBuilder.final_from_parent = flag
            try:
                m = mk().fit(df)
            finally:
                TreeBuilder.final_from_parent = True
            ts = getattr(m, "_ens", None)
            trees = ts.trees if ts is not None else [m._tree]
            outs.append((m.transform(df).toPandas()["prediction"].to_numpy(),
                         [(t.feature.copy(), t.value.copy(), t.impurity.copy(), t.count.copy()) for t in trees]))
        # GPU: fp32 per-item slab partials grouped differently (per bin of the parent vs per
        # child row block) -> leaf sums agree to ~1e-7 relative, compounding over boosting
        np.testing.assert_allclose(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-6)
        for a, b in zip(outs[0][1], outs[1][1]):
            assert np.array_equal(a[0], b[0])
            for q in (1, 2, 3):
                np.testing.assert_allclose(a[q], b[q], rtol=1e-5, atol=1e-6)


def test_final_level_from_parent_matches_full_level(cpu):
    """Leaves at maxDepth from the parent's histogram + one routing pass == histogramming
    the last level (values, impurities, counts, predictions)."""
    _final_level_parity(cpu)


@pytest.mark.gpu
def test_gpu_final_level_from_parent_matches_full_level():
    _final_level_parity(Session(SessionConf().set("o3s.device", "cuda")))


def _gbt_fused_parity(session):
    """fit_gbt's fused row-order epilogue (ops/trees.gbt_leaf_pass: every leaf applied,
    the loss, the next residuals and the last level's w*y^2 in one pass) == the reference
    path (per-level leaf_apply + last-level routing + gbt_grad_loss): trees, losses,
    impurities, predictions -- logistic with validation + subsampling, squared and
    absolute losses with weights."""
    from orange3_spark_amd.models import trees as TR
    rng = np.random.default_rng(21)
    n = 6000
    X = rng.uniform(-1, 1, size=(n, 7))
    yc = ((X[:, 0] > 0.1) ^ (X[:, 2] > -0.3)).astype(float)
    yr = np.sin(3 * X[:, 0]) + X[:, 1] * X[:, 3] + 0.1 * rng.normal(size=n)
    w = rng.uniform(0.5, 2.0, size=n)
    val = rng.random(n) < 0.2
    dfc = session.createDataFrame(pd.DataFrame({"features": list(X), "label": yc, "w": w, "v": val}))
    dfr = session.createDataFrame(pd.DataFrame({"features": list(X), "label": yr, "w": w}))
    makers = [(dfc, lambda: GBTClassifier(maxDepth=5, maxIter=6, subsamplingRate=0.8, seed=3,
                                          validationIndicatorCol="v", validationTol=0.0)),
              (dfr, lambda: GBTRegressor(maxDepth=4, maxIter=5, weightCol="w", lossType="squared")),
              (dfr, lambda: GBTRegressor(maxDepth=6, maxIter=4, weightCol="w", lossType="absolute"))]
    for df, mk in makers:
        outs = []
        for flag in (True, False):
            TR.GBT_FUSED_EPILOGUE = flag
            try:
                m = mk().fit(df)
            finally:
                TR.GBT_FUSED_EPILOGUE = True
            ens = m._ens
            outs.append((m.transform(df).toPandas()["prediction"].to_numpy(), np.array(ens.losses),
                         [(t.feature.copy(), t.value.copy(), t.impurity.copy(), t.count.copy()) for t in ens.trees]))
        np.testing.assert_allclose(outs[0][0], outs[1][0], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(outs[0][1], outs[1][1], rtol=1e-9)
        assert len(outs[0][2]) == len(outs[1][2])
        for a, b in zip(outs[0][2], outs[1][2]):
            assert np.array_equal(a[0], b[0])
            # impurity = E[y^2] - mean^2 from fp32 w*y^2 partials summed in another grouping:
            # ~1e-7 absolute noise where the variance cancels to ~0
            for q in (1, 2, 3):
                np.testing.assert_allclose(a[q], b[q], rtol=1e-5, atol=1e-6)


def test_gbt_fused_epilogue_matches_reference(cpu):
    _gbt_fused_parity(cpu)


@pytest.mark.gpu
def test_gpu_gbt_fused_epilogue_matches_reference():
    _gbt_fused_parity(Session(SessionConf().set("o3s.device", "cuda")))


@pytest.mark.gpu
@pytest.mark.parametrize("loss,first", [("logistic", True), ("logistic", False), ("squared", False)])
def test_gpu_gbt_leaf_pass_matches_torch_and_is_deterministic(gpu, loss, first):
    """The fused GBT epilogue kernel (gbt_leaf_pass_kernel) against its torch reference on
    a random depth-6 tree: Fm update, loss partials, next residuals and the per-leaf
    w*y^2 sums; two launches give bitwise-equal results (per-wave LDS sums)."""
    from orange3_spark_amd.ops import trees as T
    g = torch.Generator().manual_seed(5)
    n, F, D = 200_003, 64, 6
    bins = torch.randint(0, 32, (n, F), generator=g, dtype=torch.uint8)
    nodes = 1 << (D + 1)
    rng = np.random.default_rng(3)
    feature = -np.ones(nodes, dtype=np.int64)
    split_bin = np.zeros(nodes, dtype=np.int64)
    for nid in range(1, 1 << D):                       # a full tree except a few early leaves
        if nid in (5, 12):
            continue
        if nid > 1 and feature[nid // 2] < 0:
            continue
        feature[nid] = rng.integers(0, F)
        split_bin[nid] = rng.integers(0, 31)
    value = rng.normal(size=(nodes, 1))
    yy = (torch.randint(0, 2, (n,), generator=g).double() * 2 - 1) if loss == "logistic" else torch.randn(n, generator=g,
                                                                                                  dtype=torch.float64)
    Fm0 = torch.randn(n, generator=g, dtype=torch.float64) * 0.3
    wt = torch.rand(n, generator=g)
    out = []
    for dev in ("cpu", gpu, gpu):
        Fm = Fm0.clone().to(dev)
        tgt = torch.empty(n, dtype=torch.float32, device=dev)
        buf, y2 = T.gbt_leaf_pass(bins.to(dev), feature, split_bin, value, 0.5, D, loss, yy.to(dev), Fm, wt.to(dev),
                                  None, None, first, tgt, True)
        out.append((Fm.cpu(), buf.cpu(), y2.cpu(), tgt.cpu()))
    ref, a, b = out
    torch.testing.assert_close(a[0], ref[0], rtol=0, atol=0)
    torch.testing.assert_close(a[1], ref[1], rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(a[2], ref[2], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a[3], ref[3], rtol=1e-6, atol=1e-7)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
