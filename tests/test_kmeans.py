"""KMeans: CPU path vs scikit-learn, GPU kernels vs fp64 PyTorch references."""
import numpy as np
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.clustering import KMeans, KMeansModel
from orange3_spark_amd.ops import kmeans as K


@pytest.fixture(scope="module")
def cpu():
    return Session(SessionConf().set("o3s.device", "cpu"))


def test_kmeans_cpu_recovers_blobs(cpu):
    df = cpu.synthetic.blobs(3000, 8, k=5, seed=1, spread=0.3)
    m = KMeans(k=5, seed=3, maxIter=50).fit(df)
    C = np.array(m.clusterCenters())
    true = df.true_centers.double().numpy()
    d = ((C[:, None] - true[None]) ** 2).sum(-1)
    assert d.min(0).max() < 0.05
    assert m.summary.trainingCost < 3000 * 8 * 0.3 ** 2 * 1.5
    out = m.transform(df)
    assert out.select("prediction").count() == 3000


def test_kmeans_cost_close_to_sklearn(cpu):
    from sklearn.cluster import KMeans as SK
    rng = np.random.default_rng(0)
    X = rng.normal(size=(2000, 6))
    import pandas as pd
    df = cpu.createDataFrame(pd.DataFrame({"features": list(X)}))
    m = KMeans(k=8, seed=1, maxIter=100, tol=1e-8).fit(df)
    sk = SK(n_clusters=8, n_init=5, random_state=0).fit(X)
    assert m.summary.trainingCost < sk.inertia_ * 1.05


def test_kmeans_save_load(cpu, tmp_path):
    df = cpu.synthetic.blobs(500, 4, k=3, seed=2)
    m = KMeans(k=3, seed=0).fit(df)
    m.save(str(tmp_path / "km"))
    m2 = KMeansModel.load(str(tmp_path / "km"))
    assert np.allclose(np.array(m.clusterCenters()), np.array(m2.clusterCenters()))
    assert m2.getK() == 3 and m2.uid == m.uid


@pytest.mark.gpu
@pytest.mark.parametrize("D,Kc", [(128, 1024), (64, 100), (32, 7), (100, 33), (160, 64)])
def test_gpu_assign_matches_fp64(gpu, D, Kc):
    g = torch.Generator(device="cpu").manual_seed(D + Kc)
    X = (torch.randn(20011, D, generator=g) * 3).to(gpu)
    C = (torch.randn(Kc, D, generator=g) * 3).to(gpu)
    a, d = K.assign(X, C)
    ra, rd = K.assign_torch(X, C)
    # exact agreement except for near-ties: check the chosen centre is optimal to 1e-4 rel
    Xd, Cd = X.double(), C.double()
    dist_sel = ((Xd - Cd[a.long()]) ** 2).sum(1)
    assert torch.all(dist_sel <= rd.double() * (1 + 1e-4) + 1e-3)
    assert (a == ra).float().mean() > 0.999
    assert torch.allclose(d.double(), rd.double(), rtol=1e-4, atol=1e-2)


@pytest.mark.gpu
def test_gpu_update_matches_index_add(gpu):
    g = torch.Generator(device="cpu").manual_seed(5)
    X = torch.randn(100003, 128, generator=g).to(gpu)
    a = torch.randint(0, 1000, (100003,), generator=g, dtype=torch.int32).to(gpu)
    s, c = K.update(X, a, 1024)
    rs, rc = K.update_torch(X, a, 1024)
    assert torch.allclose(s, rs, atol=1e-3)
    assert torch.equal(c, rc)
    s2, _ = K.update(X, a, 1024)
    assert torch.equal(s.clone(), s2)   # deterministic


@pytest.mark.gpu
@pytest.mark.parametrize("k,D", [(2, 128), (7, 64), (300, 200), (4099, 32)])
def test_gpu_update_small_and_odd_k(gpu, k, D):
    """Small k gives huge buckets (the stable ballot scatter must stay linear); K=4099 runs
    with a smaller per-chunk row count; ties to the fp64 index_add reference."""
    g = torch.Generator(device="cpu").manual_seed(k)
    n = 300_001
    X = torch.randn(n, D, generator=g).to(gpu)
    a = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(gpu)
    a[:70_000] = 0                          # one very large bucket
    s, c = K_update(X, a, k)
    rs, rc = K.update_torch(X, a, k)
    assert torch.allclose(s, rs, atol=5e-3)
    assert torch.equal(c, rc)
    s2, _ = K_update(X, a, k)
    assert torch.equal(s, s2)


def K_update(X, a, K_):
    s, c = K.update(X, a, K_)
    return s.clone(), c.clone()


@pytest.mark.gpu
def test_gpu_kmeans_fit(gpu):
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.blobs(200_000, 128, k=64, seed=4, spread=0.5)
    m = KMeans(k=64, seed=1, maxIter=30).fit(df)
    assert m.summary.trainingCost / 200_000 < 128 * 0.25 * 1.3


@pytest.mark.gpu
@pytest.mark.parametrize("D", [200, 130])
def test_gpu_kmeans_fit_wide_d_uses_update_kernel(gpu, D, monkeypatch):
    """D in (160, 256] or D % 4 != 0: the assign kernel falls back to torch, but the fit
    still takes the slab update kernel (its own D <= 256 gate) and agrees with
    an all-torch fit."""
    calls = {"n": 0}
    real = K.update

    def spy(*a, **kw):
        calls["n"] += 1
        return real(*a, **kw)
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.blobs(50_000, D, k=8, seed=2, spread=0.5)
    monkeypatch.setattr(K, "update", spy)
    m = KMeans(k=8, seed=1, maxIter=10, tol=0.0).fit(df)
    assert calls["n"] >= 1
    monkeypatch.setattr(K, "update_kernel_ok", lambda X: False)
    ref = KMeans(k=8, seed=1, maxIter=10, tol=0.0).fit(df)
    np.testing.assert_allclose(np.array(m.clusterCenters()), np.array(ref.clusterCenters()), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("D,Kc,kind", [(128, 1024, "blobs"), (128, 1024, "uniform"), (64, 100, "uniform"),
                                       (160, 64, "blobs"), (32, 7, "uniform"), (100, 33, "blobs")])
def test_gpu_screen_assign_matches_split_and_fp64(gpu, D, Kc, kind):
    """One-MFMA screen + exact re-solve of near-ties == the split-precision kernel's
    answer (and the fp64 reference), on easy (blobs) and tie-heavy (uniform) data."""
    g = torch.Generator(device="cpu").manual_seed(D * 7 + Kc)
    n = 40_003
    if kind == "blobs":
        C = torch.rand(Kc, D, generator=g) * 20 - 10
        X = C[torch.randint(0, Kc, (n,), generator=g)] + torch.randn(n, D, generator=g)
        C = C + 0.3 * torch.randn(Kc, D, generator=g)
    else:
        X = torch.rand(n, D, generator=g)
        C = torch.rand(Kc, D, generator=g)
    X, C = X.to(gpu), C.to(gpu)
    P = K.prepare_centers(C)
    st = {}
    a1, d1 = K.assign(X, C, P, mode="screen", stats=st)
    a3, d3 = K.assign(X, C, P, mode="split")
    ra, rd = K.assign_torch(X, C)
    if kind == "blobs":
        assert st["flagged"] < n // 100                 # easy data: almost every row screened
    assert (a1 == a3).float().mean() > 0.9999
    assert (a1 == ra).float().mean() > 0.999
    torch.testing.assert_close(d1.double(), rd.double(), rtol=1e-4, atol=1e-2)
    # a row whose centre is duplicated is an exact tie: it must be flagged and re-solved
    C2 = torch.cat([C, C[:1]])
    a2, _ = K.assign(X[:4096], C2, mode="screen", stats=st)
    ref2, _ = K.assign(X[:4096], C2, mode="split")
    assert torch.equal(a2, ref2)


@pytest.mark.gpu
def test_gpu_screen_auto_falls_back_when_most_rows_tie(gpu):
    g = torch.Generator(device="cpu").manual_seed(3)
    X = torch.rand(20_000, 64, generator=g).to(gpu) * 1e-3      # all rows nearly equidistant
    C = torch.rand(256, 64, generator=g).to(gpu)
    st = {}
    K.assign(X, C, mode="auto", stats=st)
    assert st["mode"] == "screen"
    if st["flagged"] > K.SCREEN_MAX_FLAG_FRACTION * X.shape[0]:
        st2 = {}
        K.assign(X, C, mode="auto", stats=st2)
        assert st2["mode"] == "split" and st2["flagged"] == X.shape[0]   # split path taken directly


@pytest.mark.gpu
@pytest.mark.parametrize("D,Kc", [(128, 1024), (64, 100), (160, 64), (32, 7)])
def test_gpu_pair_screen_matches_split(gpu, D, Kc):
    """The pair screen (top-3 tracking; two-centre near ties settled by exact distances
    in-kernel) assigns exactly like the split kernel and flags no more rows than the plain
    screen; duplicated centres (exact ties) resolve to the lower index like the split."""
    g = torch.Generator(device="cpu").manual_seed(D + Kc)
    n = 40_009
    X = (torch.rand(n, D, generator=g) * 2 - 1).to(gpu)
    C = X[torch.randperm(n, generator=g)[:Kc].to(gpu)].clone() * 0.5
    P = K.prepare_centers(C)
    s1, s2 = {}, {}
    a1, d1 = K.assign(X, C, P, mode="screen", stats=s1)
    a2, d2 = K.assign(X, C, P, mode="pair", stats=s2)
    a3, d3 = K.assign(X, C, P, mode="split")
    assert s2["flagged"] <= s1["flagged"]
    assert (a2 == a3).float().mean() > 0.9999 and (a1 == a3).float().mean() > 0.9999
    torch.testing.assert_close(d2, d3, rtol=1e-4, atol=1e-4)
    C2 = torch.cat([C, C[:1]])
    b2, _ = K.assign(X[:4096], C2, mode="pair")
    ref2, _ = K.assign(X[:4096], C2, mode="split")
    assert torch.equal(b2, ref2)


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [1e-5, 1.0, 3e4])
def test_gpu_fp16_screen_scaling_keeps_exact_argmin(gpu, scale):
    """The fp16 screen scales x and -2c by powers of two (no fp16 overflow or precision
    loss at any data scale): every screened row agrees with the split kernel, and on
    structureless data the fp16 bound leaves far fewer near ties than bf16 would."""
    g = torch.Generator(device="cpu").manual_seed(11)
    n, D, Kc = 30_011, 128, 512
    X = ((torch.rand(n, D, generator=g) * 2 - 1) * scale).to(gpu)
    C = X[torch.randperm(n, generator=g)[:Kc].to(gpu)].clone()
    P = K.prepare_centers(C)
    st = {}
    a1, d1 = K.assign(X, C, P, mode="screen", stats=st)
    a3, d3 = K.assign(X, C, P, mode="split")
    assert torch.equal(a1, a3)
    # the split kernel's ||x||^2 + ||c||^2 - 2 x.c cancels to ~1e-7 ||x||^2 where the
    # screen's direct (x - c)^2 gives 0 (rows that are centres)
    torch.testing.assert_close(d1, d3, rtol=1e-4, atol=1e-3 * scale * scale)
    assert st["flagged"] < 0.5 * n, st
    assert P.h16.abs().max() <= 2 ** 15 and torch.isfinite(P.h16.float()).all()


def test_screen_scales_and_bound():
    """Power-of-two scales keep |v s| <= 2^15 and the bound grows with the data."""
    assert K._pow2_scale(1.0) == 2.0 ** 15 and K._pow2_scale(3.0) == 2.0 ** 13
    assert K._pow2_scale(0.0) == 1.0 and K._pow2_scale(float("nan")) == 1.0
    for a in (1e-30, 1e-3, 7.0, 6e4, 1e30):
        s = K._pow2_scale(a)
        assert a * s <= 2 ** 15 < 2 * a * s
    P = K.prepare_centers(torch.tensor([[3.0, 4.0], [0.0, 1.0]]))
    assert P.cmax == 5.0 and P.ms == K._pow2_scale(8.0)
    ex, e0, ee = K.screen_bound(P, 2.0 ** 10, 2)
    # [3, 4] and [0, 1] times -2 ms are exact in fp16: only the accumulation terms remain
    assert P.dm == 0.0 and P.mmax == 10.0
    assert 0 < ex < 1e-4 and 10.0 <= ee < 10.01 and 0 < e0 < 1e-3


@pytest.mark.parametrize("kind", ["uniform", "randn", "midpoints", "tiny", "huge", "offset"])
def test_screen_bound_covers_the_fp16_product_error(kind):
    """The screen bound (Cauchy-Schwarz on the actual fp16 rounding errors of x and -2c)
    covers |x^.m^ - x.m| computed exactly in fp64 for every (row, centre) pair -- including
    values on fp16 rounding midpoints, fp16-subnormal scales and offsets -- and is several
    times tighter than the per-element worst case on data with full mantissas."""
    g = torch.Generator().manual_seed(hash(kind) % 1000)
    n, D, Kc = 3000, 96, 64
    if kind == "uniform":
        X = torch.rand(n, D, generator=g)
    elif kind == "randn":
        X = torch.randn(n, D, generator=g) * 3
    elif kind == "midpoints":                 # x xs exactly halfway between fp16 neighbours
        X = (torch.randint(2 ** 10, 2 ** 11, (n, D), generator=g).float() + 0.5) / 2 ** 11
    elif kind == "tiny":
        X = torch.randn(n, D, generator=g) * 1e-30
    elif kind == "huge":
        X = torch.randn(n, D, generator=g) * 1e30
    else:
        X = torch.randn(n, D, generator=g) + 1e3
    C = X[torch.randperm(n, generator=g)[:Kc]] * 0.9
    P = K.prepare_centers(C)
    xs = K._pow2_scale(float(X.abs().max()))
    E = K.row_bound(X, P, xs)                                       # [n] fp64
    xh = (X * xs).half().double() / xs
    mh = P.h16[:Kc, :D].double() / P.ms
    err = (xh @ mh.T - X.double() @ (-2.0 * C.double()).T).abs()   # exact products in fp64
    assert bool((err <= E[:, None]).all()), float((err / E[:, None]).max())
    if kind in ("uniform", "randn"):
        worst = 2.0 ** -10 * X.double().norm(dim=1) * float(2 * C.double().norm(dim=1).max())
        assert float((E / worst).max()) < 0.6


@pytest.mark.gpu
def test_gpu_assign_after_address_reuse_with_larger_scale(gpu):
    """Regression for the round-3 fault (d527171): the fp16 data scale and the screen
    state were cached by tensor ADDRESS.  Assign on A, free it, allocate B with 1000x larger
    values at the recycled address, assign again: B's result must match the fp64 argmin
    (a stale scale overflows fp16 -> negative / garbage indices)."""
    g = torch.Generator(device="cpu").manual_seed(5)
    n, D, Kc = 40_000, 64, 96
    CA = torch.randn(Kc, D, generator=g).to(gpu)
    A = torch.randn(n, D, generator=g).to(gpu)
    a0, _ = K.assign(A, CA)
    ptr = A.data_ptr()
    del A
    torch.cuda.synchronize()
    B = torch.empty(n, D, dtype=torch.float32, device=gpu)          # same size: the caching allocator reuses the block
    B.copy_(torch.randn(n, D, generator=g).to(gpu) * 1000.0)
    CB = CA * 1000.0
    assert B.data_ptr() == ptr, "allocator did not recycle the address (test precondition)"
    a1, d1 = K.assign(B, CB)
    assert int(a1.min()) >= 0 and int(a1.max()) < Kc
    Bd, Cd = B.double(), CB.double()
    full = torch.cdist(Bd, Cd) ** 2
    best = full.min(1).values
    sel = full.gather(1, a1.long()[:, None])[:, 0]
    assert torch.all(sel <= best * (1 + 1e-5) + 1e-6 * best.max())
    assert (a1.long() == full.argmin(1)).float().mean() > 0.999
    torch.testing.assert_close(d1.double(), best, rtol=1e-4, atol=1e-3 * 1000.0 ** 2)


@pytest.mark.gpu
@pytest.mark.parametrize("D", [32, 64, 100, 128])
def test_gpu_presplit_screen_matches_plain_screen(gpu, D, monkeypatch):
    """The pre-split screen (fp16 hi / lo rows built once per data version and loaded as
    MFMA fragments) assigns exactly like the plain screen and its exact distances agree."""
    g = torch.Generator(device="cpu").manual_seed(D)
    X = (torch.randn(50_001, D, generator=g) * 2).to(gpu)
    C = X[torch.randperm(50_001, generator=g)[:256].to(gpu)].clone() + 0.01
    P = K.prepare_centers(C)
    monkeypatch.setattr(K, "PRESPLIT", False)
    a0, d0 = K.assign(X, C, P, mode="screen")
    monkeypatch.setattr(K, "PRESPLIT", True)
    a1, d1 = K.assign(X, C, P, mode="screen")
    assert K._XSPLIT[0] is not None and K._XSPLIT[0]() is X
    assert torch.equal(a0, a1)
    torch.testing.assert_close(d0, d1, rtol=1e-6, atol=1e-5)
    ra, _ = K.assign(X, C, P, mode="split")
    assert (a1 == ra).float().mean() > 0.999
    X.mul_(2.0)                                          # new data version: the cache must rebuild
    a2, _ = K.assign(X, C * 2.0, K.prepare_centers(C * 2.0), mode="screen")
    assert torch.equal(a2, a0)


def test_lloyd_cost_from_cluster_sums_equals_direct_cost():
    """The Lloyd iterations take their cost from the cluster sums (sum ||x||^2 - sum_a
    (2 c_a.S_a - n_a ||c_a||^2), fp64) so the assign pass needs no per-row distance; the
    history entry of iteration 1 equals the direct sum of squared distances to the initial
    centres, and a weighted fit keeps the per-row form."""
    from orange3_spark_amd.models.kmeans import fit_kmeans
    from orange3_spark_amd.parallel.comm import LocalComm
    g = torch.Generator().manual_seed(4)
    X = torch.randn(3000, 6, generator=g, dtype=torch.float32) * 3 + 1
    C0 = X[:5].double().clone()
    res = fit_kmeans(LocalComm("cpu"), X, 5, max_iter=1, tol=0.0, initial=C0)
    d = torch.cdist(X.double(), C0).pow(2).min(1).values.sum()
    assert abs(res.history[0] - float(d)) <= 1e-9 * float(d)
    w = torch.rand(3000, generator=g, dtype=torch.float32)
    resw = fit_kmeans(LocalComm("cpu"), X, 5, max_iter=1, tol=0.0, initial=C0, weights=w)
    dw = (torch.cdist(X.double(), C0).pow(2).min(1).values * w.double()).sum()
    assert abs(resw.history[0] - float(dw)) <= 1e-6 * float(dw)


def test_lloyd_cost_far_from_origin_keeps_its_digits():
    """Data offset by 1e6 with unit spread: the sums-based cost is taken about the global
    mean, so the history keeps ~1e-9 relative accuracy instead of cancelling."""
    from orange3_spark_amd.models.kmeans import fit_kmeans
    from orange3_spark_amd.parallel.comm import LocalComm
    g = torch.Generator().manual_seed(5)
    X = torch.randn(4000, 8, generator=g, dtype=torch.float64).float() + 1e6
    C0 = X[:6].double().clone()
    res = fit_kmeans(LocalComm("cpu"), X, 6, max_iter=1, tol=0.0, initial=C0)
    d = torch.cdist(X.double(), C0).pow(2).min(1).values.sum()
    assert abs(res.history[0] - float(d)) <= 1e-8 * float(d)


@pytest.mark.gpu
def test_gpu_presplit_dropped_after_fit(gpu, monkeypatch):
    """The presplit copy of X (as large as X) does not outlive the fit."""
    from orange3_spark_amd.models.kmeans import fit_kmeans
    from orange3_spark_amd.parallel.comm import LocalComm
    monkeypatch.setattr(K, "PRESPLIT", True)
    X = torch.randn(60_000, 64, device=gpu)
    fit_kmeans(LocalComm(gpu), X, 64, max_iter=3, seed=1)
    assert K._XSPLIT == [None, None, None]


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,D", [(16, 300, 8), (256, 1500, 64), (1024, 4100, 128)])
def test_gpu_kmeanspp_kernel_matches_torch_steps(gpu, k, m, D):
    """The k-means++ kernels (two launches per greedy step) pick the same candidates as the step-by-step torch formulation from
    the same draws (fp32-rounded coordinates, fp64 sums; then the shared Lloyd refinement
    gives the same centres)."""
    from orange3_spark_amd.models.kmeans import _local_kmeanspp
    g = torch.Generator(device="cpu").manual_seed(k + m)
    P = (torch.randn(m, D, generator=g, dtype=torch.float64) * 3).to(gpu)
    w = torch.randint(1, 50, (m,), generator=g).to(torch.float64).to(gpu)
    a = _local_kmeanspp(P, w, k, seed=5, iters=0, kernel=True)
    b = _local_kmeanspp(P, w, k, seed=5, iters=0, kernel=False)
    assert torch.equal(a, b)
    a = _local_kmeanspp(P, w, k, seed=5, iters=30, kernel=True)
    b = _local_kmeanspp(P, w, k, seed=5, iters=30, kernel=False)
    torch.testing.assert_close(a, b, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_gpu_approx_assign_is_within_the_screen_bound(gpu):
    """mode='approx' (k-means|| rounds): the screen's pick without the near-tie re-solve --
    its distance is the exact distance to the picked centre, never more than the screen
    bound above the true minimum, and most picks are the exact argmin."""
    from orange3_spark_amd.ops import kmeans as K
    g = torch.Generator().manual_seed(11)
    X = (torch.randn(200_000, 64, generator=g) * 3).to(gpu)
    C = X[torch.randperm(200_000, generator=g)[:700].to(gpu)] + 0.01
    a1, d1 = K.assign(X, C, mode="approx")
    a2, d2 = K.assign(X, C, mode="split")
    P = K.prepare_centers(C)
    bound = 2 * K.row_bound(X, P, K.x_scale(X)).float()
    dx = ((X - C[a1.long()]) ** 2).sum(1)
    assert torch.allclose(d1, dx, rtol=1e-4, atol=1e-3)
    assert bool((d1 <= d2 + bound + 1e-3).all())
    assert float((a1 == a2).float().mean()) > 0.9


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["blobs", "uniform"])
def test_gpu_hamerly_lloyd_equals_full_screens(gpu, kind, monkeypatch):
    """Lloyd with Hamerly bounds (models/kmeans.py: only rows whose moved bounds no longer
    certify their centre are screened again, cluster sums updated by the rows that changed)
    gives the iterations of the every-row screen: the same centres, costs and sizes -- and
    on clustered data later iterations screen a small fraction of the rows."""
    from orange3_spark_amd.models import kmeans as KM
    s = Session(SessionConf().set("o3s.device", "cuda"))
    if kind == "blobs":
        df = s.synthetic.blobs(400_000, 64, k=50, seed=4, spread=0.4)
    else:
        g = torch.Generator().manual_seed(2)
        import pandas as pd
        X = torch.rand(300_000, 32, generator=g)
        df = s.createDataFrame(pd.DataFrame({"features": list(X.numpy().astype(np.float64))}))
    out = []
    for flag in (True, False):
        monkeypatch.setattr(KM, "HAMERLY", flag)
        m = KMeans(k=50, seed=7, maxIter=12, tol=0.0).fit(df)
        out.append((np.array(m.clusterCenters()), m.summary.trainingCost, list(m.summary.clusterSizes),
                    list(KM.LAST_HAMERLY_STATS)))
    (c1, cost1, n1, st), (c0, cost0, n0, _) = out
    # the running sums add the changed rows' fp32 slab partials instead of re-summing all
    # rows: centres agree to ~1e-7 relative (a row exactly on a boundary may then flip)
    assert sum(abs(a - b) for a, b in zip(n1, n0)) <= 2
    np.testing.assert_allclose(c1, c0, rtol=1e-5, atol=1e-6)
    assert cost1 == pytest.approx(cost0, rel=1e-6)
    assert len(st) >= 2 and st[0]["changed"] is None                    # the first iteration screens all
    if kind == "blobs":
        assert min(x["screened"] for x in st[1:]) < 0.2 * 400_000, st


@pytest.mark.gpu
def test_gpu_bounds_recheck_matches_torch(gpu):
    """The Hamerly bound update kernel (two passes, block-prefix compaction): the same
    moved bounds and the same ascending recheck list as the torch reference."""
    g = torch.Generator().manual_seed(9)
    n, Kc = 1_000_003, 77
    a = torch.randint(0, Kc, (n,), generator=g, dtype=torch.int32)
    ub = torch.rand(n, generator=g) * 2
    lb = ub + torch.randn(n, generator=g) * 0.3
    lb[::1000] = float("nan")
    bnd = torch.stack([ub, lb], 1).contiguous()
    delta = torch.rand(Kc, generator=g) * 0.05
    dmax = float(delta.max())
    b_ref = bnd.clone()
    m_ref, r_ref = K.bounds_recheck(a, b_ref, delta, dmax)
    b_gpu = bnd.to(gpu)
    m, r = K.bounds_recheck(a.to(gpu), b_gpu, delta.to(gpu), dmax)
    assert m == m_ref and torch.equal(r.cpu(), r_ref)
    torch.testing.assert_close(b_gpu.cpu(), b_ref, rtol=0, atol=0, equal_nan=True)
    m2, r2 = K.bounds_recheck(a.to(gpu), bnd.clone().to(gpu), delta.to(gpu), dmax, max_rows=10)
    assert m2 == m_ref and r2 is None


def test_centred_moments_far_from_origin():
    """The one-pass centring (sums about a shared shift row, then the exact recentring
    identity) equals the two-pass mean / sum ||x - m||^2 on data offset by 1e6."""
    from orange3_spark_amd.models.kmeans import _centred_moments
    from orange3_spark_amd.parallel.comm import LocalComm
    g = torch.Generator().manual_seed(9)
    X = (torch.randn(5000, 12, generator=g, dtype=torch.float64) + 1e6).float()
    m, ss = _centred_moments(LocalComm("cpu"), X)
    Xd = X.double()
    mr = Xd.mean(0)
    torch.testing.assert_close(m, mr, rtol=0, atol=1e-9)
    ref = ((Xd - mr) ** 2).sum()
    assert abs(float(ss) - float(ref)) <= 1e-9 * float(ref)


@pytest.mark.gpu
@pytest.mark.parametrize("n,D", [(100_003, 128), (4097, 96), (5, 4), (70_000, 160)])
def test_gpu_moments_kernel_matches_fp64(gpu, n, D):
    """kmeans_moments_kernel (one pass, fp64 sums of x - shift and ||x - shift||^2 in
    per-block partials) equals the fp64 torch sums."""
    g = torch.Generator().manual_seed(n + D)
    X = ((torch.randn(n, D, generator=g) * 3) + 1e4).to(gpu)
    shift = X[0].clone()
    s1, s2 = K.moments(X, shift)
    d = X.double() - shift.double()
    torch.testing.assert_close(s1, d.sum(0), rtol=1e-12, atol=1e-6)
    torch.testing.assert_close(s2, (d * d).sum(), rtol=1e-12, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("n,D", [(100_003, 128), (5, 4), (70_000, 160)])
def test_gpu_cost_kernel_matches_fp64(gpu, n, D):
    """kmeans_cost_kernel: sum ||x - C[a]||^2 from the rows equals the fp64 torch sum."""
    g = torch.Generator().manual_seed(n + 3 * D)
    X = (torch.randn(n, D, generator=g) * 2 + 5).to(gpu)
    C = (torch.randn(37, D, generator=g) + 5).to(gpu)
    a = torch.randint(0, 37, (n,), generator=g).to(gpu).to(torch.int32)
    got = K.cost(X, a, C)
    ref = ((X.double() - C.double()[a.long()]) ** 2).sum()
    torch.testing.assert_close(got, ref, rtol=1e-7, atol=0)
