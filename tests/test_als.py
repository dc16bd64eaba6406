"""ALS: explicit/implicit on CPU vs a numpy reference; GPU kernel vs torch; CG vs exact."""
import numpy as np
import pandas as pd
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.evaluation import RegressionEvaluator
from orange3_spark_amd.ml.recommendation import ALS, ALSModel
from orange3_spark_amd.models import als as AE


@pytest.fixture(scope="module")
def cpu():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _ratings(n_u=60, n_i=40, rank=3, density=0.5, seed=0):
    rng = np.random.default_rng(seed)
    U = rng.normal(size=(n_u, rank))
    V = rng.normal(size=(n_i, rank))
    mask = rng.uniform(size=(n_u, n_i)) < density
    u, i = np.nonzero(mask)
    r = (U @ V.T)[u, i] + 0.01 * rng.normal(size=u.size)
    return pd.DataFrame({"user": u * 3 + 7, "item": i * 5 + 1, "rating": r})


def _numpy_als(pdf, rank, iters, reg, implicit, alpha, X, Y):
    users = np.unique(pdf.user.values)
    items = np.unique(pdf.item.values)
    ui = np.searchsorted(users, pdf.user.values)
    ii = np.searchsorted(items, pdf.item.values)
    r = pdf.rating.values
    X, Y = X.copy(), Y.copy()

    def solve(nrows, rows, cols, F, Fother_tf):
        out = np.zeros((nrows, rank))
        for u in range(nrows):
            sel = rows == u
            Fg = F[cols[sel]]
            rr = r[sel]
            if implicit:
                c1 = alpha * np.abs(rr)
                A = Fother_tf + (Fg * c1[:, None]).T @ Fg + reg * (rr > 0).sum() * np.eye(rank)
                b = ((1 + c1) * (rr > 0)) @ Fg
            else:
                A = Fg.T @ Fg + reg * sel.sum() * np.eye(rank)
                b = rr @ Fg
            out[u] = np.linalg.solve(A, b)
        return out
    for _ in range(iters):
        X = solve(len(users), ui, ii, Y, Y.T @ Y)
        Y = solve(len(items), ii, ui, X, X.T @ X)
    return X, Y


@pytest.mark.parametrize("implicit", [False, True])
def test_als_matches_numpy_reference(cpu, implicit):
    pdf = _ratings(seed=1)
    df = cpu.createDataFrame(pdf)
    m = ALS(rank=3, maxIter=5, regParam=0.05, implicitPrefs=implicit, alpha=2.0, seed=3).fit(df)
    # rebuild the same initial factors the engine used
    users, items = np.unique(pdf.user), np.unique(pdf.item)
    X0 = AE.init_factors(0, len(users), 3, 3, "cpu", False).double().numpy()
    Y0 = AE.init_factors(0, len(items), 3, 3 ^ 0x5A5A, "cpu", False).double().numpy()
    X, Y = _numpy_als(pdf, 3, 5, 0.05, implicit, 2.0, X0, Y0)
    assert np.allclose(m._U.double().numpy(), X, atol=1e-4)
    assert np.allclose(m._V.double().numpy(), Y, atol=1e-4)


def test_als_explicit_fits_low_rank(cpu):
    pdf = _ratings(n_u=80, n_i=50, seed=2, density=0.6)
    df = cpu.createDataFrame(pdf)
    m = ALS(rank=3, maxIter=15, regParam=0.01, seed=1).fit(df)
    rmse = RegressionEvaluator(labelCol="rating", metricName="rmse").evaluate(m.transform(df))
    assert rmse < 0.1
    recs = m.recommendForAllUsers(3).collect()
    assert len(recs) == 80 and len(recs[0].recommendations) == 3


def test_als_cold_start_and_save(cpu, tmp_path):
    pdf = _ratings(seed=3)
    df = cpu.createDataFrame(pdf)
    m = ALS(rank=2, maxIter=3, seed=0, coldStartStrategy="drop").fit(df)
    test = cpu.createDataFrame(pd.DataFrame({"user": [7, 99999], "item": [1, 1]}))
    assert m.transform(test).count() == 1
    m.save(str(tmp_path / "als"))
    m2 = ALSModel.load(str(tmp_path / "als"))
    assert torch.allclose(m2._U.cpu(), m._U.cpu()) and m2.rank == 2


@pytest.mark.gpu
@pytest.mark.parametrize("R", [10, 64, 100, 128, 129, 200, 255])
def test_gpu_als_pass_matches_torch(gpu, R):
    from orange3_spark_amd.ops import als as A
    g = torch.Generator(device="cpu").manual_seed(R)
    n, m, nnz = 3000, 2000, 60000
    rows = torch.sort(torch.randint(0, n, (nnz,), generator=g)).values
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n), 0)
    cols = torch.randint(0, m, (nnz,), generator=g, dtype=torch.int32)
    coef = torch.rand(nnz, generator=g)
    F = torch.randn(m, R, generator=g)
    V = torch.randn(n, R, generator=g)
    for mode in (0, 1):
        a = A.pass_(mode, indptr.to(gpu), cols.to(gpu), coef.to(gpu), F.to(gpu), V.to(gpu) if mode == 0 else None)
        b = A.pass_torch(mode, indptr, cols, coef, F, V)
        assert torch.allclose(a.cpu(), b, rtol=1e-4, atol=1e-3)
    coef2 = torch.rand(nnz, generator=g)
    mv, rhs = A.pass_both(indptr.to(gpu), cols.to(gpu), coef.to(gpu), F.to(gpu), V.to(gpu), coef2.to(gpu))
    assert torch.allclose(mv.cpu(), A.pass_torch(0, indptr, cols, coef, F, V), rtol=1e-4, atol=1e-3)
    assert torch.allclose(rhs.cpu(), A.pass_torch(1, indptr, cols, coef2, F, None), rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_gpu_als_cg_close_to_exact():
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.ratings(20000, 3000, 400000, rank=8, seed=1, implicit=True)
    ex = ALS(rank=16, maxIter=4, implicitPrefs=True, alpha=1.0, seed=1).fit(df)
    users = df.column_data("user").data.long()
    items = df.column_data("item").data.long()
    r = df.column_data("rating").data
    res = AE.fit_als(s.comm, users, items, r, 16, 4, 0.1, True, 1.0, 1, cg_iters=8, exact=False)
    pe = (ex._U @ ex._V.T)
    pc = (res.U @ res.V.T)
    assert ((pe - pc).norm() / pe.norm()).item() < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("implicit,R", [(True, 128), (False, 40), (True, 200)])
def test_gpu_fused_cg_matches_torch_cg(implicit, R):
    """als_cg_kernel (fused CG vector updates) vs the same CG as separate torch ops."""
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.ratings(30000, 4000, 500000, rank=8, seed=2, implicit=implicit)
    users = df.column_data("user").data.long()
    items = df.column_data("item").data.long()
    r = df.column_data("rating").data
    out = []
    for fused in (True, False):
        AE.FUSED_CG = fused
        try:
            res = AE.fit_als(s.comm, users, items, r, R, 2, 0.1, implicit, 1.0, 3, cg_iters=3, exact=False)
        finally:
            AE.FUSED_CG = True
        out.append((res.U.clone(), res.V.clone()))
    for a, b in zip(out[0], out[1]):
        assert ((a - b).norm() / b.norm()).item() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("implicit,R", [(True, 128), (False, 64), (True, 32), (False, 96)])
def test_gpu_dense_gram_cholesky_matches_exact_fp64(implicit, R, monkeypatch):
    """MFMA Gram (als_gram_kernel) + batched Cholesky == the fp64 dense reference solve of
    the same normal equations (the item side: many ratings per row)."""
    from orange3_spark_amd.ops import als as A
    monkeypatch.setattr(AE, "DENSE_MIN_AVG", 64)
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.ratings(20000, 1500, 300000, rank=8, seed=4, implicit=implicit)
    users = df.column_data("user").data.long()
    items = df.column_data("item").data.long()
    r = df.column_data("rating").data.float()
    uid, iid = AE.global_ids(s.comm, users), AE.global_ids(s.comm, items)
    uix, iix = torch.searchsorted(uid, users), torch.searchsorted(iid, items)
    by_item = AE.partition(s.comm, iix, uix, r, iid.numel())
    X = AE.init_factors(0, uid.numel(), R, 5, users.device, False)
    Y0 = AE.init_factors(0, iid.numel(), R, 6, users.device, False)
    G = (X.double().T @ X.double()).float() if implicit else None
    assert A.gram_ok(X) and by_item.cols.numel() >= AE.DENSE_MIN_AVG * by_item.nrows
    dense = AE.solve_side(by_item, X, Y0, 0.1, implicit, 2.0, G, 3, False, exact=None)
    ref = AE.solve_side(by_item, X, Y0, 0.1, implicit, 2.0, G, 3, False, exact=True)
    err = ((dense.double() - ref.double()).norm() / ref.double().norm()).item()
    assert err < 2e-4, err


@pytest.mark.gpu
@pytest.mark.parametrize("rank,nonneg", [(128, False), (10, True), (200, False)])
def test_gpu_init_factors_kernel_matches_torch(rank, nonneg):
    """als_init_kernel draws the same unit-norm gaussian rows as the torch path."""
    from orange3_spark_amd.models import als as AE
    ref = AE.init_factors(1000, 3001, rank, 12345 ^ 0x5A5A, torch.device("cpu"), nonneg)
    got = AE.init_factors(1000, 3001, rank, 12345 ^ 0x5A5A, torch.device("cuda"), nonneg).cpu()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)


def _exact_case(R, implicit, seed=0, n_rows=700, n_other=900, dev="cuda"):
    """A CSR with rows of 0, 1, a few, exactly 32, 33 and ~200 ratings (both kernels,
    every routing edge), implicit zero-rating entries, random factors."""
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(0, 40, (n_rows,), generator=g)
    lens[:6] = torch.tensor([0, 1, 5, 32, 33, 200])
    lens[6:40] = torch.randint(60, 260, (34,), generator=g)
    lens[6] = 1000                                  # several index-chunk refills of the gather ring
    indptr = torch.zeros(n_rows + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    cols = torch.randint(0, n_other, (nnz,), generator=g, dtype=torch.int32)
    vals = torch.randn(nnz, generator=g) * 2
    if implicit:
        vals[::17] = 0.0
    F = torch.randn((n_other, R), generator=g) / R ** 0.5
    w, b, pos = AE._weights(vals, implicit, 2.0)
    rows = torch.repeat_interleave(torch.arange(n_rows), lens)
    nu = torch.zeros(n_rows).index_add_(0, rows, pos.float())
    lam = (0.05 * nu).float()
    G = (F.double().T @ F.double()).float() if implicit else None
    to = (lambda t: None if t is None else t.to(dev))
    return [to(x) for x in (indptr, cols, w, b, F, G, lam)]


@pytest.mark.gpu
@pytest.mark.parametrize("R", [32, 64, 128])
@pytest.mark.parametrize("implicit", [False, True])
def test_gpu_exact_kernels_match_fp64_solve(R, implicit):
    """als_wood_kernel (<= 32 ratings) and als_dense_wave_kernel (longer rows) == fp64
    torch.linalg.solve of each row's normal equations (rank up to 128)."""
    from orange3_spark_amd.ops import als as A
    indptr, cols, w, b, F, G, lam = _exact_case(R, implicit)
    n = indptr.numel() - 1
    got = torch.full((n, R), float("nan"), device=F.device)
    A.exact_solve(indptr, cols, w, b, F, G, lam, implicit, got)
    ref = torch.empty((n, R), dtype=torch.float64, device=F.device)
    A.exact_solve_torch(indptr, cols, w, b, F, G, lam, ref)
    assert not torch.isnan(got).any()
    err = (got.double() - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-6)
    assert float(err.max()) < 2e-3, float(err.max())
    # a row range (the chunked multi-rank path) writes only its rows
    part = torch.zeros((n, R), device=F.device)
    A.exact_solve(indptr, cols, w, b, F, G, lam, implicit, part, row_range=(100, 300))
    assert torch.equal(part[100:300], got[100:300]) and not part[:100].any() and not part[300:].any()


@pytest.mark.gpu
def test_gpu_exact_als_rank128_fit_matches_fp64():
    """ALS rank 128 (implicit), exact solves by default: the GPU fit after 2 iterations ==
    the fp64 torch exact path on the CPU from the same initial factors."""
    g = torch.Generator().manual_seed(3)
    n = 60_000
    users = torch.randint(0, 3000, (n,), generator=g)
    items = torch.randint(0, 800, (n,), generator=g)
    r = (torch.rand(n, generator=g) * 5).round()
    from orange3_spark_amd.parallel.comm import LocalComm
    gpu = AE.fit_als(LocalComm("cuda"), users.cuda(), items.cuda(), r.cuda(), rank=128, max_iter=2, reg=0.1,
                     implicit=True, alpha=1.0, seed=1)
    cpu = AE.fit_als(LocalComm("cpu"), users, items, r, rank=128, max_iter=2, reg=0.1, implicit=True, alpha=1.0,
                     seed=1)
    for a, b in ((gpu.U, cpu.U), (gpu.V, cpu.V)):
        err = (a.cpu().double() - b.double()).norm() / b.double().norm()
        assert float(err) < 5e-3, float(err)


@pytest.mark.gpu
def test_gpu_exact_implicit_fit_in_eigenbasis_matches_rotating_each_iteration(monkeypatch):
    """fit_als keeps both tables in the moving eigenbasis of the Gram (no x = Q y rotation
    of the user side per iteration; one rotation back at the end): 3 iterations over users
    with both Woodbury (<= 32 ratings) and dense rows == the fit that rotates every
    half-iteration, up to fp32 rounding of the rotations."""
    g = torch.Generator().manual_seed(5)
    n = 80_000
    users = torch.randint(0, 3000, (n,), generator=g)
    items = torch.randint(0, 700, (n,), generator=g)
    r = (torch.rand(n, generator=g) * 5).round()
    from orange3_spark_amd.parallel.comm import LocalComm
    fits = {}
    for mode in (True, False):
        monkeypatch.setattr(AE, "EIG_BASIS", mode)
        fits[mode] = AE.fit_als(LocalComm("cuda"), users.cuda(), items.cuda(), r.cuda(), rank=128, max_iter=3,
                                reg=0.1, implicit=True, alpha=1.0, seed=2)
    cnt = torch.bincount(users, minlength=3000)
    assert bool((cnt > 32).any()) and bool((cnt <= 32).any())
    for a, b in ((fits[True].U, fits[False].U), (fits[True].V, fits[False].V)):
        err = (a.double() - b.double()).norm() / b.double().norm()
        assert float(err) < 1e-4, float(err)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [10, 40])
@pytest.mark.parametrize("implicit", [False, True])
def test_gpu_exact_kernels_pad_other_ranks(R, implicit):
    """Ranks between the compiled kernel sizes (Spark's default rank 10, or 40) run on the
    kernels with zero-padded factor columns and match the fp64 solve; a row range writes
    only its rows."""
    from orange3_spark_amd.ops import als as A
    indptr, cols, w, b, F, G, lam = _exact_case(R, implicit, seed=3)
    n = indptr.numel() - 1
    got = torch.full((n, R), float("nan"), device=F.device)
    A.exact_solve(indptr, cols, w, b, F, G, lam, implicit, got)
    ref = torch.empty((n, R), dtype=torch.float64, device=F.device)
    A.exact_solve_torch(indptr, cols, w, b, F, G, lam, ref)
    assert not torch.isnan(got).any()
    err = (got.double() - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-6)
    assert float(err.max()) < 2e-3, float(err.max())
    part = torch.zeros((n, R), device=F.device)
    A.exact_solve(indptr, cols, w, b, F, G, lam, implicit, part, row_range=(100, 300))
    assert torch.allclose(part[100:300], got[100:300], rtol=1e-5, atol=1e-6)
    assert not part[:100].any() and not part[300:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("R", [32, 64, 96, 128])
@pytest.mark.parametrize("implicit", [False, True])
def test_gpu_dense_kernel_matches_fp64_solve(R, implicit):
    """The dense exact kernel (als_dense_wave_kernel: one wave per row, 32 x 32 MFMA
    accumulator tiles) == the fp64 solve on rows routed to the dense path (lam = 0 rows and
    rows longer than the Woodbury limit), including rows of 0 and 1 ratings, an odd count
    and a row that is not a multiple of the 16-rating staging round."""
    from orange3_spark_amd.ops import als as A
    indptr, cols, w, b, F, G, lam = _exact_case(R, implicit, seed=11)
    lam = lam.clone()
    lam[:40] = 0.05 * (indptr[1:41] - indptr[:40]).float().clamp_min(1.0)   # rows < 40: dense path too
    n = indptr.numel() - 1
    dense = torch.arange(0, 40, device=F.device, dtype=torch.int32)
    got = torch.full((n, R), float("nan"), device=F.device)
    Gf = G.float().contiguous() if implicit else None
    A.dense_wave(implicit, indptr, cols, w, b, F, Gf, lam, dense, got, grid=256)
    ref = torch.empty((n, R), dtype=torch.float64, device=F.device)
    A.exact_solve_torch(indptr, cols, w, b, F, G, lam, ref)
    got, ref = got[:40], ref[:40]
    assert not torch.isnan(got).any()
    err = (got.double() - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-6)
    assert float(err.max()) < 2e-3, float(err.max())


@pytest.mark.gpu
@pytest.mark.parametrize("R", [32, 64, 96, 128])
@pytest.mark.parametrize("implicit", [False, True])
@pytest.mark.parametrize("grid", [1, 3, 256])
def test_gpu_dense_wave_streams_many_rows_per_wave(R, implicit, grid):
    """als_dense_wave_kernel with several rows per wave (grid 1 and 3 blocks: 4 / 12 waves
    walk 600 rows each way; 256: one or two): the LDS-DMA ring streams ACROSS rows (the
    next row's steps land while this row factors), rows of 0, 1, 15, 16, 17, 33 and up to
    ~2000 ratings, every row == the fp64 solve, bitwise the same for every grid."""
    from orange3_spark_amd.ops import _native as N
    from orange3_spark_amd.ops import als as A
    g = torch.Generator().manual_seed(R + 7 * implicit)
    n_rows, n_other = 600, 5000
    lens = torch.randint(33, 120, (n_rows,), generator=g)
    lens[:8] = torch.tensor([0, 1, 15, 16, 17, 33, 2000, 517])
    indptr = torch.zeros(n_rows + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    cols = torch.randint(0, n_other, (nnz,), generator=g, dtype=torch.int32)
    vals = torch.randn(nnz, generator=g) * 2
    if implicit:
        vals[::13] = 0.0
    F = torch.randn((n_other, R), generator=g) / R ** 0.5
    w, b, pos = AE._weights(vals, implicit, 2.0)
    rows = torch.repeat_interleave(torch.arange(n_rows), lens)
    nu = torch.zeros(n_rows).index_add_(0, rows, pos.float())
    lam = (0.05 * nu.clamp_min(1.0)).float()
    G = (F.double().T @ F.double()).float() if implicit else None
    dev = "cuda"
    indptr, cols, w, b, F, lam = (x.to(dev) for x in (indptr, cols, w, b, F, lam))
    Gf = G.to(dev).contiguous() if implicit else None
    order = torch.argsort(lens, descending=True).to(torch.int32).to(dev)
    got = torch.full((n_rows, R), float("nan"), device=dev)
    A.dense_wave(implicit, indptr, cols, w, b, F, Gf, lam, order, got, grid=grid)
    ref = torch.empty((n_rows, R), dtype=torch.float64, device=dev)
    A.exact_solve_torch(indptr, cols, w, b, F, None if G is None else G.to(dev), lam, ref)
    assert not torch.isnan(got).any()
    err = (got.double() - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-6)
    assert float(err.max()) < 2e-3, float(err.max())
    again = torch.full_like(got, float("nan"))
    A.dense_wave(implicit, indptr, cols, w, b, F, Gf, lam, order, again, grid=2)
    assert torch.equal(got, again)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [32, 64, 96, 128])
@pytest.mark.parametrize("grid", [1, 256])
def test_gpu_dense_wave_diagonal_g_matches_fp64(R, grid):
    """The eigenbasis dense solve with G = diag(g) passed as a vector (o3s_als_dense_wave_gd:
    no G image in LDS, the deeper gather ring) == the fp64 solve of the same systems, and
    == the full-G build fed diag(g) up to fp32 rounding; rows of 1..2000 ratings."""
    from orange3_spark_amd.ops import als as A
    g = torch.Generator().manual_seed(R + grid + 1)
    n_rows, n_other = 700, 4000
    lens = torch.randint(33, 260, (n_rows,), generator=g)
    lens[:5] = torch.tensor([1, 16, 17, 2000, 33])
    indptr = torch.zeros(n_rows + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    cols = torch.randint(0, n_other, (nnz,), generator=g, dtype=torch.int32)
    vals = torch.rand(nnz, generator=g) * 4
    vals[::11] = 0.0
    F = torch.randn((n_other, R), generator=g) / R ** 0.5
    gdiag = torch.rand(R, generator=g) * n_other / R
    w, b, pos = AE._weights(vals, True, 1.5)
    rows = torch.repeat_interleave(torch.arange(n_rows), lens)
    lam = (0.05 * torch.zeros(n_rows).index_add_(0, rows, pos.float()).clamp_min(1.0)).float()
    dev = "cuda"
    indptr, cols, w, b, F, lam, gdiag = (x.to(dev) for x in (indptr, cols, w, b, F, lam, gdiag))
    order = torch.argsort(lens, descending=True).to(torch.int32).to(dev)
    got = torch.full((n_rows, R), float("nan"), device=dev)
    A.dense_wave(True, indptr, cols, w, b, F, None, lam, order, got, grid=grid, gdiag=gdiag.contiguous())
    ref = torch.empty((n_rows, R), dtype=torch.float64, device=dev)
    A.exact_solve_torch(indptr, cols, w, b, F, torch.diag(gdiag), lam, ref)
    assert not torch.isnan(got).any()
    err = (got.double() - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-6)
    assert float(err.max()) < 2e-3, float(err.max())
    full = torch.full_like(got, float("nan"))
    A.dense_wave(True, indptr, cols, w, b, F, torch.diag(gdiag).contiguous(), lam, order, full, grid=grid)
    assert float(((full - got).norm(dim=1) / full.norm(dim=1).clamp_min(1e-6)).max()) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("R", [32, 128])
@pytest.mark.parametrize("grid", [1, 256])
def test_gpu_dense_wave_short_rows_metadata_ring(R, grid):
    """Rows of 1..20 ratings (one or two 16-rating steps each, the fastest the index cursor
    can move through rows) through the dense kernel: its row metadata ring (DMA'd MAHEAD =
    DEPTH rows ahead of the cursor, MR = 3 DEPTH + 1 slots) must hold every row until the
    consumer has read it -- every row == the fp64 solve; rows without ratings give 0."""
    from orange3_spark_amd.ops import als as A
    g = torch.Generator().manual_seed(R + grid)
    n_rows, n_other = 1500, 3000
    lens = torch.randint(1, 21, (n_rows,), generator=g)
    lens[::97] = 0
    indptr = torch.zeros(n_rows + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    cols = torch.randint(0, n_other, (nnz,), generator=g, dtype=torch.int32)
    vals = torch.rand(nnz, generator=g) * 3
    F = torch.randn((n_other, R), generator=g) / R ** 0.5
    w, b, pos = AE._weights(vals, True, 1.5)
    lam = torch.full((n_rows,), 0.3)
    G = (F.double().T @ F.double()).float()
    dev = "cuda"
    indptr, cols, w, b, F, lam, G = (x.to(dev) for x in (indptr, cols, w, b, F, lam, G))
    order = torch.randperm(n_rows, generator=g).to(torch.int32).to(dev)
    got = torch.full((n_rows, R), float("nan"), device=dev)
    A.dense_wave(True, indptr, cols, w, b, F, G.contiguous(), lam, order, got, grid=grid)
    ref = torch.empty((n_rows, R), dtype=torch.float64, device=dev)
    A.exact_solve_torch(indptr, cols, w, b, F, G, lam, ref)
    assert not torch.isnan(got).any()
    assert not got[lens.to(dev) == 0].any()
    err = (got.double() - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-6)
    assert float(err.max()) < 2e-3, float(err.max())


def test_blockwise_topk_recommendations_match_brute_force():
    """recommendForAll*: blockwise top-k (bounded score blocks, running merge) equals the
    full score matrix's top-k; the column stays on the device until read."""
    from orange3_spark_amd.ml.recommendation import RecsColumn, topk_scores
    g = torch.Generator().manual_seed(0)
    Q, T = torch.randn(300, 8, generator=g), torch.randn(1000, 8, generator=g)
    v, i = topk_scores(Q, T, 7, budget=300)              # tiny budget: many query / target blocks
    rv, ri = torch.topk(Q @ T.T, 7, dim=1)
    assert torch.allclose(v, rv) and torch.equal(i, ri)
    s = Session(SessionConf().set("o3s.device", "cpu"))
    rng = np.random.default_rng(2)
    pdf = pd.DataFrame({"user": rng.integers(0, 50, 2000), "item": rng.integers(0, 80, 2000),
                        "rating": rng.integers(1, 6, 2000).astype(float)})
    m = ALS(rank=4, maxIter=3, seed=1).fit(s.createDataFrame(pdf))
    recs = m.recommendForAllUsers(5)
    col = recs.column_data("recommendations")
    assert isinstance(col, RecsColumn) and col.ids.shape == (50, 5)
    first = recs.orderBy("user").collect()[0]
    U_, V_ = m._U.double(), m._V.double()
    u0 = int(torch.searchsorted(m._uid_t, torch.tensor(first.user)))
    want = torch.topk(U_[u0] @ V_.T, 5).indices
    assert [r.item for r in first.recommendations] == m._iid_t[want].tolist()
    assert recs.filter(recs.user < 10).count() == 10


@pytest.mark.gpu
@pytest.mark.parametrize("R", [10, 32, 64, 96, 128])
@pytest.mark.parametrize("n", [1, 3, 1001, 300_007])
def test_gpu_ftf_kernel_matches_fp64(R, n):
    """ftf_kernel (the implicit-ALS Gram F^T F on the matrix cores, wave partials summed in
    fp64 in a fixed order) == the fp64 product, for ranks that pad to 32-column blocks, odd
    row counts, a row stride wider than R, and bitwise repeatable."""
    from orange3_spark_amd.ops import als as A
    g = torch.Generator(device="cuda").manual_seed(R + n)
    base = torch.randn((n, R + 3), generator=g, device="cuda")
    F = base[:, :R]                                   # stride(0) = R + 3
    got = A.ftf(F)
    ref = F.double().T @ F.double()
    err = (got - ref).abs().max() / ref.abs().max()
    assert float(err) < 1e-6, float(err)
    assert torch.equal(got, got.T)
    assert torch.equal(A.ftf(F), got)
    assert torch.allclose(AE.gram(F.contiguous()), ref, rtol=1e-6, atol=1e-6 * float(ref.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("R", [32, 64, 96, 128])
@pytest.mark.parametrize("n", [1, 33, 100_003])
def test_gpu_rotated_table_matches_fp64(R, n):
    """F Q for the Woodbury gathers comes from the in-place rotation kernel (Q passed where
    the x = Q y path passes Q^T): equal to the fp64 product, F itself untouched."""
    from orange3_spark_amd.ops import als as A
    g = torch.Generator(device="cuda").manual_seed(R * 7 + n)
    F = torch.randn((n, R), generator=g, device="cuda")
    Q = torch.linalg.qr(torch.randn((R, R), generator=g, device="cuda", dtype=torch.float64))[0].float()
    F0 = F.clone()
    got = A.rotated_table(F, Q)
    ref = F.double() @ Q.double()
    assert torch.equal(F, F0)
    assert float((got.double() - ref).abs().max()) < 2e-5 * float(ref.abs().max())


def test_row_counts_equal_scatter_count():
    """Per-row positive-rating counts from the prefix sum == the repeat_interleave +
    index_add form, empty rows (leading, inner, trailing) included."""
    g = torch.Generator().manual_seed(3)
    lens = torch.randint(0, 6, (1000,), generator=g)
    lens[0] = lens[500] = lens[-1] = 0
    indptr = torch.zeros(1001, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    pos = torch.rand(int(indptr[-1]), generator=g) > 0.3
    rows = torch.repeat_interleave(torch.arange(1000), lens)
    ref = torch.zeros(1000).index_add_(0, rows, pos.float())
    assert torch.equal(AE._row_counts(indptr, pos), ref)
    assert torch.equal(AE._row_counts(torch.zeros(4, dtype=torch.int64), pos[:0]), torch.zeros(3))


@pytest.mark.parametrize("dt", [torch.int32, torch.int64])
def test_id_maps_int32_and_int64(dt):
    """Distinct ids and dense positions are the same for int32 and int64 id columns, on the
    bitmap / lookup-table path (dense span, including the int32 minimum) and the sorted one."""
    class _C:
        world_size = 1
    lo = -(1 << 31) if dt == torch.int32 else -(1 << 40)
    for ids in (torch.tensor([3, 1, 2, 9, 1, 3, 5]), torch.tensor([5, -3, 7, 5, -3, 100]),
                torch.tensor([lo + 5, lo, lo + 3, lo])):
        ids = ids.to(dt)
        uid = AE.global_ids(_C(), ids)
        assert uid.tolist() == sorted(set(ids.tolist()))
        pos = AE.dense_index(uid, ids)
        assert uid[pos.long()].tolist() == ids.tolist()


def test_dense_meta_layout_cpu():
    """ops/als.py dense_meta: the dense kernel's per-row metadata, int32 [n][8] in list
    order = {p0 lo, p0 hi, n, u, lam_u bits, 0, 0, 0} (csrc/als_dense.hip DMAs it into an
    LDS ring ahead of use), including a 64-bit p0 beyond 2^32."""
    from orange3_spark_amd.ops import als as A
    indptr = torch.tensor([0, 5, 5, 12, (1 << 33) + 7, (1 << 33) + 40], dtype=torch.int64)
    lam = torch.tensor([0.5, 0.0, 2.25, 1e-3, 7.0])
    rows = torch.tensor([4, 0, 2], dtype=torch.int32)
    m = A.dense_meta(indptr, rows, lam)
    assert m.dtype == torch.int32 and m.shape == (3, 8)
    p0 = (m[:, 1].long() << 32) | (m[:, 0].long() & 0xFFFFFFFF)
    assert p0.tolist() == [(1 << 33) + 7, 0, 5]
    assert m[:, 2].tolist() == [33, 5, 7]
    assert m[:, 3].tolist() == [4, 0, 2]
    assert m[:, 4].view(torch.float32).tolist() == [7.0, 0.5, 2.25]
    assert not m[:, 5:].any()
