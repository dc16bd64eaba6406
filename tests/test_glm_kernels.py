"""Numerics of the fused GLM kernels (csrc/glm.hip) vs plain PyTorch fp64 references."""
import pytest
import torch

from orange3_spark_amd.ops import glm as G


def test_layout_matches_native_rule():
    assert G.layout(256) == (256, 260)
    assert G.layout(24) == (32, 36)
    assert G.layout(1024) == (1024, 1028)
    with pytest.raises(ValueError):
        G.layout(8 * 64 * 32)


def test_synth_cpu_deterministic_and_partition_invariant():
    X, y = G.synth_glm(1000, 32, seed=7)
    X2, y2 = G.synth_glm(500, 32, seed=7, row0=500)
    assert torch.equal(X[500:], X2) and torch.equal(y[500:], y2)
    assert X.dtype == torch.bfloat16 and X.shape == (1000, 32)
    assert 0.2 < y.mean().item() < 0.8
    assert X.float().abs().max() <= 1.0


def test_cpu_grad_matches_closed_form():
    X, y = G.synth_glm(300, 16, seed=3)
    coef = torch.randn(16) * 0.1
    for loss in (0, 1, 2):
        out = G.glm_grad(X, y, None, coef, 0.3, loss)
        ref = G.glm_grad_torch(X, y, None, coef.double(), 0.3, loss)
        dpad, _ = G.layout(16)
        assert torch.allclose(out[:16], ref[:16])
        assert torch.allclose(out[dpad:], ref[16:])


@pytest.mark.gpu
@pytest.mark.parametrize("d", [8, 20, 64, 256, 520, 1024])
def test_gpu_synth_matches_torch(gpu, d):
    n = 4099
    Xg, yg = G.synth_glm(n, d, seed=11, row0=12345, device=gpu)
    Xc, yc = G.synth_glm(n, d, seed=11, row0=12345)
    assert torch.equal(Xg.cpu(), Xc)
    assert (yg.cpu() != yc).float().mean().item() < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("d", [8, 24, 256, 520, 1024])
@pytest.mark.parametrize("loss", [0, 1, 2])
def test_gpu_grad_matches_fp64(gpu, d, loss):
    n = 30001
    X, y = G.synth_glm(n, d, seed=5, device=gpu)
    ld = X.shape[1]
    coef = (torch.randn(ld, generator=torch.Generator().manual_seed(1)) * 0.05)
    sw = torch.rand(n, generator=torch.Generator().manual_seed(2)).to(gpu) if loss == 0 else None
    out = G.glm_grad(X, y, sw, coef.to(gpu), -0.2, loss).cpu()
    ref = G.glm_grad_torch(X.cpu(), y.cpu(), None if sw is None else sw.cpu(), coef.double(), -0.2, loss)
    dpad, _ = G.layout(ld)
    scale = ref[:ld].abs().max().item() + 1.0
    assert (out[:ld] - ref[:ld]).abs().max().item() < 2e-4 * scale * (n ** 0.5) / 50
    assert abs(out[dpad] - ref[ld]) < 1e-3 * (abs(ref[ld].item()) + 10)
    assert abs(out[dpad + 1] - ref[ld + 1]) < 1e-4 * abs(ref[ld + 1].item()) + 1e-2
    assert abs(out[dpad + 2] - ref[ld + 2]) < 1e-3


@pytest.mark.gpu
def test_gpu_grad_synth_lineage_equals_materialised(gpu):
    n, d, seed = 50000, 256, 9
    wt, bt = G.synth_truth(seed, d)
    X, y = G.synth_glm(n, d, seed, row0=777, device=gpu, wtrue=wt, btrue=bt)
    coef = torch.randn(d, generator=torch.Generator().manual_seed(4)).to(gpu) * 0.02
    ws = G.GlmWorkspace(gpu, d)
    a = G.glm_grad(X, y, None, coef, 0.1, 0, ws).clone()
    b = G.glm_grad_synth(n, d, d, seed, 777, wt, bt, coef, 0.1, 0, ws).clone()
    # identical rows; labels may flip on ~1e-6 of rows due to sum order -> tiny tolerance
    assert torch.allclose(a, b, rtol=1e-4, atol=1e-2)


@pytest.mark.gpu
def test_gpu_margin(gpu):
    X, _ = G.synth_glm(10007, 256, seed=1, device=gpu)
    coef = torch.randn(256).to(gpu)
    m = G.glm_margin(X, coef, 0.5)
    ref = X.double() @ coef.double() + 0.5
    assert torch.allclose(m.double(), ref, atol=1e-3, rtol=1e-4)


@pytest.mark.gpu
def test_gpu_grad_deterministic(gpu):
    X, y = G.synth_glm(100000, 256, seed=2, device=gpu)
    coef = torch.full((256,), 0.01, device=gpu)
    a = G.glm_grad(X, y, None, coef, 0.0, 0).clone()
    b = G.glm_grad(X, y, None, coef, 0.0, 0).clone()
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("d,loss", [(256, 0), (256, 1), (256, 2), (20, 0), (100, 0), (600, 0)])
def test_gpu_grad_mixed_matches_fp64(gpu, d, loss):
    """One-launch resident + lineage pass == fp64 torch over the materialised rows."""
    n_res, n_lin, seed = 30011, 20007, 13
    ld = G.padded_width(d)
    wt, bt = G.synth_truth(seed, d, ld)
    # resident rows: arbitrary data (rows 0..n_res); lineage: global rows n_res..
    Xr, yr = G.synth_glm(n_res, d, seed + 1, device=gpu, ld=ld)
    Xl, yl = G.synth_glm(n_lin, d, seed, row0=n_res, device=gpu, ld=ld, wtrue=wt, btrue=bt)
    coef = torch.randn(ld, generator=torch.Generator().manual_seed(4)).to(gpu) * 0.05
    ws = G.GlmWorkspace(gpu, ld, grid=96)
    yall = torch.cat([yr, 1.0 - yl])           # lineage labels come from the label column
    out = G.glm_grad_mixed(Xr, yall, None, n_lin, d, seed, n_res, coef, 0.1, loss, ws).clone()
    ref = G.glm_grad_torch(torch.cat([Xr, Xl]), yall, None, coef.double(), 0.1, loss)
    dpad = ws.dpad
    assert torch.allclose(out[:ld], ref[:ld], rtol=1e-3, atol=0.05), (out[:ld] - ref[:ld]).abs().max()
    assert torch.allclose(out[dpad:], ref[ld:], rtol=1e-3, atol=0.5)
    again = G.glm_grad_mixed(Xr, yall, None, n_lin, d, seed, n_res, coef, 0.1, loss, ws).clone()
    assert torch.equal(out, again)                      # deterministic slab reduction


def test_cpu_grad_mixed_matches_split():
    d, seed = 24, 3
    ld = G.padded_width(d)
    wt, bt = G.synth_truth(seed, d, ld)
    Xr, yr = G.synth_glm(500, d, seed + 1, ld=ld)
    Xl, yl = G.synth_glm(300, d, seed, row0=500, ld=ld, wtrue=wt, btrue=bt)
    coef = torch.linspace(-0.1, 0.1, ld)
    ws = G.GlmWorkspace("cpu", ld)
    out = G.glm_grad_mixed(Xr, torch.cat([yr, yl]), None, 300, d, seed, 500, coef, 0.2, 0, ws)
    ref = G.glm_grad(torch.cat([Xr, Xl]), torch.cat([yr, yl]), None, coef, 0.2, 0)
    assert torch.allclose(out, ref, rtol=1e-10, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [2, 3])
def test_gpu_grad_mixed_register_budgets_agree(gpu, waves, monkeypatch):
    """The mixed kernel compiled for 2 and for 3 waves per SIMD computes the same pass as
    the split resident + lineage passes (up to fp32 block-sum order)."""
    n_res, n_lin, d, seed = 40009, 30011, 256, 21
    Xr, yr = G.synth_glm(n_res, d, seed + 1, device=gpu)
    yall = torch.cat([yr, (torch.arange(n_lin, device=gpu) % 3 == 0).float()])
    coef = torch.randn(d, generator=torch.Generator().manual_seed(2)).to(gpu) * 0.05
    ws = G.GlmWorkspace(gpu, d, grid=512)
    monkeypatch.setattr(G, "MIX_WAVES", waves)
    out = G.glm_grad_mixed(Xr, yall, None, n_lin, d, seed, n_res, coef, -0.2, 0, ws).clone()
    wt, bt = G.synth_truth(seed, d, d)
    Xl, _ = G.synth_glm(n_lin, d, seed, row0=n_res, ld=d, wtrue=wt, btrue=bt, device=gpu)
    ref = G.glm_grad(torch.cat([Xr, Xl]).cpu(), yall.cpu(), None, coef.cpu(), -0.2, 0)    # fp64 torch
    assert torch.allclose(out.cpu(), ref, rtol=1e-4, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("slice_rows", [7000, 30000])
@pytest.mark.parametrize("frac", [1.0, 0.3])
def test_gpu_grad_mixed_split_launches_agree(gpu, slice_rows, frac, monkeypatch):
    """A mixed pass run as several launches over row slices (o3s_glm_grad_mixed splits,
    later slices adding into the first slice's slabs) == one launch up to fp32 block-sum
    order, with and without mini-batch sampling (global row keys shifted per slice); the
    split pass is deterministic."""
    n_res, n_lin, d, seed = 40009, 30011, 256, 21
    Xr, yr = G.synth_glm(n_res, d, seed + 1, device=gpu)
    yall = torch.cat([yr, (torch.arange(n_lin, device=gpu) % 3 == 0).float()])
    coef = torch.randn(d, generator=torch.Generator().manual_seed(2)).to(gpu) * 0.05
    ws = G.GlmWorkspace(gpu, d, grid=512)
    kw = dict(res_row0=123, sample_seed=9, fraction=frac)
    monkeypatch.setattr(G, "MIX_SLICE_ROWS", 1 << 40)
    ref = G.glm_grad_mixed(Xr, yall, None, n_lin, d, seed, n_res, coef, -0.2, 0, ws, **kw).clone()
    monkeypatch.setattr(G, "MIX_SLICE_ROWS", slice_rows)
    assert G.mix_splits(n_res + n_lin) > 1
    out = G.glm_grad_mixed(Xr, yall, None, n_lin, d, seed, n_res, coef, -0.2, 0, ws, **kw).clone()
    again = G.glm_grad_mixed(Xr, yall, None, n_lin, d, seed, n_res, coef, -0.2, 0, ws, **kw).clone()
    assert torch.equal(out, again)
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("d,K,weighted,pad", [(256, 10, False, 0), (20, 3, True, 12), (100, 32, True, 4),
                                             (64, 2, False, 0), (200, 7, False, 56)])
def test_gpu_softmax_pass_matches_fp64(gpu, d, K, weighted, pad):
    """glm_softmax_kernel (MFMA margins + gradient, split-bf16 W and R) vs the fp64 torch
    pass on the same bf16 rows; padded row strides (vector columns) and ragged tiles."""
    g = torch.Generator().manual_seed(d + K)
    n = 40_003
    Xf = torch.rand((n, d + pad), generator=g) * 2 - 1
    Xf[:, d:] = 0
    Xb = Xf.to(torch.bfloat16).to(gpu)
    X = Xb[:, :d]
    y = torch.randint(0, K, (n,), generator=g).to(gpu)
    sw = (torch.rand(n, generator=g) + 0.5).to(gpu) if weighted else None
    W = (torch.randn((K, d), generator=g) * 0.3).to(gpu)
    b = (torch.randn(K, generator=g) * 0.5).to(gpu)
    assert G.softmax_kernel_ok(X, K)
    Gk, gb, loss = G.softmax_pass(X, y, sw, W, b)
    Gr, gbr, lr = G.softmax_pass_torch(X, y, sw, W, b)
    scale = Gr.abs().max().item()
    assert (Gk - Gr).abs().max().item() <= 2e-5 * scale
    assert torch.allclose(gb, gbr, rtol=1e-5, atol=1e-6 * n)
    assert abs(loss.item() - lr.item()) <= 1e-5 * abs(lr.item())


@pytest.mark.gpu
def test_gpu_multinomial_fit_kernel_matches_chunked(gpu, monkeypatch):
    from orange3_spark_amd.models import glm as GLM
    from orange3_spark_amd.parallel.comm import LocalComm
    g = torch.Generator().manual_seed(5)
    n, d, K = 50_000, 24, 4
    X = (torch.rand((n, d), generator=g) * 2 - 1).to(torch.bfloat16).to(gpu)
    z = X[:, 0].float() + 0.5 * X[:, 1].float()
    y = ((z + 1.5) / 3 * K).floor().clamp(0, K - 1).double()
    comm = LocalComm(gpu)
    B1, b1, r1 = GLM.fit_multinomial(comm, X, y, None, K, reg=0.01, max_iter=50)
    monkeypatch.setenv("O3S_SOFTMAX_KERNEL", "0")
    B0, b0, r0 = GLM.fit_multinomial(comm, X, y, None, K, reg=0.01, max_iter=50)
    assert abs(r1.f - r0.f) <= 1e-6 * abs(r0.f)
    assert abs(B1 - B0).max() < 1e-3 and abs(b1 - b0).max() < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("d,weighted", [(256, False), (256, True), (20, False), (100, True), (600, False),
                                        (2048, False)])
def test_gpu_stats_mixed_matches_fp64(gpu, d, weighted):
    """Fused summarizer + first-gradient pass (glm_stats_mixed_kernel) vs fp64 torch over
    the materialised resident + lineage rows."""
    n_res, n_lin, seed = 30011, 20007, 17
    ld = G.padded_width(d)
    wt, bt = G.synth_truth(seed, d, ld)
    Xr, yr = G.synth_glm(n_res, d, seed + 1, device=gpu, ld=ld)
    Xl, yl = G.synth_glm(n_lin, d, seed, row0=n_res, device=gpu, ld=ld, wtrue=wt, btrue=bt)
    yall = torch.cat([yr, yl])
    sw = (torch.rand(n_res + n_lin, generator=torch.Generator().manual_seed(3)) + 0.5).to(gpu) if weighted else None
    out = G.glm_stats_mixed(Xr, yall, sw, n_lin, d, seed, n_res)
    assert out is not None
    out = out.cpu()
    ref = G.glm_stats_torch(torch.cat([Xr, Xl]).cpu(), yall.cpu(), None if sw is None else sw.cpu())
    dpad, _ = G.layout(ld)
    for k in range(3):
        a, b = out[k * dpad:k * dpad + ld], ref[k * dpad:k * dpad + ld]
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-5 * (1 + b.abs().max().item())), (k, (a - b).abs().max())
    assert torch.allclose(out[3 * dpad:], ref[3 * dpad:], rtol=1e-6)
    again = G.glm_stats_mixed(Xr, yall, sw, n_lin, d, seed, n_res).cpu()
    assert torch.equal(out, again)


@pytest.mark.gpu
@pytest.mark.parametrize("frac", [0.3, 0.05])
def test_gpu_grad_mixed_minibatch_matches_cpu_mask(gpu, frac):
    """In-kernel Bernoulli row mask == the torch twin's mask (same rows kept): the sampled
    pass equals the fp64 pass with the mask as row weights, for resident and lineage rows,
    and the iteration key comes from the device step counter."""
    n_res, n_lin, d, seed = 40009, 20011, 256, 23
    Xr, yr = G.synth_glm(n_res, d, seed + 1, device=gpu)
    Xl, yl = G.synth_glm(n_lin, d, seed, row0=5_000_000 + n_res, device=gpu)
    yall = torch.cat([yr, yl])
    coef = torch.randn(d, generator=torch.Generator().manual_seed(2)).to(gpu) * 0.05
    ws = G.GlmWorkspace(gpu, d, grid=512)
    t_dev = torch.tensor([4], dtype=torch.int64, device=gpu)          # iteration 5
    out = G.glm_grad_mixed(Xr, yall, None, n_lin, d, seed, 5_000_000 + n_res, coef, 0.1, 0, ws,
                           res_row0=5_000_000, t_dev=t_dev, sample_seed=99, fraction=frac).clone().cpu()
    grows = torch.arange(5_000_000, 5_000_000 + n_res + n_lin)
    keep = G.sample_mask(99, 5, grows, frac).double()
    ref = G.glm_grad_torch(torch.cat([Xr, Xl]).cpu(), yall.cpu(), keep, coef.double().cpu(), 0.1, 0)
    assert abs(out[d + 2].item() - keep.sum().item()) < 0.5           # identical kept set
    assert torch.allclose(out[:d], ref[:d], rtol=1e-3, atol=0.05)
    assert torch.allclose(out[d:], ref[d:], rtol=1e-3, atol=0.5)


@pytest.mark.gpu
def test_gpu_sgd_fit_matches_cpu(gpu):
    """LogisticRegression(solver='sgd').fit on the GPU (fused stats pass, graph-replayed
    steps, mini-batches) == the CPU fp64 path on the same bf16 rows."""
    import numpy as np
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.frame import column as Cc
    from orange3_spark_amd.frame.dataframe import DataFrame
    from orange3_spark_amd.ml.classification import LogisticRegression
    from collections import OrderedDict
    X, y = G.synth_glm(60_000, 64, seed=31, device=gpu)
    sg = Session(SessionConf().setAppName("g"), device=gpu)
    sc = Session(SessionConf().set("o3s.device", "cpu"))
    dg = DataFrame(sg, OrderedDict(features=Cc.VectorColumn(X, 64), label=Cc.NumericColumn(y)), X.shape[0])
    dc = DataFrame(sc, OrderedDict(features=Cc.VectorColumn(X.cpu().double(), 64),
                                   label=Cc.NumericColumn(y.cpu().double())), X.shape[0])
    for frac in (1.0, 0.2):
        kw = dict(solver="sgd", maxIter=12, tol=0.0, miniBatchFraction=frac, seed=5, regParam=0.01)
        a = LogisticRegression(**kw).fit(dg)
        b = LogisticRegression(**kw).fit(dc)
        assert np.allclose(a.coefficients.toArray(), b.coefficients.toArray(), rtol=2e-3, atol=2e-4)
        assert abs(a.intercept - b.intercept) < 2e-4
        assert a.summary.totalIterations == 12
