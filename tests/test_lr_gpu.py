"""LogisticRegression on the GPU kernel path vs the CPU fp64 path (same synthetic data)."""
import numpy as np
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.classification import LinearSVC, LogisticRegression
from orange3_spark_amd.ml.evaluation import BinaryClassificationEvaluator
from orange3_spark_amd.ops import _native


@pytest.mark.gpu
def test_native_loaded_on_gpu():
    lib = _native.kernels()
    assert lib is not None


@pytest.mark.gpu
def test_lr_gpu_matches_cpu():
    g = Session(SessionConf().set("o3s.device", "cuda"))
    c = Session(SessionConf().set("o3s.device", "cpu"))
    dg = g.synthetic.classification(50_000, 64, seed=3)
    dc = c.synthetic.classification(50_000, 64, seed=3)
    # identical bf16 data (CPU copy upcast to f64 exactly)
    mg = LogisticRegression(maxIter=50, regParam=0.01).fit(dg)
    mc = LogisticRegression(maxIter=50, regParam=0.01).fit(dc)
    assert np.allclose(mg.coefficients.toArray(), mc.coefficients.toArray(), atol=2e-3, rtol=1e-2)
    auc_g = BinaryClassificationEvaluator().evaluate(mg.transform(dg))
    auc_c = BinaryClassificationEvaluator().evaluate(mc.transform(dc))
    assert abs(auc_g - auc_c) < 1e-3


@pytest.mark.gpu
def test_lr_lineage_rows_equal_resident():
    s = Session(SessionConf().set("o3s.device", "cuda"))
    full = s.synthetic.classification(200_000, 256, seed=5)
    part = s.synthetic.classification(200_000, 256, seed=5, resident_fraction=0.0)
    assert part.column_data("features").lineage_rows == 200_000
    a = LogisticRegression(maxIter=10).fit(full)
    b = LogisticRegression(maxIter=10).fit(part)
    assert np.allclose(a.coefficients.toArray(), b.coefficients.toArray(), atol=1e-3)


@pytest.mark.gpu
def test_device_sgd_trainer():
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.classification(100_000, 256, seed=1)
    t = LogisticRegression(solver="sgd").trainer(df)
    for _ in range(20):
        t.step()
    h = t.result().history
    assert h[-1] < h[0]


@pytest.mark.gpu
def test_linear_svc_gpu():
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.classification(50_000, 32, seed=2)
    m = LinearSVC(maxIter=50, regParam=0.001).fit(df)
    out = m.transform(df)
    acc = (out.toPandas()["prediction"].values == out.toPandas()["label"].values).mean()
    assert acc > 0.75


@pytest.mark.gpu
@pytest.mark.parametrize("resident_fraction", [None, 0.0])
def test_sgd_graph_replay_equals_eager(monkeypatch, resident_fraction):
    """HIP-graph replayed SGD steps reproduce the eager launches bit for bit."""
    import time
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.classification(120_000, 256, seed=4, resident_fraction=resident_fraction)

    def run(mode, steps=12):
        monkeypatch.setenv("O3S_SGD_GRAPH", mode)
        t = LogisticRegression(solver="sgd", stepSize=0.5).trainer(df)
        for _ in range(steps):
            t.step()
        torch.cuda.synchronize()
        return t, t.result()
    te, eager = run("0")
    tg, graph = run("1")
    assert te._graphs is None and tg._graphs is not None
    assert eager.history == graph.history and len(graph.history) == 12
    assert np.array_equal(eager.coef, graph.coef) and eager.intercept == graph.intercept
    # the replay is cheaper per step than the eager launch sequence on a small problem
    small = s.synthetic.classification(4096, 16, seed=1)
    for mode in ("0", "1"):
        monkeypatch.setenv("O3S_SGD_GRAPH", mode)
        t = LogisticRegression(solver="sgd").trainer(small)
        for _ in range(5):
            t.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            t.step()
        torch.cuda.synchronize()
        if mode == "0":
            eager_s = time.perf_counter() - t0
        else:
            graph_s = time.perf_counter() - t0
    print(f"200 small SGD steps: eager {eager_s * 1e3:.2f} ms, graph {graph_s * 1e3:.2f} ms")
    assert graph_s < eager_s * 1.2


@pytest.mark.gpu
@pytest.mark.parametrize("loss", [0, 1, 2])
def test_gpu_sparse_glm_kernels_match_fp64(loss):
    """csr_glm_kernel (margin + loss + residual) and the CSC piece/combine gradient vs an
    fp64 torch reference, with a frequent-term column spanning many pieces."""
    from orange3_spark_amd.ops.glm import _loss_terms
    from orange3_spark_amd.ops.sparse import SparseRows
    g = torch.Generator().manual_seed(loss)
    n, d = 50_001, 5000
    nnz_row = torch.randint(0, 40, (n,), generator=g)
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(nnz_row, 0)
    nnz = int(indptr[-1])
    idx = torch.randint(0, d, (nnz,), generator=g, dtype=torch.int32)
    idx[::3] = 7                                   # one very frequent column (many 256-entry pieces)
    val = torch.randn(nnz, generator=g)
    y = (torch.rand(n, generator=g) < 0.5).float()
    w = torch.rand(n, generator=g) + 0.5
    coef = torch.randn(d, generator=g, dtype=torch.float64) * 0.1
    rows = SparseRows(indptr.cuda(), idx.cuda(), val.cuda(), d)
    got = rows.loss_grad(coef, 0.25, loss, y.cuda(), w.cuda()).cpu()
    row = torch.repeat_interleave(torch.arange(n), nnz_row)
    m = torch.zeros(n, dtype=torch.float64).index_add_(0, row, val.double() * coef[idx.long()]) + 0.25
    r, l = _loss_terms(m, y.double(), w.double(), loss)
    gref = torch.zeros(d, dtype=torch.float64).index_add_(0, idx.long(), val.double() * r[row])
    ref = torch.cat([gref, torch.stack([r.sum(), l.sum(), w.double().sum()])])
    torch.testing.assert_close(got, ref, rtol=2e-4, atol=2e-3)
    again = rows.loss_grad(coef, 0.25, loss, y.cuda(), w.cuda()).cpu()
    assert torch.equal(got, again)                 # deterministic: no atomics
    mm = rows.margins(coef, 0.25).cpu().double()
    torch.testing.assert_close(mm, m, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_gpu_text_pipeline_tokenizer_hashingtf_lr_stays_sparse():
    """Tokenizer -> HashingTF (2^18 features) -> LogisticRegression on the GPU: the CSR
    features go through the sparse GLM kernels (a dense copy would be 200K x 2^18 x 4 B
    = 210 GB) and the model separates the two synthetic topics."""
    import pandas as pd
    from orange3_spark_amd.ml import Pipeline
    from orange3_spark_amd.ml.feature import HashingTF, Tokenizer
    s = Session(SessionConf().set("o3s.device", "cuda"))
    rng = np.random.default_rng(0)
    a_words = [f"alpha{i}" for i in range(300)]
    b_words = [f"beta{i}" for i in range(300)]
    common = [f"w{i}" for i in range(3000)]
    n = 200_000
    lab = rng.integers(0, 2, n)
    docs = []
    for i in range(n):
        topic = a_words if lab[i] else b_words
        k = 3 + int(rng.integers(0, 4))
        ws = list(rng.choice(topic, k)) + list(rng.choice(common, 12))
        docs.append(" ".join(ws))
    df = s.createDataFrame(pd.DataFrame({"text": docs, "label": lab.astype(float)}))
    pipe = Pipeline(stages=[Tokenizer(inputCol="text", outputCol="words"),
                            HashingTF(inputCol="words", outputCol="features"),
                            LogisticRegression(maxIter=20, regParam=0.001)])
    model = pipe.fit(df)
    auc = BinaryClassificationEvaluator().evaluate(model.transform(df))
    assert auc > 0.99, auc


@pytest.mark.gpu
def test_gpu_naive_bayes_sparse_counts():
    """Multinomial NB on CSR term counts on the GPU == the CPU fp64 fit."""
    import pandas as pd
    from orange3_spark_amd.frame import column as C
    from orange3_spark_amd.ml.classification import NaiveBayes
    rng = np.random.default_rng(2)
    n, d = 20_000, 3000
    X = rng.poisson(0.02, size=(n, d)).astype(np.float32)
    y = (X[:, :50].sum(1) > X[:, 50:100].sum(1)).astype(float)
    nz = [np.nonzero(r)[0] for r in X]
    indptr = torch.tensor(np.concatenate([[0], np.cumsum([len(z) for z in nz])]), dtype=torch.int64)
    idx = torch.tensor(np.concatenate(nz), dtype=torch.int32)
    val = torch.tensor(np.concatenate([X[i, z] for i, z in enumerate(nz)]), dtype=torch.float32)
    out = []
    for dev in ("cpu", "cuda"):
        s = Session(SessionConf().set("o3s.device", dev))
        df = s.createDataFrame(pd.DataFrame({"label": y}))
        df = df.withColumnData("features", C.SparseVectorColumn(indptr.to(s.device), idx.to(s.device),
                                                                val.to(s.device), d))
        m = NaiveBayes().fit(df)
        prob = np.stack(m.transform(df).toPandas()["probability"].map(lambda v: v.toArray()))
        out.append((m.theta.toArray(), prob))
    np.testing.assert_allclose(out[1][0], out[0][0], rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(out[1][1], out[0][1], rtol=1e-3, atol=5e-5)   # fp32 sparse margins
