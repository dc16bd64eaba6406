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
    assert te._graph is None and tg._graph is not None
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
