"""Evaluator kernels (csrc/eval.hip) vs their PyTorch fp64 references, and the
evaluators end to end on CPU vs scikit-learn-style closed forms."""
import numpy as np
import pandas as pd
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.evaluation import (BinaryClassificationEvaluator, MulticlassClassificationEvaluator,
                                             RegressionEvaluator)
from orange3_spark_amd.ops import evaluation as EV


def test_evaluators_cpu_reference():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    rng = np.random.default_rng(0)
    y = rng.normal(size=500)
    p = y + rng.normal(scale=0.3, size=500)
    df = s.createDataFrame(pd.DataFrame({"label": y, "prediction": p}))
    assert RegressionEvaluator(metricName="rmse").evaluate(df) == pytest.approx(np.sqrt(np.mean((p - y) ** 2)))
    assert RegressionEvaluator(metricName="mae").evaluate(df) == pytest.approx(np.mean(np.abs(p - y)))
    r2 = 1 - np.sum((p - y) ** 2) / np.sum((y - y.mean()) ** 2)
    assert RegressionEvaluator(metricName="r2").evaluate(df) == pytest.approx(r2)
    yc = rng.integers(0, 3, 500).astype(float)
    pc = np.where(rng.uniform(size=500) < 0.7, yc, rng.integers(0, 3, 500)).astype(float)
    dfc = s.createDataFrame(pd.DataFrame({"label": yc, "prediction": pc}))
    assert MulticlassClassificationEvaluator(metricName="accuracy").evaluate(dfc) == pytest.approx(np.mean(yc == pc))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("weighted", [False, True])
def test_gpu_eval_kernels_match_torch(gpu, dtype, weighted):
    g = torch.Generator().manual_seed(1)
    n = 1_000_003
    y = torch.randn(n, generator=g, dtype=torch.float64).to(dtype)
    p = (y.double() + 0.2 * torch.randn(n, generator=g, dtype=torch.float64)).to(dtype)
    w = torch.rand(n, generator=g, dtype=torch.float64) if weighted else None
    a = EV.regression_stats(y.to(gpu), p.to(gpu), None if w is None else w.to(gpu)).cpu()
    b = EV.regression_stats_torch(y, p, w)
    assert torch.allclose(a, b, rtol=1e-10)
    k = 7
    yc = torch.randint(0, k, (n,), generator=g).to(dtype)
    pc = torch.randint(0, k, (n,), generator=g).to(dtype)
    a = EV.confusion(yc.to(gpu), pc.to(gpu), k, None if w is None else w.to(gpu)).cpu()
    b = EV.confusion_torch(yc, pc, k, w)
    assert torch.allclose(a, b, rtol=1e-10)
    raw = torch.randn(n, 2, generator=g, dtype=torch.float64).to(dtype)
    lab = (torch.rand(n, generator=g) < 0.3).to(dtype)
    lo, span = float(raw[:, 1].min()), float(raw[:, 1].max() - raw[:, 1].min())
    a = EV.score_hist(raw.to(gpu)[:, 1], lab.to(gpu), lo, span, 1 << 16, None if w is None else w.to(gpu)).cpu()
    b = EV.score_hist_torch(raw[:, 1], lab, lo, span, 1 << 16, w)
    assert torch.allclose(a, b, rtol=1e-9, atol=1e-9)
    if not weighted:
        assert torch.equal(a, b)                          # integer counts: exact


@pytest.mark.gpu
def test_gpu_binary_evaluator_hist_path_matches_exact(gpu, monkeypatch):
    from orange3_spark_amd.ml import evaluation as ME
    s = Session(SessionConf().set("o3s.device", "cuda"))
    rng = np.random.default_rng(2)
    y = (rng.uniform(size=200_000) < 0.4).astype(float)
    sc = y * 0.8 + rng.normal(size=200_000)
    df = s.createDataFrame(pd.DataFrame({"label": y, "rawPrediction": sc}))
    exact = BinaryClassificationEvaluator().evaluate(df)
    monkeypatch.setattr(ME, "EXACT_AUC_MAX_ROWS", 10)
    approx = BinaryClassificationEvaluator().evaluate(df)
    assert approx == pytest.approx(exact, abs=1e-4)


def test_training_summaries_match_evaluators():
    from orange3_spark_amd.ml.classification import LinearSVC, LogisticRegression
    from orange3_spark_amd.ml.regression import LinearRegression
    s = Session(SessionConf().set("o3s.device", "cpu"))
    df = s.synthetic.classification(3000, 6, seed=3)
    m = LogisticRegression(maxIter=30).fit(df)
    sm = m.summary
    out = m.transform(df)
    assert sm.areaUnderROC == pytest.approx(BinaryClassificationEvaluator(rawPredictionCol="probability")
                                            .evaluate(out), rel=1e-12)
    acc = MulticlassClassificationEvaluator(metricName="accuracy").evaluate(out)
    assert sm.accuracy == pytest.approx(acc) and sm.totalIterations > 0 and len(sm.objectiveHistory) > 1
    assert sm.labels == [0.0, 1.0] and len(sm.precisionByLabel) == 2
    assert sm.weightedRecall == pytest.approx(acc)
    roc = sm.roc.toPandas()
    assert roc.FPR.iloc[0] == 0 and roc.TPR.iloc[-1] == 1 and roc.FPR.is_monotonic_increasing
    f = sm.fMeasureByThreshold.toPandas()
    assert set(f.columns) == {"threshold", "F-Measure"} and f.threshold.is_monotonic_decreasing
    ev = m.evaluate(df)
    assert ev.areaUnderROC == pytest.approx(sm.areaUnderROC)
    svc = LinearSVC(maxIter=20).fit(df)
    assert 0.5 < svc.summary.areaUnderROC <= 1.0 and svc.evaluate(df).accuracy == pytest.approx(svc.summary.accuracy)
    rng = np.random.default_rng(1)
    X = rng.normal(size=(400, 3))
    y = X @ np.array([1.0, -2.0, 0.5]) + 3 + rng.normal(scale=0.5, size=400)
    rdf = s.createDataFrame(pd.DataFrame({"features": list(X), "label": y}))
    lm = LinearRegression().fit(rdf)
    rs = lm.summary
    A = np.c_[X, np.ones(400)]
    beta, *_ = np.linalg.lstsq(A, y, rcond=None)
    resid = y - A @ beta
    sigma2 = resid @ resid / (400 - 4)
    se = np.sqrt(np.diag(np.linalg.inv(A.T @ A)) * sigma2)
    assert np.allclose(rs.coefficientStandardErrors, se, rtol=1e-6)
    assert np.allclose(rs.tValues, beta / se, rtol=1e-6)
    assert rs.numInstances == 400 and rs.degreesOfFreedom == 396
    assert rs.r2 == pytest.approx(1 - resid @ resid / np.sum((y - y.mean()) ** 2), rel=1e-8)
    assert rs.rootMeanSquaredError == pytest.approx(np.sqrt(np.mean(resid ** 2)), rel=1e-8)
    assert rs.residuals.count() == 400 and lm.evaluate(rdf).meanAbsoluteError == pytest.approx(rs.meanAbsoluteError)


@pytest.mark.gpu
def test_gpu_exact_curve_matches_host(gpu):
    import numpy as np
    from orange3_spark_amd.ml import evaluation as EV
    g = torch.Generator().manual_seed(3)
    n = 200_000
    s = (torch.randint(0, 5000, (n,), generator=g).double() / 5000)      # many ties
    y = (torch.rand(n, generator=g) < 0.4).double()
    w = torch.rand(n, generator=g).double() + 0.5
    host = EV._exact_curve(s.numpy(), y.numpy(), w.numpy())
    dev = EV._exact_curve_device(s.to(gpu), y.to(gpu), w.to(gpu))
    for a, b in zip(host[:3], dev[:3]):
        assert a.shape == b.shape and np.allclose(a, b, rtol=1e-10)
    assert abs(host[3] - dev[3]) < 1e-6 and abs(host[4] - dev[4]) < 1e-6
