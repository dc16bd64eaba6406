"""LogisticRegression / LinearSVC on the CPU path vs scikit-learn (BASELINE config #1 plumbing)."""
import numpy as np
import pandas as pd
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.classification import LinearSVC, LogisticRegression
from orange3_spark_amd.ml.evaluation import BinaryClassificationEvaluator


@pytest.fixture(scope="module")
def session():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _data(session, n=1000, d=20, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)) * rng.uniform(0.5, 3, size=d)
    w = rng.normal(size=d)
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-(X @ w * 0.5 + 0.3)))).astype(float)
    import pandas as pd
    pdf = pd.DataFrame(X, columns=[f"f{i}" for i in range(d)])
    pdf["label"] = y
    from orange3_spark_amd.ml.feature import VectorAssembler
    df = VectorAssembler(inputCols=[f"f{i}" for i in range(d)], outputCol="features").transform(
        session.createDataFrame(pdf))
    return df, X, y


def test_lr_matches_sklearn_unregularised(session):
    from sklearn.linear_model import LogisticRegression as SK
    df, X, y = _data(session)
    m = LogisticRegression(maxIter=200, tol=1e-10).fit(df)
    sk = SK(penalty=None, max_iter=5000, tol=1e-12).fit(X, y)
    assert np.allclose(m.coefficients.toArray(), sk.coef_[0], rtol=2e-3, atol=2e-3)
    assert abs(m.intercept - sk.intercept_[0]) < 2e-3


def test_lr_l2_matches_sklearn_without_standardization(session):
    from sklearn.linear_model import LogisticRegression as SK
    df, X, y = _data(session, seed=1)
    lam = 0.05
    m = LogisticRegression(maxIter=300, tol=1e-12, regParam=lam, standardization=False).fit(df)
    # spark objective: mean loss + lam/2 ||w||^2  <=>  sklearn C = 1/(n*lam)
    sk = SK(C=1.0 / (len(y) * lam), max_iter=5000, tol=1e-12).fit(X, y)
    assert np.allclose(m.coefficients.toArray(), sk.coef_[0], rtol=1e-3, atol=1e-3)


def test_lr_l1_produces_sparsity(session):
    df, X, y = _data(session, seed=2)
    m = LogisticRegression(maxIter=200, regParam=0.1, elasticNetParam=1.0).fit(df)
    assert np.sum(m.coefficients.toArray() == 0) >= 3


def test_lr_transform_and_auc(session):
    from sklearn.metrics import roc_auc_score
    df, X, y = _data(session, seed=3)
    m = LogisticRegression(maxIter=50).fit(df)
    out = m.transform(df)
    p = np.array([r.probability[1] for r in out.select("probability").collect()])
    auc = BinaryClassificationEvaluator(rawPredictionCol="probability").evaluate(out)
    assert abs(auc - roc_auc_score(y, p)) < 1e-9
    pred = np.array([r.prediction for r in out.select("prediction").collect()])
    assert np.array_equal(pred, (p > 0.5).astype(float))


def test_lr_multinomial(session):
    from sklearn.linear_model import LogisticRegression as SK
    rng = np.random.default_rng(5)
    X = rng.normal(size=(600, 5))
    y = np.argmax(X @ rng.normal(size=(5, 3)) + rng.gumbel(size=(600, 3)), axis=1).astype(float)
    import pandas as pd
    pdf = pd.DataFrame({"features": list(X), "label": y})
    df = session.createDataFrame(pdf)
    m = LogisticRegression(maxIter=300, tol=1e-12, regParam=0.01, standardization=False).fit(df)
    sk = SK(C=1.0 / (600 * 0.01), max_iter=5000, tol=1e-12).fit(X, y)
    B = m.coefficientMatrix.toArray()
    assert np.allclose(B - B.mean(0), sk.coef_ - sk.coef_.mean(0), atol=2e-3)
    acc = (np.array([r.prediction for r in m.transform(df).collect()]) == y).mean()
    assert acc > 0.6


def test_linear_svc(session):
    from sklearn.svm import LinearSVC as SK
    df, X, y = _data(session, seed=4)
    m = LinearSVC(maxIter=300, regParam=0.01).fit(df)
    pred = np.array([r.prediction for r in m.transform(df).collect()])
    sk = SK(C=1.0 / (len(y) * 0.01), loss="hinge", max_iter=100000).fit(X, y)
    assert (pred == y).mean() > 0.8
    assert (pred == sk.predict(X)).mean() > 0.9


def test_sgd_solver_decreases_loss(session):
    df = session.synthetic.classification(5000, 16, seed=9)
    m = LogisticRegression(solver="sgd", maxIter=30, stepSize=1.0).fit(df)
    h = m.summary.objectiveHistory
    assert h[-1] < h[0] - 0.05


def test_weight_col(session):
    df, X, y = _data(session, seed=6)
    import torch as T
    from orange3_spark_amd.frame.column import NumericColumn
    w = np.where(y > 0, 2.0, 1.0)
    dfw = df.withColumnData("w", NumericColumn(T.from_numpy(w)))
    m = LogisticRegression(maxIter=200, tol=1e-10, weightCol="w").fit(dfw)
    from sklearn.linear_model import LogisticRegression as SK
    sk = SK(penalty=None, max_iter=5000, tol=1e-12).fit(X, y, sample_weight=w)
    assert np.allclose(m.coefficients.toArray(), sk.coef_[0], rtol=3e-3, atol=3e-3)


def _sparse_vs_dense(s, loss_model):
    from orange3_spark_amd.frame import column as C
    from orange3_spark_amd.frame.dataframe import DataFrame
    rng = np.random.default_rng(3)
    n, d = 1200, 40
    X = rng.normal(size=(n, d)) * (rng.uniform(size=(n, d)) < 0.15)            # ~15% dense
    X = X.astype(np.float32).astype(np.float64)          # CSR values are fp32: same data both ways
    y = (X @ rng.normal(size=d) + 0.2 * rng.normal(size=n) > 0).astype(float)
    dense = s.createDataFrame(pd.DataFrame({"features": list(X), "label": y}))
    nz = [np.nonzero(r)[0] for r in X]
    indptr = torch.tensor(np.concatenate([[0], np.cumsum([len(z) for z in nz])]), dtype=torch.int64)
    idx = torch.tensor(np.concatenate(nz), dtype=torch.int32)
    val = torch.tensor(np.concatenate([X[i, z] for i, z in enumerate(nz)]), dtype=torch.float32)
    sp = dense.withColumnData("features", C.SparseVectorColumn(indptr, idx, val, d))
    a = loss_model().fit(dense)
    b = loss_model().fit(sp)
    np.testing.assert_allclose(b.coefficients.toArray(), a.coefficients.toArray(), rtol=1e-6, atol=1e-7)
    pa = a.transform(dense).toPandas()["prediction"].to_numpy()
    pb = b.transform(sp).toPandas()["prediction"].to_numpy()
    np.testing.assert_allclose(pb, pa, rtol=1e-6, atol=1e-7)
    return sp, DataFrame


def test_sparse_features_match_dense_lr_svc_linreg(session):
    """CSR features take the sparse GLM path (never densified) and fit the same model."""
    from orange3_spark_amd.ml.classification import LinearSVC
    from orange3_spark_amd.ml.regression import LinearRegression
    from orange3_spark_amd.models.glm import SparseGlmData, make_glm_data
    sp, _ = _sparse_vs_dense(session, lambda: LogisticRegression(maxIter=100, regParam=0.01, tol=1e-10))
    assert isinstance(make_glm_data(sp.comm, sp.column_data("features"), torch.zeros(len(sp))), SparseGlmData)
    _sparse_vs_dense(session, lambda: LinearSVC(maxIter=100, regParam=0.01, tol=1e-10))
    _sparse_vs_dense(session, lambda: LinearRegression(maxIter=100, regParam=0.01, tol=1e-10))
