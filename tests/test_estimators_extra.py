"""NaiveBayes, MLP, OneVsRest, FM, Isotonic, AFT and GLR against scikit-learn / scipy
oracles on small data (CPU), plus save/load round trips."""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml import classification as CL
from orange3_spark_amd.ml import regression as RG
from orange3_spark_amd.ml.feature import VectorAssembler


@pytest.fixture(scope="module")
def session():
    return Session.getOrCreate()


def frame(session, X, **cols):
    pdf = pd.DataFrame(X, columns=[f"f{i}" for i in range(X.shape[1])])
    for k, v in cols.items():
        pdf[k] = v
    return VectorAssembler(inputCols=[f"f{i}" for i in range(X.shape[1])], outputCol="features").transform(
        session.createDataFrame(pdf))


def column(df, name):
    v = df.select(name).toPandas()[name]
    if len(v) and hasattr(v.iloc[0], "toArray"):
        return np.stack([x.toArray() for x in v])
    return np.asarray(v.tolist())


@pytest.fixture(scope="module")
def counts3(session):
    rng = np.random.default_rng(0)
    X = rng.poisson(2.0, (600, 5)).astype(float)
    y = rng.integers(0, 3, 600)
    X[y == 1, 0] += 3
    X[y == 2, 1] += 3
    return X, y, frame(session, X, label=y.astype(float))


def test_naive_bayes_multinomial_matches_sklearn(counts3):
    from sklearn.naive_bayes import MultinomialNB
    X, y, df = counts3
    m = CL.NaiveBayes(smoothing=1.0).fit(df)
    sk = MultinomialNB(alpha=1.0).fit(X, y)
    np.testing.assert_allclose(m.theta.toArray(), sk.feature_log_prob_, atol=1e-12)
    # Spark smooths the priors too: log((n_c + l) / (n + K l))
    cnt = np.bincount(y)
    np.testing.assert_allclose(m.pi.toArray(), np.log((cnt + 1) / (len(y) + 3)), atol=1e-12)
    assert (column(m.transform(df), "prediction") == sk.predict(X)).mean() > 0.99


def test_naive_bayes_gaussian_and_bernoulli(session, counts3):
    from sklearn.naive_bayes import BernoulliNB, GaussianNB
    X, y, df = counts3
    g = CL.NaiveBayes(modelType="gaussian").fit(df)
    sk = GaussianNB().fit(X, y)
    np.testing.assert_allclose(g.theta.toArray(), sk.theta_, atol=1e-10)
    np.testing.assert_allclose(g.sigma.toArray(), sk.var_, rtol=1e-8)
    np.testing.assert_allclose(column(g.transform(df), "probability"), sk.predict_proba(X), atol=1e-8)
    Xb = (X > 2).astype(float)
    dfb = frame(session, Xb, label=y.astype(float))
    b = CL.NaiveBayes(modelType="bernoulli").fit(dfb)
    skb = BernoulliNB(alpha=1.0).fit(Xb, y)
    np.testing.assert_allclose(b.theta.toArray(), skb.feature_log_prob_, atol=1e-12)
    assert (column(b.transform(dfb), "prediction") == skb.predict(Xb)).mean() > 0.99
    with pytest.raises(ValueError):
        CL.NaiveBayes(modelType="bernoulli").fit(df)


def test_naive_bayes_save_load(tmp_path, counts3):
    _, _, df = counts3
    m = CL.NaiveBayes(modelType="complement").fit(df)
    m.save(str(tmp_path / "nb"))
    m2 = CL.NaiveBayesModel.load(str(tmp_path / "nb"))
    np.testing.assert_allclose(column(m.transform(df), "rawPrediction"), column(m2.transform(df), "rawPrediction"))


def test_mlp_learns_and_roundtrips(tmp_path, counts3):
    X, y, df = counts3
    m = CL.MultilayerPerceptronClassifier(layers=[5, 8, 3], maxIter=200, seed=1).fit(df)
    acc = (column(m.transform(df), "prediction") == y).mean()
    assert acc > 0.75
    assert m.weights.size == 5 * 8 + 8 + 8 * 3 + 3
    m.save(str(tmp_path / "mlp"))
    m2 = CL.MultilayerPerceptronClassificationModel.load(str(tmp_path / "mlp"))
    np.testing.assert_allclose(column(m2.transform(df), "probability"), column(m.transform(df), "probability"))


def test_one_vs_rest(tmp_path, counts3):
    X, y, df = counts3
    ovr = CL.OneVsRest(classifier=CL.LogisticRegression(maxIter=50)).fit(df)
    pred = column(ovr.transform(df), "prediction")
    assert (pred == y).mean() > 0.7
    ovr.save(str(tmp_path / "ovr"))
    o2 = CL.OneVsRestModel.load(str(tmp_path / "ovr"))
    np.testing.assert_array_equal(column(o2.transform(df), "prediction"), pred)


def test_fm_classifier_and_regressor(session):
    rng = np.random.default_rng(1)
    X = rng.normal(0, 1, (800, 4))
    yb = ((X[:, 0] * X[:, 1] + 0.5 * X[:, 2]) > 0).astype(float)
    df = frame(session, X, label=yb)
    m = CL.FMClassifier(stepSize=0.05, maxIter=300, seed=3, factorSize=4).fit(df)
    assert (column(m.transform(df), "prediction") == yb).mean() > 0.85     # needs the pairwise term
    yr = X[:, 0] * X[:, 1] + 0.3 * X[:, 3]
    r = RG.FMRegressor(stepSize=0.05, maxIter=400, seed=3, factorSize=4).fit(frame(session, X, label=yr))
    pred = column(r.transform(frame(session, X, label=yr)), "prediction")
    assert np.mean((pred - yr) ** 2) < 0.1 * np.var(yr)


def test_isotonic_matches_sklearn(session, tmp_path):
    from sklearn.isotonic import IsotonicRegression as SkIso
    rng = np.random.default_rng(0)
    x = np.round(rng.uniform(0, 10, 500), 1)
    y = np.sin(x / 3) * 3 + x * 0.3 + rng.normal(0, 0.5, 500)
    df = frame(session, x[:, None], label=y)
    xt = np.linspace(-1, 11, 301)
    for inc in (True, False):
        m = RG.IsotonicRegression(isotonic=inc).fit(df)
        sk = SkIso(increasing=inc, out_of_bounds="clip").fit(x, y)
        np.testing.assert_allclose([m.predict(v) for v in xt], sk.predict(xt), atol=1e-10)
    m.save(str(tmp_path / "iso"))
    m2 = RG.IsotonicRegressionModel.load(str(tmp_path / "iso"))
    np.testing.assert_allclose(m2.boundaries.toArray(), m.boundaries.toArray())


def test_glr_families_match_sklearn(session):
    from sklearn.linear_model import GammaRegressor, LogisticRegression, PoissonRegressor
    rng = np.random.default_rng(0)
    X = rng.normal(0, 1, (500, 3))
    eta = 0.3 + X @ np.array([0.5, -0.2, 0.1])
    yp = rng.poisson(np.exp(eta)).astype(float)
    g = RG.GeneralizedLinearRegression(family="poisson", link="log").fit(frame(session, X, label=yp))
    sk = PoissonRegressor(alpha=0, tol=1e-10, max_iter=1000).fit(X, yp)
    np.testing.assert_allclose(g.coefficients.toArray(), sk.coef_, atol=1e-7)
    assert abs(g.intercept - sk.intercept_) < 1e-7
    yg = rng.gamma(2.0, np.exp(eta) / 2.0)
    g2 = RG.GeneralizedLinearRegression(family="gamma", link="log").fit(frame(session, X, label=yg))
    sk2 = GammaRegressor(alpha=0, tol=1e-10, max_iter=1000).fit(X, yg)
    np.testing.assert_allclose(g2.coefficients.toArray(), sk2.coef_, atol=1e-6)
    yb = (rng.uniform(size=500) < 1 / (1 + np.exp(-eta))).astype(float)
    g3 = RG.GeneralizedLinearRegression(family="binomial").fit(frame(session, X, label=yb))
    sk3 = LogisticRegression(penalty=None, tol=1e-10, max_iter=1000).fit(X, yb)
    np.testing.assert_allclose(g3.coefficients.toArray(), sk3.coef_[0], atol=1e-6)
    assert len(g3.summary.pValues) == 4 and g3.summary.numIterations < 25


def test_aft_matches_scipy(session):
    from scipy.optimize import minimize
    rng = np.random.default_rng(0)
    X = rng.normal(0, 1, (400, 3))
    eta = 0.3 + X @ np.array([0.5, -0.2, 0.1])
    t = np.exp(eta + 0.5 * np.log(rng.exponential(1.0, 400)))
    cens = (rng.uniform(size=400) < 0.8).astype(float)
    df = frame(session, X, label=t, censor=cens)
    a = RG.AFTSurvivalRegression(quantilesCol="q").fit(df)

    def nll(th):
        e = (np.log(t) - X @ th[:3] - th[3]) / np.exp(th[4])
        return np.mean(cens * (th[4] - e) + np.exp(e))
    r = minimize(nll, np.zeros(5), method="BFGS", options=dict(gtol=1e-10))
    np.testing.assert_allclose(a.coefficients.toArray(), r.x[:3], atol=1e-4)
    assert abs(a.scale - np.exp(r.x[4])) < 1e-4
    q = column(a.transform(df), "q")
    assert q.shape == (400, 9) and np.all(np.diff(q, axis=1) > 0)


@pytest.mark.parametrize("mt", ["multinomial", "bernoulli", "complement"])
def test_naive_bayes_sparse_counts_match_dense(mt):
    """Term-count (CSR) features fit and predict without densifying, same model as dense."""
    import torch
    from orange3_spark_amd.frame import column as C
    from orange3_spark_amd.ml.classification import NaiveBayes
    s = Session(SessionConf().set("o3s.device", "cpu"))
    rng = np.random.default_rng(7)
    n, d = 600, 30
    X = rng.poisson(0.4, size=(n, d)).astype(float)
    if mt == "bernoulli":
        X = (X > 0).astype(float)
    y = (X[:, :5].sum(1) > X[:, 5:10].sum(1)).astype(float)
    dense = s.createDataFrame(pd.DataFrame({"features": list(X), "label": y}))
    nz = [np.nonzero(r)[0] for r in X]
    indptr = torch.tensor(np.concatenate([[0], np.cumsum([len(z) for z in nz])]), dtype=torch.int64)
    sp = dense.withColumnData("features", C.SparseVectorColumn(
        indptr, torch.tensor(np.concatenate(nz), dtype=torch.int32),
        torch.tensor(np.concatenate([X[i, z] for i, z in enumerate(nz)]), dtype=torch.float32), d))
    a = NaiveBayes(modelType=mt).fit(dense)
    b = NaiveBayes(modelType=mt).fit(sp)
    np.testing.assert_allclose(b.theta.toArray(), a.theta.toArray(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(b.pi.toArray(), a.pi.toArray(), rtol=1e-12)
    pa = np.stack(a.transform(dense).toPandas()["probability"].map(lambda v: v.toArray()))
    pb = np.stack(b.transform(sp).toPandas()["probability"].map(lambda v: v.toArray()))
    np.testing.assert_allclose(pb, pa, rtol=1e-9, atol=1e-12)
