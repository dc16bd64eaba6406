"""RFormula, UnivariateFeatureSelector/ANOVA/F-value tests, Word2Vec and the multilabel /
ranking evaluators (CPU; sklearn oracles where one exists)."""
import numpy as np
import pandas as pd
import pytest
import torch

from orange3_spark_amd import Session
from orange3_spark_amd.ml import evaluation as EV
from orange3_spark_amd.ml import feature as F
from orange3_spark_amd.ml import stat as ST


@pytest.fixture(scope="module")
def session():
    return Session.getOrCreate()


def vec(df, name):
    return np.stack([v.toArray() for v in df.select(name).toPandas()[name]])


def test_rformula_encoding_and_roundtrip(session, tmp_path):
    pdf = pd.DataFrame({"y": ["a", "b", "a", "b", "a", "a"], "s": ["x", "y", "x", "z", "y", "x"],
                        "b": [1.0, 2, 3, 4, 5, 6], "c": [0.5, 0.1, 0.2, 0.3, 0.4, 0.9]})
    df = session.createDataFrame(pdf)
    m = F.RFormula(formula="y ~ s + b + s:b").fit(df)
    X = vec(m.transform(df), "features")
    # s levels by frequency: x(3), y(2), z(1) -> one-hot drops z; then b; then s:b
    np.testing.assert_allclose(X[0], [1, 0, 1, 1, 0])
    np.testing.assert_allclose(X[3], [0, 0, 4, 0, 0])
    lab = np.asarray(m.transform(df).select("label").toPandas()["label"])
    np.testing.assert_array_equal(lab, [0, 1, 0, 1, 0, 0])          # 'a' most frequent -> 0
    assert F.RFormula(formula="y ~ . - c").fit(df).resolvedFormula == "y ~ s + b"
    no_int = F.RFormula(formula="y ~ s - 1").fit(df)
    assert vec(no_int.transform(df), "features").shape[1] == 3      # no intercept: all levels
    m.save(str(tmp_path / "rf"))
    m2 = F.RFormulaModel.load(str(tmp_path / "rf"))
    np.testing.assert_allclose(vec(m2.transform(df), "features"), X)


def test_univariate_tests_match_sklearn(session):
    from sklearn.feature_selection import f_classif, f_regression
    rng = np.random.default_rng(0)
    X = rng.normal(size=(300, 5))
    yc = (X[:, 1] > 0).astype(float)
    yr = X[:, 2] * 2 + rng.normal(size=300)
    pdf = pd.DataFrame(X, columns=list("pqrst"))
    pdf["label"] = yc
    pdf["lr"] = yr
    df = F.VectorAssembler(inputCols=list("pqrst"), outputCol="features").transform(session.createDataFrame(pdf))
    a = ST.ANOVATest.test(df, "features", "label", flatten=True).toPandas()
    np.testing.assert_allclose(a["fValue"], f_classif(X, yc)[0], rtol=1e-9)
    np.testing.assert_allclose(a["pValue"], f_classif(X, yc)[1], rtol=1e-6, atol=1e-300)
    fv = ST.FValueTest.test(df, "features", "lr", flatten=True).toPandas()
    np.testing.assert_allclose(fv["fValue"], f_regression(X, yr)[0], rtol=1e-9)
    sel = F.UnivariateFeatureSelector(outputCol="sel").setFeatureType("continuous").setLabelType(
        "categorical").setSelectionThreshold(1).fit(df)
    assert sel.selectedFeatures == [1]
    sel2 = F.UnivariateFeatureSelector(outputCol="sel", labelCol="lr").setFeatureType("continuous").setLabelType(
        "continuous").setSelectionThreshold(1).fit(df)
    assert sel2.selectedFeatures == [2]
    assert vec(sel2.transform(df), "sel").shape == (300, 1)


def test_word2vec_groups_cooccurring_words(session, tmp_path):
    rng = np.random.default_rng(0)
    A = ["cat", "dog", "pet", "fur", "paw", "tail"]
    B = ["car", "road", "wheel", "engine", "fuel", "drive"]
    docs = [" ".join(rng.choice(A if i % 2 else B, 8)) for i in range(2000)]
    dd = F.Tokenizer(inputCol="t", outputCol="w").transform(session.createDataFrame(pd.DataFrame({"t": docs})))
    m = F.Word2Vec(vectorSize=16, minCount=1, inputCol="w", outputCol="v", maxIter=5, seed=1).fit(dd)
    syn = [w for w, _ in m.findSynonymsArray("cat", 5)]
    assert set(syn) <= set(A)
    assert m.getVectors().count() == 12
    V = vec(m.transform(dd), "v")
    assert V.shape == (2000, 16) and np.isfinite(V).all()
    m.save(str(tmp_path / "w2v"))
    m2 = F.Word2VecModel.load(str(tmp_path / "w2v"))
    assert [w for w, _ in m2.findSynonymsArray("cat", 5)] == syn


def test_multilabel_and_ranking_evaluators(session):
    pdf = pd.DataFrame({"prediction": [[0.0, 1.0], [0.0, 2.0], [], [2.0], [2.0, 0.0], [0.0, 1.0, 2.0], [1.0]],
                        "label": [[0.0, 2.0], [0.0, 1.0], [0.0], [2.0], [2.0, 0.0], [0.0, 1.0], [1.0, 2.0]]})
    df = session.createDataFrame(pdf)
    ev = EV.MultilabelClassificationEvaluator()
    # reference values from Spark's MultilabelMetrics documentation example
    assert ev.evaluate(df, {ev.metricName: "subsetAccuracy"}) == pytest.approx(2 / 7)
    assert ev.evaluate(df, {ev.metricName: "accuracy"}) == pytest.approx(0.5476190476, rel=1e-8)
    assert ev.evaluate(df, {ev.metricName: "hammingLoss"}) == pytest.approx(0.3333333333, rel=1e-8)
    assert ev.evaluate(df, {ev.metricName: "microF1Measure"}) == pytest.approx(16 / 23)   # tp 8, fp 3, fn 4
    rk = pd.DataFrame({"prediction": [[1.0, 6.0, 2.0, 7.0, 8.0, 3.0, 9.0, 10.0, 4.0, 5.0],
                                      [4.0, 1.0, 5.0, 6.0, 2.0, 7.0, 3.0, 8.0, 9.0, 10.0],
                                      [1.0, 2.0, 3.0, 4.0, 5.0]],
                       "label": [[1.0, 2.0, 3.0, 4.0, 5.0], [1.0, 2.0, 3.0], []]})
    rdf = session.createDataFrame(rk)
    re_ = EV.RankingEvaluator()
    # Spark RankingMetrics doc example: MAP 0.355026, precision@1 1/3, ndcg@3 1/3
    assert re_.evaluate(rdf) == pytest.approx(0.355026, abs=1e-6)
    assert re_.evaluate(rdf, {re_.metricName: "precisionAtK", re_.k: 1}) == pytest.approx(1 / 3)
    assert re_.evaluate(rdf, {re_.metricName: "ndcgAtK", re_.k: 3}) == pytest.approx(1 / 3)
    _ = torch
