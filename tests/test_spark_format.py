"""Spark save-format parity, pinned by hand-written fixtures (tools/make_spark_fixtures.py
writes them from Spark 3.5's documented schemas, not with this framework's writers):
every fixture loads, predicts what the Spark model would (closed forms below), and
re-saving it reproduces Spark's layout -- the same parquet column names / types, the same
Spark row-metadata schema (VectorUDT / MatrixUDT annotations) and the same metadata keys."""
import json
import math
import os

import numpy as np
import pandas as pd
import pyarrow.parquet as pq
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.linalg import Vectors

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "spark_models")
ROW_META = b"org.apache.spark.sql.parquet.row.metadata"


@pytest.fixture(scope="module")
def s():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _parquet(path, sub):
    d = os.path.join(path, sub)
    f = sorted(x for x in os.listdir(d) if x.endswith(".parquet"))[0]
    return pq.read_table(os.path.join(d, f))


def _meta(path):
    with open(os.path.join(path, "metadata", "part-00000")) as f:
        return json.loads(f.readline())


def _strip(t):
    """Spark schema JSON without nullability (pyarrow round trips may relax it)."""
    if isinstance(t, dict):
        return {k: _strip(v) for k, v in t.items() if k not in ("nullable", "containsNull")}
    if isinstance(t, list):
        return [_strip(x) for x in t]
    return t


def _same_layout(fixture, saved, subs=("data",)):
    for sub in subs:
        a, b = _parquet(fixture, sub), _parquet(saved, sub)
        assert a.schema.names == b.schema.names, sub
        for fa, fb in zip(a.schema, b.schema):
            assert str(fa.type) == str(fb.type), (sub, fa.name, fa.type, fb.type)
        ra, rb = a.schema.metadata.get(ROW_META), (b.schema.metadata or {}).get(ROW_META)
        assert rb is not None, f"{sub}: no Spark row metadata in the saved parquet"
        assert _strip(json.loads(ra)) == _strip(json.loads(rb)), sub
    ma, mb = _meta(fixture), _meta(saved)
    assert ma["class"] == mb["class"] and ma["uid"] == mb["uid"]
    assert set(ma) <= set(mb), set(ma) - set(mb)
    for k, v in ma["paramMap"].items():
        assert mb["paramMap"][k] == v, k


def _frame(s, rows):
    return s.createDataFrame([(Vectors.dense(r),) for r in rows], ["features"])


def test_logistic_regression_fixture(s, tmp_path):
    from orange3_spark_amd.ml.classification import LogisticRegressionModel
    path = os.path.join(FIX, "logistic_regression")
    m = LogisticRegressionModel.load(path)
    assert m.uid == "LogisticRegression_4d3a1b2c5e6f" and m.getOrDefault("maxIter") == 25
    assert list(m.coefficients.toArray()) == [0.5, -1.25, 2.0] and m.intercept == 0.3
    X = [[1.0, 2.0, 3.0], [0.0, 0.0, 0.0], [-1.0, 0.5, 1.0]]
    out = m.transform(_frame(s, X)).toPandas()
    for x, p, pred in zip(X, out["probability"], out["prediction"]):
        z = 0.5 * x[0] - 1.25 * x[1] + 2.0 * x[2] + 0.3
        q = 1 / (1 + math.exp(-z))
        assert abs(p[1] - q) < 1e-12 and pred == (1.0 if q > 0.5 else 0.0)
    m.write().overwrite().save(str(tmp_path / "lr"))
    _same_layout(path, str(tmp_path / "lr"))


def test_kmeans_fixture(s, tmp_path):
    from orange3_spark_amd.ml.clustering import KMeansModel
    path = os.path.join(FIX, "kmeans")
    m = KMeansModel.load(path)
    assert [list(c) for c in m.clusterCenters()] == [[0.0, 0.0], [5.0, 5.0]]
    out = m.transform(_frame(s, [[0.1, -0.2], [4.0, 6.0], [2.4, 2.4]])).toPandas()
    assert list(out["prediction"]) == [0, 1, 0]
    m.write().overwrite().save(str(tmp_path / "km"))
    _same_layout(path, str(tmp_path / "km"))


def test_gbt_classifier_fixture(s, tmp_path):
    from orange3_spark_amd.ml.classification import GBTClassificationModel
    path = os.path.join(FIX, "gbt_classifier")
    m = GBTClassificationModel.load(path)
    assert m.getNumTrees == 2 and m.numFeatures == 2 and list(m.treeWeights) == [1.0, 0.1]
    X = [[0.2, 0.0], [0.9, 3.0], [0.7, 0.5]]
    out = m.transform(_frame(s, X)).toPandas()
    for x, raw, p in zip(X, out["rawPrediction"], out["probability"]):
        margin = (-0.6 if x[0] <= 0.5 else 0.8) * 1.0 + (0.2 if x[1] <= 1.0 else -0.3) * 0.1
        assert abs(raw[1] - margin) < 1e-12 and abs(raw[0] + margin) < 1e-12
        assert abs(p[1] - 1 / (1 + math.exp(-2 * margin))) < 1e-12
    m.write().overwrite().save(str(tmp_path / "gbt"))
    _same_layout(path, str(tmp_path / "gbt"), subs=("data", "treesMetadata"))


def test_als_fixture(s, tmp_path):
    from orange3_spark_amd.ml.recommendation import ALSModel
    path = os.path.join(FIX, "als")
    m = ALSModel.load(path)
    assert m.rank == 2
    df = s.createDataFrame(pd.DataFrame({"user": [10, 20, 10, 99], "item": [1, 2, 3, 1]}))
    out = m.transform(df).toPandas()
    U = {10: [1.0, 0.5], 20: [0.0, 2.0]}
    V = {1: [1.0, 1.0], 2: [2.0, -1.0], 3: [0.5, 0.25]}
    for u, i, p in zip(out["user"], out["item"], out["prediction"]):
        if u in U:
            assert abs(p - float(np.dot(U[u], V[i]))) < 1e-6
        else:
            assert math.isnan(p)                   # coldStartStrategy "nan"
    m.write().overwrite().save(str(tmp_path / "als"))
    _same_layout(path, str(tmp_path / "als"), subs=("userFactors", "itemFactors"))


def test_pipeline_fixture(s, tmp_path):
    from orange3_spark_amd.ml.base import PipelineModel
    path = os.path.join(FIX, "pipeline")
    m = PipelineModel.load(path)
    assert [type(st).__name__ for st in m.stages] == ["VectorAssembler", "LogisticRegressionModel"]
    df = s.createDataFrame(pd.DataFrame({"a": [1.0, -1.0], "b": [2.0, 0.5], "c": [3.0, 1.0]}))
    out = m.transform(df).toPandas()
    for (a, b, c), p in zip([(1.0, 2.0, 3.0), (-1.0, 0.5, 1.0)], out["probability"]):
        z = 0.5 * a - 1.25 * b + 2.0 * c + 0.3
        assert abs(p[1] - 1 / (1 + math.exp(-z))) < 1e-12
    m.write().overwrite().save(str(tmp_path / "pm"))
    assert _meta(str(tmp_path / "pm"))["paramMap"]["stageUids"] == _meta(path)["paramMap"]["stageUids"]
    stage = "stages/1_LogisticRegression_4d3a1b2c5e6f"
    _same_layout(os.path.join(path, stage), str(tmp_path / "pm" / stage))


def test_linear_svc_fixture(s, tmp_path):
    from orange3_spark_amd.ml.classification import LinearSVCModel
    path = os.path.join(FIX, "linear_svc")
    m = LinearSVCModel.load(path)
    assert list(m.coefficients.toArray()) == [1.5, -0.5] and m.intercept == -0.25
    X = [[1.0, 2.0], [0.0, 1.0], [2.0, 0.0]]
    out = m.transform(_frame(s, X)).toPandas()
    for x, raw, pred in zip(X, out["rawPrediction"], out["prediction"]):
        z = 1.5 * x[0] - 0.5 * x[1] - 0.25
        assert abs(raw[1] - z) < 1e-12 and abs(raw[0] + z) < 1e-12 and pred == (1.0 if z > 0.0 else 0.0)
    m.write().overwrite().save(str(tmp_path / "svc"))
    _same_layout(path, str(tmp_path / "svc"))


def test_linear_regression_fixture(s, tmp_path):
    from orange3_spark_amd.ml.regression import LinearRegressionModel
    path = os.path.join(FIX, "linear_regression")
    m = LinearRegressionModel.load(path)
    assert list(m.coefficients.toArray()) == [3.0, -1.0, 0.5] and m.intercept == 2.0
    X = [[1.0, 1.0, 1.0], [0.0, 2.0, -2.0]]
    out = m.transform(_frame(s, X)).toPandas()
    for x, p in zip(X, out["prediction"]):
        assert abs(p - (3.0 * x[0] - x[1] + 0.5 * x[2] + 2.0)) < 1e-12
    m.write().overwrite().save(str(tmp_path / "linreg"))
    _same_layout(path, str(tmp_path / "linreg"))


def test_standard_scaler_fixture(s, tmp_path):
    from orange3_spark_amd.ml.feature import StandardScalerModel
    path = os.path.join(FIX, "standard_scaler")
    m = StandardScalerModel.load(path)
    assert list(m.std.toArray()) == [2.0, 0.5] and list(m.mean.toArray()) == [1.0, -1.0]
    assert m.getOrDefault("withMean") is True and m.getOrDefault("withStd") is True
    out = m.transform(_frame(s, [[3.0, 0.0], [1.0, -1.5]])).toPandas()
    assert [list(v) for v in out["scaled"]] == [[1.0, 2.0], [0.0, -1.0]]
    m.write().overwrite().save(str(tmp_path / "ss"))
    _same_layout(path, str(tmp_path / "ss"))


def test_string_indexer_fixture(s, tmp_path):
    from orange3_spark_amd.ml.feature import StringIndexerModel
    path = os.path.join(FIX, "string_indexer")
    m = StringIndexerModel.load(path)
    assert list(m.labels) == ["red", "green", "blue"]
    out = m.transform(s.createDataFrame(pd.DataFrame({"color": ["blue", "red", "green", "red"]}))).toPandas()
    assert list(out["color_idx"]) == [2.0, 0.0, 1.0, 0.0]
    m.write().overwrite().save(str(tmp_path / "si"))
    _same_layout(path, str(tmp_path / "si"))


def test_random_forest_classifier_fixture(s, tmp_path):
    from orange3_spark_amd.ml.classification import RandomForestClassificationModel
    path = os.path.join(FIX, "random_forest_classifier")
    m = RandomForestClassificationModel.load(path)
    assert m.getNumTrees == 2 and m.numFeatures == 2 and m.numClasses == 2
    X = [[0.2, 1.0], [0.9, 3.0], [0.4, 2.5]]
    out = m.transform(_frame(s, X)).toPandas()
    for x, p in zip(X, out["probability"]):
        # Spark averages each tree's normalised leaf class counts
        t0 = [30 / 40, 10 / 40] if x[0] <= 0.5 else [5 / 60, 55 / 60]
        t1 = [8 / 40, 32 / 40] if x[1] <= 2.0 else [40 / 60, 20 / 60]
        assert abs(p[1] - (t0[1] + t1[1]) / 2) < 1e-12
    m.write().overwrite().save(str(tmp_path / "rf"))
    _same_layout(path, str(tmp_path / "rf"), subs=("data", "treesMetadata"))


def test_decision_tree_classifier_fixture(s, tmp_path):
    from orange3_spark_amd.ml.classification import DecisionTreeClassificationModel
    path = os.path.join(FIX, "decision_tree_classifier")
    m = DecisionTreeClassificationModel.load(path)
    assert m.numFeatures == 2 and m.numClasses == 2 and m.depth == 1
    out = m.transform(_frame(s, [[5.0, -1.0], [5.0, 0.0]])).toPandas()
    assert list(out["prediction"]) == [0.0, 1.0]
    assert abs(out["probability"][0][0] - 12 / 15) < 1e-12 and abs(out["probability"][1][1] - 21 / 25) < 1e-12
    m.write().overwrite().save(str(tmp_path / "dt"))
    _same_layout(path, str(tmp_path / "dt"))


def test_naive_bayes_fixture(s, tmp_path):
    from orange3_spark_amd.ml.classification import NaiveBayesModel
    path = os.path.join(FIX, "naive_bayes")
    m = NaiveBayesModel.load(path)
    theta = np.log([[0.5, 0.3, 0.2], [0.1, 0.2, 0.7]])
    np.testing.assert_allclose(m.theta.toArray(), theta, rtol=0, atol=1e-15)
    X = [[1.0, 0.0, 2.0], [3.0, 1.0, 0.0]]
    out = m.transform(_frame(s, X)).toPandas()
    for x, raw in zip(X, out["rawPrediction"]):
        ref = np.log([0.4, 0.6]) + theta @ np.asarray(x)
        np.testing.assert_allclose(np.asarray(raw), ref, rtol=1e-12, atol=1e-12)
    m.write().overwrite().save(str(tmp_path / "nb"))
    _same_layout(path, str(tmp_path / "nb"))


def test_min_max_scaler_fixture(s, tmp_path):
    from orange3_spark_amd.ml.feature import MinMaxScalerModel
    path = os.path.join(FIX, "min_max_scaler")
    m = MinMaxScalerModel.load(path)
    out = m.transform(_frame(s, [[1.0, 0.0], [4.0, -2.0]])).toPandas()
    assert [list(v) for v in out["scaled"]] == [[0.25, 0.5], [1.0, 0.0]]
    m.write().overwrite().save(str(tmp_path / "mm"))
    _same_layout(path, str(tmp_path / "mm"))


def test_idf_fixture(s, tmp_path):
    from orange3_spark_amd.ml.feature import IDFModel
    path = os.path.join(FIX, "idf")
    m = IDFModel.load(path)
    assert list(m.idf.toArray()) == [0.5, 1.25, 0.0] and list(m.docFreq) == [3, 1, 4] and m.numDocs == 4
    df = s.createDataFrame([(Vectors.dense([2.0, 1.0, 5.0]),)], ["tf"])
    assert list(m.transform(df).toPandas()["tfidf"][0]) == [1.0, 1.25, 0.0]
    m.write().overwrite().save(str(tmp_path / "idf"))
    _same_layout(path, str(tmp_path / "idf"))


def test_one_hot_encoder_fixture(s, tmp_path):
    from orange3_spark_amd.ml.feature import OneHotEncoderModel
    path = os.path.join(FIX, "one_hot_encoder")
    m = OneHotEncoderModel.load(path)
    assert list(m.categorySizes) == [3]
    out = m.transform(s.createDataFrame(pd.DataFrame({"c": [0.0, 1.0, 2.0]}))).toPandas()
    assert [list(v.toArray()) for v in out["c_vec"]] == [[1.0, 0.0], [0.0, 1.0], [0.0, 0.0]]   # dropLast
    m.write().overwrite().save(str(tmp_path / "ohe"))
    _same_layout(path, str(tmp_path / "ohe"))


def test_count_vectorizer_fixture(s, tmp_path):
    from orange3_spark_amd.ml.feature import CountVectorizerModel
    path = os.path.join(FIX, "count_vectorizer")
    m = CountVectorizerModel.load(path)
    assert list(m.vocabulary) == ["a", "b", "c"]
    df = s.createDataFrame([(["c", "a", "c", "z"],)], ["words"])
    assert list(m.transform(df).toPandas()["counts"][0].toArray()) == [1.0, 0.0, 2.0]
    m.write().overwrite().save(str(tmp_path / "cv"))
    _same_layout(path, str(tmp_path / "cv"))
