"""BisectingKMeans, GaussianMixture, LDA and PowerIterationClustering (CPU)."""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session
from orange3_spark_amd.ml import clustering as CL
from orange3_spark_amd.ml.feature import CountVectorizer, Tokenizer, VectorAssembler


@pytest.fixture(scope="module")
def session():
    return Session.getOrCreate()


@pytest.fixture(scope="module")
def blobs(session):
    rng = np.random.default_rng(0)
    cent = np.array([[0, 0, 0], [10, 0, 0], [0, 10, 0], [0, 0, 10]], dtype=float)
    X = np.concatenate([c + rng.normal(0, 0.5, (100, 3)) for c in cent])
    df = VectorAssembler(inputCols=list("abc"), outputCol="features").transform(
        session.createDataFrame(pd.DataFrame(X, columns=list("abc"))))
    return X, df


def test_bisecting_kmeans(blobs, tmp_path):
    X, df = blobs
    m = CL.BisectingKMeans(k=4, seed=1, maxIter=20).fit(df)
    assert len(m.clusterCenters()) == 4 and sum(m.summary.clusterSizes) == 400
    pred = np.asarray(m.transform(df).select("prediction").toPandas()["prediction"])
    # every cluster is a union of whole blobs or a part of one blob: blob purity per cluster
    for c in np.unique(pred):
        assert len(np.unique(np.arange(400)[pred == c] // 100)) <= 2
    assert m.computeCost(df) == pytest.approx(m.summary.trainingCost, rel=1e-9)
    m.save(str(tmp_path / "bkm"))
    m2 = CL.BisectingKMeansModel.load(str(tmp_path / "bkm"))
    np.testing.assert_array_equal(np.asarray(m2.transform(df).select("prediction").toPandas()["prediction"]), pred)


def test_gaussian_mixture_matches_sklearn_likelihood(blobs, tmp_path):
    from sklearn.mixture import GaussianMixture as SkG
    X, df = blobs
    m = CL.GaussianMixture(k=4, seed=2, tol=1e-6).fit(df)
    sk = SkG(4, random_state=0, reg_covar=0, tol=1e-8).fit(X)
    assert m.summary.logLikelihood == pytest.approx(sk.score(X) * len(X), rel=1e-4)
    assert sorted(m.summary.clusterSizes) == [100, 100, 100, 100]
    P = np.stack([v.toArray() for v in m.transform(df).select("probability").toPandas()["probability"]])
    np.testing.assert_allclose(P.sum(1), 1.0)
    m.save(str(tmp_path / "gmm"))
    m2 = CL.GaussianMixtureModel.load(str(tmp_path / "gmm"))
    np.testing.assert_allclose(m2.gaussians[0].cov.toArray(), m.gaussians[0].cov.toArray())


def test_lda_separates_topics(session, tmp_path):
    docs = ["apple banana apple fruit", "banana fruit smoothie", "car engine wheel", "engine car road wheel",
            "fruit apple pie", "road car traffic"] * 20
    dd = Tokenizer(inputCol="text", outputCol="words").transform(session.createDataFrame(pd.DataFrame({"text": docs})))
    cv = CountVectorizer(inputCol="words", outputCol="features").fit(dd)
    dd = cv.transform(dd)
    m = CL.LDA(k=2, maxIter=30, seed=1, subsamplingRate=0.5).fit(dd)
    tops = [set(cv.vocabulary[i] for i in r) for r in m.describeTopics(3).toPandas()["termIndices"]]
    fruit, cars = {"apple", "banana", "fruit", "smoothie", "pie"}, {"car", "engine", "wheel", "road", "traffic"}
    assert any(t <= fruit for t in tops) and any(t <= cars for t in tops)
    assert m.topicsMatrix().numRows == m.vocabSize() and m.topicsMatrix().numCols == 2
    assert np.isfinite(m.logPerplexity(dd)) and m.logLikelihood(dd) < 0
    th = np.stack([v.toArray() for v in m.transform(dd).select("topicDistribution").toPandas()["topicDistribution"]])
    np.testing.assert_allclose(th.sum(1), 1.0)
    assert (th[0].argmax() != th[2].argmax())
    m.save(str(tmp_path / "lda"))
    m2 = CL.LocalLDAModel.load(str(tmp_path / "lda"))
    np.testing.assert_allclose(m2.topicsMatrix().toArray(), m.topicsMatrix().toArray())
    assert not m.isDistributed()
    # optimizer="em": a DistributedLDAModel with the EM diagnostics; toLocal() keeps the topics
    me = CL.LDA(k=2, maxIter=15, seed=1, optimizer="em").fit(dd)
    assert isinstance(me, CL.DistributedLDAModel) and me.isDistributed()
    assert me.trainingLogLikelihood() < 0 and np.isfinite(me.logPrior())
    loc = me.toLocal()
    assert not loc.isDistributed()
    np.testing.assert_allclose(loc.topicsMatrix().toArray(), me.topicsMatrix().toArray())
    me.save(str(tmp_path / "lda_em"))
    assert isinstance(CL.DistributedLDAModel.load(str(tmp_path / "lda_em")), CL.DistributedLDAModel)


def test_power_iteration_clustering(session):
    edges = pd.DataFrame({"src": [0, 1, 2, 3, 4, 5, 0], "dst": [1, 2, 0, 4, 5, 3, 3],
                          "weight": [1, 1, 1, 1, 1, 1, 0.01]})
    out = CL.PowerIterationClustering(k=2, weightCol="weight").assignClusters(
        session.createDataFrame(edges)).toPandas().sort_values("id")
    c = out["cluster"].to_numpy()
    assert len(set(c[:3])) == 1 and len(set(c[3:])) == 1 and c[0] != c[3]
