"""Every estimator family fitted on the GPU session vs the same fit on the CPU session.

The GPU path stores feature vectors as padded bf16 and computes in fp32 (hipBLASLt GEMMs,
gfx950 kernels); the CPU path is fp64.  Inputs are chosen exactly representable in bf16
so both sessions see identical data; predictions must agree (classification / cluster
assignments) or be close (regression values).
"""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml import classification as CL
from orange3_spark_amd.ml import clustering as CU
from orange3_spark_amd.ml import feature as F
from orange3_spark_amd.ml import regression as RG

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sessions():
    return (Session(SessionConf().set("o3s.device", "cuda")), Session(SessionConf().set("o3s.device", "cpu")))


def _frames(sessions, X, **cols):
    pdf = pd.DataFrame(X, columns=[f"f{i}" for i in range(X.shape[1])])
    for k, v in cols.items():
        pdf[k] = v
    va = F.VectorAssembler(inputCols=[f"f{i}" for i in range(X.shape[1])], outputCol="features")
    return [va.transform(s.createDataFrame(pdf)) for s in sessions]


def _col(df, name):
    v = df.select(name).toPandas()[name]
    if len(v) and hasattr(v.iloc[0], "toArray"):
        return np.stack([x.toArray() for x in v])
    return np.asarray(v.tolist(), dtype=np.float64)


@pytest.fixture(scope="module")
def cls_data(sessions):
    rng = np.random.default_rng(0)
    X = np.round(rng.normal(size=(4000, 6)) * 8) / 8            # exact in bf16
    y = ((X[:, 0] + 0.5 * X[:, 1] - 0.25 * X[:, 2] + 0.3 * rng.normal(size=4000)) > 0).astype(float)
    y3 = np.digitize(X[:, 0] + X[:, 3], [-0.7, 0.7]).astype(float)
    g, c = _frames(sessions, X, label=y, label3=y3, pos=np.abs(X[:, 0]) + 0.125)
    return X, y, y3, g, c


CLASSIFIERS = [
    lambda: CL.LogisticRegression(maxIter=50),
    lambda: CL.LinearSVC(maxIter=50),
    lambda: CL.DecisionTreeClassifier(maxDepth=4, seed=1),
    lambda: CL.RandomForestClassifier(numTrees=5, maxDepth=4, seed=1),
    lambda: CL.GBTClassifier(maxIter=5, maxDepth=3, seed=1),
    lambda: CL.NaiveBayes(modelType="gaussian"),
    lambda: CL.MultilayerPerceptronClassifier(layers=[6, 8, 2], maxIter=100, seed=1),
    lambda: CL.FMClassifier(maxIter=100, stepSize=0.05, seed=1),
]


@pytest.mark.parametrize("make", CLASSIFIERS, ids=lambda f: type(f()).__name__)
def test_classifier_gpu_matches_cpu(cls_data, make):
    _, y, _, g, c = cls_data
    pg = _col(make().fit(g).transform(g), "prediction")
    pc = _col(make().fit(c).transform(c), "prediction")
    assert (pg == pc).mean() > 0.97
    assert (pg == y).mean() > 0.8


def test_multiclass_and_ovr_gpu(cls_data):
    _, _, y3, g, c = cls_data
    for make in (lambda: CL.LogisticRegression(maxIter=50, labelCol="label3"),
                 lambda: CL.OneVsRest(classifier=CL.LogisticRegression(maxIter=30), labelCol="label3")):
        pg = _col(make().fit(g).transform(g), "prediction")
        pc = _col(make().fit(c).transform(c), "prediction")
        assert (pg == pc).mean() > 0.97 and (pg == y3).mean() > 0.8


def test_regressors_gpu_matches_cpu(sessions):
    rng = np.random.default_rng(1)
    X = np.round(rng.normal(size=(3000, 4)) * 8) / 8
    y = X @ np.array([1.0, -0.5, 0.25, 0.0]) + 0.1 * rng.normal(size=3000)
    yp = rng.poisson(np.exp(0.3 * X[:, 0])).astype(float)
    g, c = _frames(sessions, X, label=y, cnt=yp, t=np.exp(0.2 * X[:, 1]) + 0.1, censor=np.ones(3000))
    makers = [lambda: RG.LinearRegression(), lambda: RG.DecisionTreeRegressor(maxDepth=5),
              lambda: RG.GBTRegressor(maxIter=5, maxDepth=3), lambda: RG.RandomForestRegressor(numTrees=5),
              lambda: RG.GeneralizedLinearRegression(family="poisson", labelCol="cnt"),
              lambda: RG.IsotonicRegression(), lambda: RG.AFTSurvivalRegression(labelCol="t"),
              lambda: RG.FMRegressor(maxIter=100, stepSize=0.05)]
    for make in makers:
        pg = _col(make().fit(g).transform(g), "prediction")
        pc = _col(make().fit(c).transform(c), "prediction")
        scale = max(np.std(pc), 1e-6)
        assert np.sqrt(np.mean((pg - pc) ** 2)) < 0.05 * scale, type(make()).__name__


def test_clustering_gpu_matches_cpu(sessions):
    rng = np.random.default_rng(2)
    cent = np.array([[0, 0, 0], [6, 0, 0], [0, 6, 0], [0, 0, 6]], dtype=float)
    X = np.round(np.concatenate([c + rng.normal(0, 0.5, (500, 3)) for c in cent]) * 8) / 8
    g, c = _frames(sessions, X)
    for make in (lambda: CU.KMeans(k=4, seed=1), lambda: CU.BisectingKMeans(k=4, seed=1),
                 lambda: CU.GaussianMixture(k=4, seed=1)):
        mg, mc = make().fit(g), make().fit(c)
        pg, pc = _col(mg.transform(g), "prediction"), _col(mc.transform(c), "prediction")
        # same partition up to label permutation
        from sklearn.metrics import adjusted_rand_score
        assert adjusted_rand_score(pg, pc) > 0.99, type(mg).__name__
