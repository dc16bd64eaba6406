"""Driver + executor-pool runtime (runtime/executors.py): a Session with
``spark.executor.instances = N`` spawns N worker processes (gloo on CPU here, RCCL on the
GPU box); DataFrames are handles, fits ship the estimator and return local models.  Every
result must equal the single-process run on the same data (row sharding never changes the
answer), and the tutorial chain must run from the widgets with N executors."""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.frame import expr as F
from orange3_spark_amd.frame.dataframe import DataFrame
from orange3_spark_amd.runtime.executors import ExecutorError, RemoteDataFrame

pytestmark = pytest.mark.timeout(600)


def _pdf(n=1200, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 5))
    y = (X @ np.array([1.0, -2.0, 0.5, 0.0, 1.5]) + rng.normal(scale=0.3, size=n) > 0).astype(float)
    pdf = pd.DataFrame(X, columns=list("abcde"))
    pdf["label"] = y
    pdf["g"] = ["p", "q", "r"] * (n // 3)
    return pdf


def _workload(s):
    from orange3_spark_amd.ml.classification import GBTClassifier, LogisticRegression
    from orange3_spark_amd.ml.clustering import KMeans
    from orange3_spark_amd.ml.evaluation import BinaryClassificationEvaluator
    from orange3_spark_amd.ml.feature import StandardScaler, VectorAssembler
    from orange3_spark_amd.ml.base import Pipeline
    df = s.createDataFrame(_pdf())
    out = {"count": df.count(), "columns": df.columns}
    va = VectorAssembler(inputCols=list("abcde"), outputCol="features")
    feats = va.transform(df)
    lr = LogisticRegression(maxIter=30, regParam=0.01).fit(feats)
    out["lr"] = np.concatenate([lr.coefficients.toArray(), [lr.intercept]])
    out["lr_iters"] = lr.summary.totalIterations
    out["auc"] = BinaryClassificationEvaluator().evaluate(lr.transform(feats))
    sgd = LogisticRegression(solver="sgd", maxIter=6, tol=0.0, miniBatchFraction=0.3, seed=2).fit(feats)
    out["sgd"] = sgd.coefficients.toArray()
    pm = Pipeline(stages=[va, StandardScaler(inputCol="features", outputCol="sf"),
                          LogisticRegression(featuresCol="sf", maxIter=10)]).fit(df)
    out["pipe"] = pm.stages[-1].coefficients.toArray()
    km = KMeans(k=3, seed=1, maxIter=8).fit(feats)
    out["km"] = km.summary.trainingCost
    gbt = GBTClassifier(maxIter=3, maxDepth=3, seed=1).fit(feats)
    out["gbt"] = gbt.trainingLossHistory if hasattr(gbt, "trainingLossHistory") else None
    agg = df.groupBy("g").agg(F.sum("a").alias("sa")).orderBy("g").toPandas()
    out["agg"] = agg["sa"].round(9).tolist()
    out["filter"] = df.filter(df.a > 0.5).withColumn("z", df.b * 2).count()
    df.createOrReplaceTempView("t")
    out["sql"] = [tuple(r) for r in s.sql("SELECT g, count(*) AS n FROM t GROUP BY g ORDER BY g").collect()]
    return out


@pytest.fixture(scope="module")
def pool_session():
    s = Session(SessionConf().set("spark.executor.instances", "2").set("o3s.device", "cpu"))
    yield s
    s.stop()


def test_driver_session_is_a_pool(pool_session):
    s = pool_session
    assert type(s).__name__ == "DriverSession" and s.world_size == 2 and s.executors == 2
    assert "executors=2" in repr(s)
    info = s.executor_info()
    assert info["world"] == 2 and info["backend"] == "gloo"


def test_pool_results_match_single_process(pool_session):
    local = Session(SessionConf().set("o3s.device", "cpu"))
    try:
        a = _workload(local)
    finally:
        local.stop()
    b = _workload(pool_session)
    assert a["count"] == b["count"] == 1200 and a["columns"] == b["columns"]
    assert np.allclose(a["lr"], b["lr"], atol=1e-7) and a["lr_iters"] == b["lr_iters"]
    assert abs(a["auc"] - b["auc"]) < 1e-12
    assert np.allclose(a["sgd"], b["sgd"], rtol=1e-9, atol=1e-12)
    assert np.allclose(a["pipe"], b["pipe"], atol=1e-7)
    assert a["km"] == pytest.approx(b["km"], rel=1e-9)
    assert a["gbt"] is None or np.allclose(a["gbt"], b["gbt"], rtol=1e-9)
    assert a["agg"] == b["agg"] and a["filter"] == b["filter"] and a["sql"] == b["sql"]


def test_handles_behave_like_dataframes(pool_session):
    s = pool_session
    df = s.createDataFrame(_pdf(300))
    assert isinstance(df, DataFrame) and type(df) is RemoteDataFrame
    sel = df.select("a", (df.b + 1).alias("b1"))
    p = sel.toPandas()
    assert list(p.columns) == ["a", "b1"] and len(p) == 300
    assert df.schema.names == list(df.columns)
    rows = df.limit(3).collect()
    assert len(rows) == 3 and rows[0].g == "p"
    assert len(df) == 300                                  # len() of a handle = global rows
    # scatter: each executor holds only its slice of the host table
    assert s.pool.apply(_local_rows, df) == 150


def _executor_warmup_seconds():
    from orange3_spark_amd import Session
    return dict(Session.active().warmup_seconds)


def _local_rows(df):
    return int(df._n)


def test_executor_errors_surface_and_pool_survives(pool_session):
    s = pool_session
    df = s.createDataFrame(_pdf(60))
    with pytest.raises(ExecutorError, match="nope"):
        df.select("nope").count()
    assert s.pool.alive and df.count() == 60


def test_pool_fit_relays_progress_and_cancels_collectively(pool_session):
    """The multi-GPU canvas path (SURVEY Q14 on a DriverSession): a fit shipped to the
    executors reports rank 0's per-iteration progress into the caller's sink, and a cancel
    request stops every rank at the same iteration (FitCancelled on the driver, no
    watchdog teardown); the next fit on the same pool succeeds."""
    from orange3_spark_amd.ml.classification import GBTClassifier, LogisticRegression
    from orange3_spark_amd.ml.feature import VectorAssembler
    from orange3_spark_amd.runtime.progress import FitCancelled
    s = pool_session
    pids = list(s.pool.pids)
    feats = VectorAssembler(inputCols=list("abcde"), outputCol="features").transform(s.createDataFrame(_pdf(6000)))
    seen = []
    lr = LogisticRegression(maxIter=20, tol=0.0, regParam=0.01).fit(feats, progress=seen.append)
    assert seen[-1] == 100.0 and all(b >= a for a, b in zip(seen, seen[1:]))
    assert len(seen) >= 15 and any(40 <= v <= 60 for v in seen)      # per iteration, from rank 0
    gb = []
    GBTClassifier(maxIter=5, maxDepth=3, seed=1).fit(feats, progress=gb.append)
    assert gb[-1] == 100.0 and all(b >= a for a, b in zip(gb, gb[1:])) and len(gb) >= 5
    got = []
    with pytest.raises(FitCancelled):
        LogisticRegression(solver="sgd", maxIter=200, tol=0.0, regParam=0.01).fit(
            feats, progress=got.append, cancelled=lambda: bool(got) and got[-1] >= 50.0)
    assert 50.0 <= got[-1] <= 50.0 + 2 * 100.0 / 200       # stopped within about one iteration
    assert s.pool.alive and s.pool.pids == pids             # collective stop: no teardown
    again = LogisticRegression(maxIter=20, tol=0.0, regParam=0.01).fit(feats)
    np.testing.assert_allclose(again.coefficients.toArray(), lr.coefficients.toArray(), rtol=1e-9, atol=1e-12)


def test_dropped_handles_are_freed_on_executors(pool_session):
    import gc
    s = pool_session
    before = s.executor_info()["objects"]
    for _ in range(20):
        d = s.createDataFrame(_pdf(30))
        d.withColumn("z", d.a * 2)
    del d
    gc.collect()
    s.executor_info()                                      # garbage goes out with the next command
    after = s.executor_info()["objects"]
    assert after <= before + 2


def test_tutorial_replay_with_executors_matches_one_process(tmp_path):
    """The reference tutorial chain driven through the widgets with a Context of
    spark.executor.instances=4 gives the 1-process model, and the Context widget reports
    the executor count."""
    from orangecontrib.spark_amd.widgets.base import SharedSession
    from orangecontrib.spark_amd.workflow import Workflow
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tutorial = os.path.join(root, "orangecontrib", "spark_amd", "tutorials", "spark_ml.ows")
    res = {}
    for n in ("1", "4"):
        SharedSession._session = None
        Session._active = None
        wf = Workflow.load(tutorial).instantiate()
        ctx = wf.widget("Context")
        ctx.set_param("o3s.device", "cpu").set_param("spark.sql.warehouse.dir", str(tmp_path / f"wh{n}"))
        ctx.set_param("spark.executor.instances", n)
        s = ctx.create_context()
        try:
            if n == "4":
                assert any("executors=4" in str(m) for m in ctx.messages.values()), ctx.messages
            rng = np.random.default_rng(0)
            for name, rows in (("train", 1500), ("test", 500)):
                X = rng.normal(size=(rows, 6))
                y = (X @ [1.0, -1.0, 0.5, 0.0, 2.0, -0.5] + rng.normal(scale=0.5, size=rows) > 0).astype(int)
                pdf = pd.DataFrame(X, columns=[f"f{i}" for i in range(6)])
                pdf["outcome"] = y
                s.createDataFrame(pdf).write.mode("overwrite").saveAsTable(name)
            for title in ("Training data", "Testing Data"):
                w = wf.widget(title)
                w.refresh()
                w.submit()
            for title in ("Dataset Builder", "Dataset Builder (1)"):
                b = wf.widget(title)
                b.set_features([f"f{i}" for i in range(6)])
                b.set_label("outcome")
                b.commit()
            clf = wf.widget("Classification")
            clf.select_method("LogisticRegression").set_param("maxIter", "40")
            model = clf.apply()
            assert model is not None, clf.messages
            ev = wf.widget("Evaluation")
            ev.select_method("BinaryClassificationEvaluator")
            vals = ev.apply()
            res[n] = (model.coefficients.toArray(), vals["areaUnderROC"])
        finally:
            s.stop()
            SharedSession._session = None
            Session._active = None
    assert np.allclose(res["1"][0], res["4"][0], atol=1e-7)
    assert abs(res["1"][1] - res["4"][1]) < 1e-12


def _scatter_work(rank, world, port, out):
    import os
    import tracemalloc
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    s = Session(SessionConf().set("o3s.device", "cpu").set("spark.master", "spmd"))
    n = 1_000_000
    data = None
    if rank == 0:
        rng = np.random.default_rng(1)
        data = pd.DataFrame({c: rng.normal(size=n) for c in "abcd"})     # 32 MB on rank 0 only
    tracemalloc.start()
    df = s.createDataFrame(data, scatter_from=0)
    _, peak = tracemalloc.get_traced_memory()
    tracemalloc.stop()
    res = {"local": len(df), "count": df.count(), "peak": peak,
           "sum": float(df.agg(F.sum("a")).collect()[0][0])}
    import torch.distributed as dist
    objs = [None] * world
    dist.all_gather_object(objs, res)
    if rank == 0:
        import pickle
        with open(out, "wb") as f:
            pickle.dump(objs, f)
    dist.barrier()
    dist.destroy_process_group()


def test_spmd_scatter_ingest_keeps_host_memory_per_rank(tmp_path):
    """createDataFrame(data on rank 0 only, scatter_from=0): each rank receives only its
    row slice -- the non-source rank's peak host allocation is about half the table."""
    import pickle
    import socket
    import torch.multiprocessing as mp
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    out = str(tmp_path / "scatter.pkl")
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_scatter_work, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    r0, r1 = pickle.load(open(out, "rb"))
    table = 1_000_000 * 4 * 8
    assert r0["local"] == r1["local"] == 500_000 and r0["count"] == 1_000_000
    assert r1["peak"] < 0.75 * table, r1["peak"]          # ~half the table (+ framing)
    assert r0["sum"] == pytest.approx(float(np.random.default_rng(1).normal(size=1_000_000).sum()), rel=1e-9)


@pytest.mark.gpu
def test_gpu_pool_fits_and_transforms(monkeypatch):
    """Two executors sharing cuda:0 (gloo; RCCL needs a GPU per rank): the headline
    estimators fit through handles, the returned local models (host tensors) transform
    executor frames again, and the results match a single-process GPU session."""
    monkeypatch.setenv("O3S_DIST_BACKEND", "gloo")
    from orange3_spark_amd.ml.classification import GBTClassifier, LogisticRegression
    from orange3_spark_amd.ml.clustering import KMeans
    from orange3_spark_amd.ml.evaluation import BinaryClassificationEvaluator
    from orange3_spark_amd.ml.recommendation import ALS

    def run(s):
        out = {}
        df = s.synthetic.classification(200_000, 64, seed=3)
        lr = LogisticRegression(maxIter=10).fit(df)
        out["lr"] = lr.coefficients.toArray()
        out["auc"] = BinaryClassificationEvaluator().evaluate(lr.transform(df))
        sgd = LogisticRegression(solver="sgd", maxIter=5, tol=0.0).fit(df)
        out["sgd"] = sgd.coefficients.toArray()
        blobs = s.synthetic.blobs(50_000, 16, k=8, seed=2)
        km = KMeans(k=8, seed=1, maxIter=5).fit(blobs)
        out["km"] = km.summary.trainingCost
        out["km_pred"] = km.transform(blobs).select("prediction").toPandas()["prediction"].to_numpy()[:100]
        trees = s.synthetic.trees(60_000, 8, seed=4)
        gbt = GBTClassifier(maxIter=3, maxDepth=4, seed=1).fit(trees)
        out["gbt_auc"] = BinaryClassificationEvaluator().evaluate(gbt.transform(trees))
        r = s.synthetic.ratings(500, 300, 20_000, rank=4, seed=5)
        als = ALS(rank=4, maxIter=3, seed=1).fit(r)
        out["als"] = als.transform(r).select("prediction").toPandas()["prediction"].to_numpy()[:50]
        return out

    monkeypatch.delenv("O3S_DIST_BACKEND")
    local = Session(SessionConf().setAppName("local"))
    try:
        a = run(local)
    finally:
        local.stop()
    monkeypatch.setenv("O3S_DIST_BACKEND", "gloo")
    pool = Session(SessionConf().set("spark.executor.instances", "2"))
    try:
        assert type(pool).__name__ == "DriverSession" and all(d.startswith("cuda") for d in pool.pool.devices)
        # the executors warmed every estimator family at pool start (runtime/warmup.py):
        # the canvas's first fit on the pool is not a cold fit
        warm = pool.pool.apply(_executor_warmup_seconds)
        assert {"preload", "trees", "glm", "kmeans", "als"} <= set(warm) and all(warm.values()), warm
        b = run(pool)
    finally:
        pool.stop()
    assert np.allclose(a["lr"], b["lr"], atol=1e-4) and abs(a["auc"] - b["auc"]) < 1e-4
    assert np.allclose(a["sgd"], b["sgd"], rtol=1e-4, atol=1e-6)
    assert a["km"] == pytest.approx(b["km"], rel=1e-6) and (a["km_pred"] == b["km_pred"]).all()
    assert abs(a["gbt_auc"] - b["gbt_auc"]) < 1e-3
    assert np.allclose(a["als"], b["als"], atol=1e-3)
