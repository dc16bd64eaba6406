"""Runtime services: tracing, failure surfacing / fault injection, checkpoint + resume."""
import json

import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.classification import LogisticRegression
from orange3_spark_amd.ml.clustering import KMeans
from orange3_spark_amd.ml.recommendation import ALS
from orange3_spark_amd.runtime import faults
from orange3_spark_amd.runtime.tracing import TRACER, trace


@pytest.fixture
def session():
    return Session(SessionConf().set("o3s.device", "cpu"))


@pytest.fixture(autouse=True)
def _clean():
    yield
    faults.INJECTOR.reset("")
    TRACER.enable(False)
    TRACER.reset()


def test_tracing_records_phases_and_exports(session, tmp_path):
    TRACER.reset()
    TRACER.enable()
    df = session.synthetic.classification(4000, 8, seed=1)
    LogisticRegression(maxIter=5).fit(df)
    with trace("user.phase", note="x"):
        pass
    s = TRACER.summary()
    assert s["LogisticRegression.fit"]["calls"] == 1
    assert s["glm.pass"]["calls"] >= 2 and "comm.all_reduce" in s and "user.phase" in s
    assert "LogisticRegression.fit" in TRACER.table()
    out = json.load(open(TRACER.export_chrome(str(tmp_path / "t.json"))))
    names = {e["name"] for e in out["traceEvents"]}
    assert {"LogisticRegression.fit", "glm.pass"} <= names
    assert all(e["ph"] == "X" and e["dur"] >= 0 for e in out["traceEvents"])


def test_tracing_disabled_is_free(session):
    TRACER.reset()
    TRACER.enable(False)
    LogisticRegression(maxIter=2).fit(session.synthetic.classification(500, 4, seed=1))
    assert TRACER.summary() == {}


def test_injected_comm_fault_surfaces_in_estimator_and_widget(session):
    df = session.synthetic.classification(2000, 6, seed=2)
    faults.INJECTOR.reset("comm.all_reduce:3")
    with pytest.raises(faults.InjectedFault):
        LogisticRegression(maxIter=5).fit(df)
    # the widget layer reports it through self.error instead of raising
    from orangecontrib.spark_amd.widgets.ml.owclassification import OWClassification
    w = OWClassification()
    w.select_method("LogisticRegression")
    w.get_input(df)
    faults.INJECTOR.reset("comm.all_reduce:2")
    assert w.apply() is None
    assert "InjectedFault" in (w.messages["error"] or "")
    faults.INJECTOR.reset("")
    assert w.apply() is not None and not w.messages["error"]


def test_health_check_single_rank(session):
    assert session.health_check()["ok"]


def _crash_after_first_checkpoint(fit):
    faults.INJECTOR.reset("checkpoint.saved:1")
    with pytest.raises(faults.InjectedFault):
        fit()
    faults.INJECTOR.reset("")


def test_kmeans_resumes_from_checkpoint(tmp_path):
    s = Session(SessionConf().set("o3s.device", "cpu").set("o3s.checkpoint.interval", "2"))
    df = s.synthetic.blobs(3000, 4, k=5, seed=3)
    ref = KMeans(k=5, seed=1, maxIter=8, tol=0.0).fit(df)          # no checkpoint dir: plain run
    s.setCheckpointDir(str(tmp_path / "ck"))
    est = KMeans(k=5, seed=1, maxIter=8, tol=0.0)
    _crash_after_first_checkpoint(lambda: est.fit(df))
    steps = list((tmp_path / "ck").glob("KMeans-*/step-*"))
    assert len(steps) == 1 and steps[0].name.endswith("2")
    resumed = est.fit(df)
    np.testing.assert_allclose(np.array(resumed.clusterCenters()), np.array(ref.clusterCenters()), atol=1e-9)


def test_lr_and_als_resume(tmp_path):
    s = Session(SessionConf().set("o3s.device", "cpu").set("o3s.checkpoint.interval", "3"))
    df = s.synthetic.classification(3000, 8, seed=4)
    ref = LogisticRegression(maxIter=60, regParam=0.01, tol=1e-10).fit(df)
    s.setCheckpointDir(str(tmp_path / "ck"))
    est = LogisticRegression(maxIter=60, regParam=0.01, tol=1e-10)
    _crash_after_first_checkpoint(lambda: est.fit(df))
    res = est.fit(df)
    np.testing.assert_allclose(res.coefficients.toArray(), ref.coefficients.toArray(), atol=1e-6)   # both converged

    rng = np.random.default_rng(0)
    pdf = pd.DataFrame({"user": rng.integers(0, 40, 800), "item": rng.integers(0, 30, 800),
                        "rating": rng.normal(size=800)})
    rd = s.createDataFrame(pdf)
    als_ref = ALS(rank=3, maxIter=6, seed=1, checkpointInterval=2)
    s.conf.set("spark.checkpoint.dir", "")
    a0 = als_ref.fit(rd)
    s.setCheckpointDir(str(tmp_path / "ck2"))
    est2 = ALS(rank=3, maxIter=6, seed=1, checkpointInterval=2)
    _crash_after_first_checkpoint(lambda: est2.fit(rd))
    a1 = est2.fit(rd)
    np.testing.assert_allclose(a1._U.numpy(), a0._U.numpy(), atol=1e-6)


def test_checkpoint_key_tracks_data_and_completed_fits_clear(tmp_path):
    """A same-size fit on DIFFERENT data must not resume from the first fit's state, and a
    completed fit leaves no checkpoint behind (stale-resume bug)."""
    s = Session(SessionConf().set("o3s.device", "cpu"))
    s.setCheckpointDir(str(tmp_path / "ck"))
    def ratings(seed):
        r = np.random.default_rng(seed)
        return s.createDataFrame(pd.DataFrame({"user": r.integers(0, 40, 800), "item": r.integers(0, 30, 800),
                                               "rating": r.normal(size=800)}))
    a, b = ratings(1), ratings(2)
    ALS(rank=3, maxIter=4, seed=1, checkpointInterval=2).fit(a)
    assert not list((tmp_path / "ck").glob("ALS-*/step-*"))          # cleared on completion
    # leave a stale mid-fit checkpoint of A behind, then fit B (same row count)
    _crash_after_first_checkpoint(lambda: ALS(rank=3, maxIter=4, seed=1, checkpointInterval=2).fit(a))
    assert list((tmp_path / "ck").glob("ALS-*/step-*"))
    got = ALS(rank=3, maxIter=4, seed=1, checkpointInterval=2).fit(b)
    s.conf.set("spark.checkpoint.dir", "")
    fresh = ALS(rank=3, maxIter=4, seed=1, checkpointInterval=2).fit(b)
    np.testing.assert_allclose(got._U.numpy(), fresh._U.numpy(), atol=1e-9)
    np.testing.assert_allclose(got._V.numpy(), fresh._V.numpy(), atol=1e-9)

    s.setCheckpointDir(str(tmp_path / "ck2"))
    s.conf.set("o3s.checkpoint.interval", "2")
    x1 = s.synthetic.blobs(2000, 4, k=3, seed=5)
    x2 = s.synthetic.blobs(2000, 4, k=3, seed=6)
    _crash_after_first_checkpoint(lambda: KMeans(k=3, seed=1, maxIter=6, tol=0.0).fit(x1))
    got = KMeans(k=3, seed=1, maxIter=6, tol=0.0).fit(x2)
    s.conf.set("spark.checkpoint.dir", "")
    fresh = KMeans(k=3, seed=1, maxIter=6, tol=0.0).fit(x2)
    np.testing.assert_allclose(np.array(got.clusterCenters()), np.array(fresh.clusterCenters()), atol=1e-12)


def test_fit_stats_attached():
    """Every fitted model carries fitStats: wall seconds, local rows, collectives issued."""
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.classification import LogisticRegression
    df = Session(SessionConf().set("o3s.device", "cpu")).synthetic.classification(500, 4, seed=1)
    m = LogisticRegression(maxIter=5).fit(df)
    st = m.fitStats
    assert st["seconds"] > 0 and st["rows_local"] == 500 and st["rows_per_s_local"] > 0
    assert isinstance(st["collectives"], dict)


def test_fit_progress_per_iteration_and_cancellation():
    """Estimator.fit(progress=, cancelled=): per-iteration progress for KMeans
    / ALS / GBT, non-decreasing to 100, nested Pipeline stages mapped onto sub-ranges, and a
    cancel request stops the fit at the next iteration."""
    import numpy as np
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.base import Pipeline
    from orange3_spark_amd.ml.classification import GBTClassifier
    from orange3_spark_amd.ml.clustering import KMeans
    from orange3_spark_amd.ml.recommendation import ALS
    from orange3_spark_amd.runtime.progress import FitCancelled
    s = Session(SessionConf().set("o3s.device", "cpu"))
    blobs = s.synthetic.blobs(2000, 4, k=3, seed=1)
    seen = []
    KMeans(k=3, maxIter=8, tol=0.0, seed=1).fit(blobs, progress=seen.append)
    assert seen[0] == 0.0 and seen[-1] == 100.0 and all(b >= a for a, b in zip(seen, seen[1:])) and len(seen) >= 3
    assert all(v % 12.5 == 0 for v in seen)            # per Lloyd iteration of 8 (converged early)
    rng = np.random.default_rng(0)
    r = s.createDataFrame(pd.DataFrame({"user": rng.integers(0, 40, 500), "item": rng.integers(0, 30, 500),
                                        "rating": rng.normal(size=500)}))
    als = []
    ALS(rank=4, maxIter=5, seed=1).fit(r, progress=als.append)
    assert als == [0.0, 20.0, 40.0, 60.0, 80.0, 100.0]
    pipe = []
    Pipeline(stages=[KMeans(k=3, maxIter=4, tol=0.0, seed=1, predictionCol="c"),
                     KMeans(k=2, maxIter=4, tol=0.0, seed=1)]).fit(blobs, progress=pipe.append)
    assert pipe[-1] == 100.0 and all(b >= a for a, b in zip(pipe, pipe[1:]))
    assert any(0 < v < 50 for v in pipe) and any(50 <= v < 100 for v in pipe)
    calls = []

    def stop():
        calls.append(1)
        return len(calls) > 2
    with pytest.raises(FitCancelled):
        GBTClassifier(maxIter=10, maxDepth=3).fit(s.synthetic.trees(1000, 5, seed=2), cancelled=stop)
