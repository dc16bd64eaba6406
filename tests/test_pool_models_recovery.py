"""Executor-resident models and lineage recovery of the driver + executor pool
(runtime/executors.py, session.DriverSession).

* A large fitted model (ALS factors) stays on the executors: the driver gets a handle that
  is still ``isinstance(h, ALSModel)``; fit + transform + userFactors + save + load move
  well under 1 MB through the driver pipes for a >= 100 MB model (reference: the Model
  Transformer's ``model.transform(df)``, orangecontrib/spark/widgets/ml/spark_ml_model.py:53,
  and ``method().fit`` in orangecontrib/spark/base/spark_ml_estimator.py:19-25).
* An executor killed with SIGKILL mid-session: the next call respawns the pool and
  rebuilds handles from their lineage (catalog table, derived frames, driver-held host
  frames, temp views) -- Spark's lineage recompute behind ``df.cache()``
  (orangecontrib/spark/widgets/data/spark_df_cache.py:39).
* A wedged rank surfaces as an error within the watchdog instead of hanging the GUI.
"""
import os
import signal
import time

import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.runtime.executors import ExecutorLost, RemoteModel, payload_bytes

pytestmark = pytest.mark.timeout(900)


def _pool(tmp_path, n=2, **extra):
    conf = (SessionConf().set("spark.executor.instances", str(n)).set("o3s.device", "cpu")
            .set("spark.sql.warehouse.dir", str(tmp_path / "wh")))
    for k, v in extra.items():
        conf.set(k, v)
    return Session(conf)


def _local_payload(model):
    return payload_bytes(model)


def test_large_als_model_stays_on_executors(tmp_path):
    from orange3_spark_amd.ml.recommendation import ALS, ALSModel
    s = _pool(tmp_path)
    prev = Session._active
    Session._active = s
    try:
        pool = s.pool
        df = s.synthetic.ratings(450_000, 2_000, 1_200_000, rank=8, seed=3, implicit=True)
        b0 = pool.bytes_sent + pool.bytes_received
        model = ALS(rank=64, maxIter=1, implicitPrefs=True, cgIters=1, seed=0).fit(df)
        assert type(model) is RemoteModel
        assert isinstance(model, ALSModel) and model.uid.startswith("ALS")
        pred = model.transform(df)
        n_pred = pred.count()
        n_users = model.userFactors.count()
        path = str(tmp_path / "als_model")
        model.write().overwrite().save(path)
        loaded = ALSModel.load(path)
        s_loaded = loaded.transform(df).agg({"prediction": "sum"}).collect()[0][0]
        s_orig = pred.agg({"prediction": "sum"}).collect()[0][0]
        moved = pool.bytes_sent + pool.bytes_received - b0
        size = pool.apply(_local_payload, model)
        assert size >= 100e6, size                      # factors: >= 100 MB on every executor
        assert moved < 1 << 20, moved                   # ... and < 1 MB crossed the driver pipes
        assert n_pred == 1_200_000 and 400_000 < n_users <= 450_000
        assert type(loaded) is RemoteModel and isinstance(loaded, ALSModel)
        assert s_loaded == pytest.approx(s_orig, rel=1e-6)
        assert os.path.isdir(os.path.join(path, "userFactors")) and os.path.isdir(os.path.join(path, "metadata"))
        # recommendations are row-sharded: one row per user over all executors
        recs = model.recommendForUserSubset(df.limit(50), 3)
        assert recs.count() == df.limit(50).select("user").distinct().count()
    finally:
        Session._active = prev
        s.stop()


def test_small_models_still_travel_by_value(tmp_path):
    from orange3_spark_amd.ml.classification import LogisticRegression
    from orange3_spark_amd.ml.feature import VectorAssembler
    s = _pool(tmp_path)
    try:
        rng = np.random.default_rng(0)
        pdf = pd.DataFrame(rng.normal(size=(400, 3)), columns=list("abc"))
        pdf["label"] = (pdf.a > 0).astype(float)
        df = VectorAssembler(inputCols=list("abc"), outputCol="features").transform(s.createDataFrame(pdf))
        m = LogisticRegression(maxIter=5).fit(df)
        assert type(m).__name__ == "LogisticRegressionModel"          # a plain local object
        # a tiny resident threshold keeps even LR on the executors
        s2 = _pool(tmp_path, **{"o3s.executor.residentModelBytes": "1"})
        try:
            df2 = VectorAssembler(inputCols=list("abc"), outputCol="features").transform(s2.createDataFrame(pdf))
            h = LogisticRegression(maxIter=5).fit(df2)
            assert type(h) is RemoteModel and h.coefficients.toArray().shape == (3,)
            assert np.allclose(h.coefficients.toArray(), m.coefficients.toArray())
            assert h.transform(df2).count() == 400
        finally:
            s2.stop()
    finally:
        s.stop()


def _kill(pool, r):
    os.kill(pool.pids[r], signal.SIGKILL)
    t = time.time()
    while pool._procs[r].is_alive() and time.time() - t < 30:
        time.sleep(0.05)


def test_executor_loss_respawns_and_replays_lineage(tmp_path):
    s = _pool(tmp_path)
    events = []
    s.add_listener(events.append)
    try:
        rng = np.random.default_rng(1)
        pdf = pd.DataFrame({"a": rng.normal(size=500), "b": rng.normal(size=500), "g": ["x", "y"] * 250})
        s.createDataFrame(pdf).write.mode("overwrite").saveAsTable("t")
        tbl = s.table("t")
        derived = tbl.filter(tbl.a > 0).withColumn("z", tbl.b * 2)
        host = s.createDataFrame(pdf.iloc[:123])
        derived.createOrReplaceTempView("v")
        want = (tbl.count(), derived.count(), host.count(), float(derived.agg({"z": "sum"}).collect()[0][0]))
        old = s.pool
        _kill(old, 1)
        assert tbl.count() == want[0]                    # next call: respawn + replay
        assert s.pool is not old and s.pool.alive and not old.alive
        assert derived.count() == want[1] and host.count() == want[2]
        assert float(derived.agg({"z": "sum"}).collect()[0][0]) == pytest.approx(want[3], rel=1e-12)
        assert s.sql("SELECT count(*) AS n FROM v").collect()[0][0] == want[1]    # temp view replayed
        assert len(s.events) == 1 and events and "exited" in events[0]["reason"]
        assert s.executor_info()["respawns"] == 1
    finally:
        s.stop()


def test_replay_after_adopted_parent_is_dropped(tmp_path):
    """Respawn, use h1 (adopted), drop h1, then use h2 = f(h1) built before the kill: the
    replay must not reuse h1's released executor id, and the replay cache
    must not keep un-adopted ancestors alive."""
    import gc
    s = _pool(tmp_path)
    try:
        h1 = s.range(0, 1000)
        h2 = h1.filter(h1.id % 3 == 0)
        want = h2.count()
        _kill(s.pool, 0)
        assert h1.count() == 1000                     # respawn + adopt h1
        pool = s.pool
        del h1
        gc.collect()
        assert h2.count() == want                     # replays h1's recipe afresh
        assert h2.filter(h2.id > 500).count() == len([i for i in range(501, 1000) if i % 3 == 0])
        gc.collect()
        live = [k for k, r in pool._proxies.items() if r() is not None]
        assert len(live) <= 3, live                   # session + h2 (+ a transient), no pinned ancestors
    finally:
        s.stop()


def _wedge_straggler():
    from orange3_spark_amd.session import Session
    if Session.active().comm.rank == 1:
        time.sleep(3600)
    return 1


def _wedge_collective():
    from orange3_spark_amd.session import Session
    s = Session.active()
    if s.comm.rank == 1:
        time.sleep(3600)
    s.comm.barrier()
    return 1


@pytest.mark.parametrize("fn", [_wedge_straggler, _wedge_collective])
def test_wedged_rank_surfaces_within_watchdog(tmp_path, fn):
    s = _pool(tmp_path, **{"o3s.executor.commTimeout": "5", "o3s.executor.errorGrace": "2",
                           "o3s.executor.stragglerTimeout": "4"})
    try:
        df = s.range(0, 1000)
        assert df.count() == 1000
        t = time.time()
        with pytest.raises(ExecutorLost, match="timeout"):
            s.pool.apply(fn)
        assert time.time() - t < 60
        assert df.count() == 1000                        # the pool came back, range replayed
    finally:
        s.stop()


def test_unreplayable_handle_asks_to_rerun_upstream(tmp_path):
    s = _pool(tmp_path)
    try:
        df = s.range(0, 10)
        object.__setattr__(df, "_recipe", None)          # e.g. lineage lost with its executors
        _kill(s.pool, 0)
        with pytest.raises(ExecutorLost, match="re-run the upstream widgets"):
            df.count()
        assert s.range(0, 5).count() == 5
    finally:
        s.stop()


def test_executor_instances_auto_counts_gpus_without_initialising(monkeypatch):
    import torch
    from orange3_spark_amd import conf as CF
    from orange3_spark_amd.session import _wants_pool, resolve_executors
    assert CF.DEFAULTS["spark.executor.instances"] == "auto"
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    init = []
    monkeypatch.setattr(torch.cuda, "init", lambda: init.append(1))
    auto = lambda: SessionConf().set("spark.executor.instances", "auto")   # noqa: E731 (conftest pins 1)
    assert resolve_executors("auto") == 8 and resolve_executors("3") == 3
    assert _wants_pool(auto()) and not _wants_pool(auto().set("spark.master", "local[1]"))
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert resolve_executors("auto") == 1 and not _wants_pool(auto())
    assert _wants_pool(auto().set("o3s.executor.pool", "true"))
    assert not init


def test_context_widget_lists_devices_and_reports_respawn(tmp_path):
    from orangecontrib.spark_amd.widgets.base import SharedSession
    from orangecontrib.spark_amd.widgets.data.owcontext import OWSessionContext
    SharedSession._session = None
    Session._active = None
    ctx = OWSessionContext()
    from orange3_spark_amd.conf import DEFAULTS, SessionConf
    assert DEFAULTS["spark.executor.instances"] == "auto"
    # the editor shows the configured value (tests/conftest.py sets O3S_CONF_SPARK__EXECUTOR__INSTANCES)
    assert ctx.gui_parameters["spark.executor.instances"].get_value() == SessionConf().get("spark.executor.instances")
    ctx.set_param("o3s.device", "cpu").set_param("spark.sql.warehouse.dir", str(tmp_path / "wh"))
    ctx.set_param("spark.executor.instances", "2")
    s = ctx.create_context()
    try:
        assert "2 executors: cpu, cpu" in ctx.messages["info"]
        df = s.range(0, 100)
        _kill(s.pool, 0)
        assert df.count() == 100
        assert "respawned" in ctx.messages["warning"] and "re-run upstream" in ctx.messages["warning"]
    finally:
        s.stop()
        SharedSession._session = None
        Session._active = None


def test_pipeline_with_resident_stage_saves_and_loads_on_executors(tmp_path):
    """A PipelineModel travels by value while its large stages stay on the executors; saving
    it writes those stages from the executors and loading under the pool session brings
    them back as handles."""
    from orange3_spark_amd.ml.base import Pipeline, PipelineModel
    from orange3_spark_amd.ml.classification import LogisticRegression, LogisticRegressionModel
    from orange3_spark_amd.ml.feature import VectorAssembler
    s = _pool(tmp_path, **{"o3s.executor.residentModelBytes": "1"})
    prev = Session._active
    Session._active = s
    try:
        rng = np.random.default_rng(3)
        pdf = pd.DataFrame(rng.normal(size=(300, 3)), columns=list("abc"))
        pdf["label"] = (pdf.a - pdf.b > 0).astype(float)
        df = s.createDataFrame(pdf)
        pm = Pipeline(stages=[VectorAssembler(inputCols=list("abc"), outputCol="features"),
                              LogisticRegression(maxIter=10)]).fit(df)
        assert type(pm) is PipelineModel and type(pm.stages[-1]) is RemoteModel
        assert isinstance(pm.stages[-1], LogisticRegressionModel)
        before = pm.transform(df).agg({"prediction": "sum"}).collect()[0][0]
        path = str(tmp_path / "pm")
        pm.write().overwrite().save(path)
        back = PipelineModel.load(path)
        assert type(back.stages[-1]) is RemoteModel
        assert back.transform(df).agg({"prediction": "sum"}).collect()[0][0] == before
    finally:
        Session._active = prev
        s.stop()
