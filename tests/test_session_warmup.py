"""Session warm-up (runtime/warmup.py): tiny fits of each estimator family at session
start, once per process, so the first user fit does not pay one-time kernel-loading costs
(profiles/gbt_cold_fit_r5.json)."""
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.runtime import warmup as W


@pytest.fixture
def fresh(monkeypatch):
    monkeypatch.setattr(W, "_DONE", set())
    a = Session.active()
    if a is not None:
        a.stop()
    yield
    a = Session.active()
    if a is not None:
        a.stop()


def test_auto_is_off_on_cpu(fresh):
    s = Session.getOrCreate(SessionConf().set("o3s.device", "cpu"))
    assert s.warmup_seconds == {}
    assert W._DONE == set()


def test_listed_families_run_once_per_process(fresh):
    s = Session.getOrCreate(SessionConf().set("o3s.device", "cpu").set("o3s.session.warmup", "glm,kmeans"))
    assert set(s.warmup_seconds) == {"glm", "kmeans"}
    assert all(v >= 0 for v in s.warmup_seconds.values())
    s.stop()
    s2 = Session.getOrCreate(SessionConf().set("o3s.device", "cpu").set("o3s.session.warmup", "glm,kmeans,trees"))
    assert set(s2.warmup_seconds) == {"trees"}          # glm / kmeans already warm in this process


def test_unknown_family_is_an_error(fresh):
    with pytest.raises(ValueError, match="unknown value or families"):
        Session.getOrCreate(SessionConf().set("o3s.device", "cpu").set("o3s.session.warmup", "glm,nope"))
    assert Session.active() is None                     # not published with the bad value
    with pytest.raises(ValueError):
        Session.getOrCreate(SessionConf().set("o3s.device", "cpu").set("o3s.session.warmup", "glm,nope"))


def test_false_disables(fresh):
    s = Session.getOrCreate(SessionConf().set("o3s.device", "cpu").set("o3s.session.warmup", "false"))
    assert s.warmup_seconds == {}


def test_user_fits_and_background_warmup_never_overlap():
    """The gate between user fits (shared, nested, any thread) and the background tiny
    fit (exclusive): a user fit waits for the tiny fit in flight, and the warm-up waits
    while any user fit runs."""
    import threading
    import time
    g = W._Gate()
    order = []
    g.warm_enter()

    def user():
        g.user_enter()
        order.append("user-in")
        g.user_exit()
    t = threading.Thread(target=user)
    t.start()
    time.sleep(0.05)
    order.append("warm-out")
    g.warm_exit()
    t.join(5)
    assert order == ["warm-out", "user-in"]
    g.user_enter()
    g.user_enter()                                    # nested fits (Pipeline stages)
    got = []
    w = threading.Thread(target=lambda: (g.warm_enter(), got.append("warm"), g.warm_exit()))
    w.start()
    time.sleep(0.05)
    assert got == []
    g.user_exit()
    time.sleep(0.05)
    assert got == []
    g.user_exit()
    w.join(5)
    assert got == ["warm"]


def test_lazy_and_preload_modes_parse():
    assert W.plan("auto") == ("preload", ()) and W.plan("background") == ("background", W.FAMILIES)
    assert W.plan("lazy") == ("lazy", ()) and W.plan("preload") == ("preload", ())
    assert W.plan("all") == ("eager", W.FAMILIES) and W.plan("false") == ("off", ())


def test_context_widget_warms_every_family_by_default():
    """The canvas creates its session ahead of the first fit: the Context widget's editor
    defaults to o3s.session.warmup=all (a plain script's auto only preloads)."""
    from orangecontrib.spark_amd.widgets.data.owcontext import OWSessionContext
    w = OWSessionContext()
    assert w.gui_parameters["o3s.session.warmup"].get_value() == "all"


@pytest.fixture
def fresh_gpu(fresh, monkeypatch):
    monkeypatch.setattr(W, "_PRELOADED", set())
    monkeypatch.setattr(W, "_FAILED", set())
    W.wait_background(120)
    monkeypatch.setattr(W, "_THREAD", None)
    yield
    W.wait_background(120)


@pytest.mark.gpu
def test_gpu_auto_only_preloads(fresh_gpu):
    """auto in a script: the session start loads the kernel code objects (~40 ms, no
    fit) and warms no family -- a session that only fits LR pays no GBT/ALS/KMeans fits."""
    import time
    t = time.perf_counter()
    s = Session.getOrCreate(SessionConf())
    start = time.perf_counter() - t
    assert s.device.type == "cuda"
    assert set(s.warmup_seconds) == {"preload"} and s.warmup_seconds["preload"] < 0.1 and start < 1.0
    from orange3_spark_amd.ml.classification import LogisticRegression
    LogisticRegression(maxIter=3).fit(s.synthetic.classification(50_000, 32, seed=1))
    assert set(s.warmup_seconds) == {"preload"} and W._DONE == {"glm"}
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_background_warmup_then_fits(fresh_gpu):
    """background: the families warm on a thread (private single-rank session, own
    stream) and finish; a fit afterwards is an ordinary fit."""
    s = Session.getOrCreate(SessionConf().set("o3s.session.warmup", "background"))
    assert W.wait_background(120)
    assert set(W.FAMILIES) <= set(s.warmup_seconds) and all(s.warmup_seconds[f] for f in W.FAMILIES)
    from orange3_spark_amd.ml.classification import LogisticRegression
    LogisticRegression(maxIter=3).fit(s.synthetic.classification(50_000, 32, seed=1))
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_user_fit_during_background_warmup(fresh_gpu):
    """A fit issued right after the session start runs while the background warm-up is
    still going: it preempts the tiny fit in flight, gives the same model as a fit with
    the warm-up off, and its family is not warmed again afterwards."""
    from orange3_spark_amd.ml.clustering import KMeans
    s = Session.getOrCreate(SessionConf().set("o3s.session.warmup", "background"))
    m1 = KMeans(k=8, maxIter=5, seed=3).fit(s.synthetic.blobs(200_000, 32, 8, seed=2))
    assert "kmeans" in W._DONE
    assert W.wait_background(120)
    assert "kmeans" not in s.warmup_seconds or s.warmup_seconds["kmeans"] is not None
    s.stop()
    s2 = Session.getOrCreate(SessionConf().set("o3s.session.warmup", "false"))
    m2 = KMeans(k=8, maxIter=5, seed=3).fit(s2.synthetic.blobs(200_000, 32, 8, seed=2))
    assert m1.summary.trainingCost == pytest.approx(m2.summary.trainingCost, rel=1e-9)


@pytest.mark.gpu
def test_gpu_lazy_warms_only_the_fitted_family(fresh_gpu):
    s = Session.getOrCreate(SessionConf().set("o3s.session.warmup", "lazy"))
    assert set(s.warmup_seconds) == {"preload"}
    from orange3_spark_amd.ml.classification import LogisticRegression
    df = s.synthetic.classification(50_000, 32, seed=1)
    LogisticRegression(maxIter=3).fit(df)
    assert set(s.warmup_seconds) == {"preload", "glm"} and W._DONE == {"glm"}
    LogisticRegression(maxIter=3).fit(df)
    assert set(s.warmup_seconds) == {"preload", "glm"}
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_listed_families_warm_at_session_start(fresh):
    s = Session.getOrCreate(SessionConf().set("o3s.session.warmup", "true"))
    assert set(s.warmup_seconds) >= set(W.FAMILIES)
    assert sum(v for v in s.warmup_seconds.values() if v) < 30
    torch.cuda.synchronize()


def test_warmup_fits_stay_out_of_the_trace(fresh):
    from orange3_spark_amd.runtime.tracing import TRACER
    TRACER.reset()
    s = Session.getOrCreate(SessionConf().set("o3s.device", "cpu").set("o3s.session.warmup", "kmeans")
                            .set("o3s.trace", "true"))
    try:
        assert set(s.warmup_seconds) == {"kmeans"}
        assert TRACER.enabled
        assert not any(k.startswith("kmeans") for k in TRACER.summary())
    finally:
        TRACER.enable(False)
        TRACER.reset()


def test_a_failing_warmup_fit_warns_and_the_session_still_starts(fresh, monkeypatch):
    def boom(s):
        raise RuntimeError("no kernel")
    monkeypatch.setitem(W._FIT, "glm", boom)
    with pytest.warns(RuntimeWarning, match="glm warm-up fit failed"):
        s = Session.getOrCreate(SessionConf().set("o3s.device", "cpu").set("o3s.session.warmup", "glm"))
    assert s.warmup_seconds == {"glm": None}
    assert "glm" not in W._DONE
