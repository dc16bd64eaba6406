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


@pytest.mark.gpu
def test_gpu_auto_preloads_then_warms_only_the_fitted_family(fresh, monkeypatch):
    """auto: the session start only loads the kernel code objects (no fit); a family's
    tiny warm-up fit runs right before its first real fit, once per process, and a
    session that only fits LR never warms the other families."""
    monkeypatch.setattr(W, "_PRELOADED", set())
    s = Session.getOrCreate(SessionConf())
    assert s.device.type == "cuda"
    assert set(s.warmup_seconds) == {"preload"} and s.warmup_seconds["preload"] < 1.0
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
