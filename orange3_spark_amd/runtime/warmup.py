"""Device warm-up: what a process's first fit would otherwise pay once.

The first fit of an estimator family in a process pays one-time costs that later fits do
not.  Measured on the GBT config (``tools/prof_coldfit.py``, ``profiles/coldstart_r6.json``):
the cold cost is almost all PyTorch's kernel code objects, loaded at the first launch of
each op (``index_select`` alone 133 ms, ``max`` / ``sum`` / ``zeros_like`` / ``stack`` /
``cumsum`` 8-23 ms each); this framework's own 13 fatbins load in 37 ms.  The reference's
estimators run on a JVM whose executors are already started and JIT-warm when the Orange
canvas fits its first model (``orangecontrib/spark/base/spark_ml_estimator.py:22``, the
cluster started at ``widgets/data/spark_context.py:76``).

Conf ``o3s.session.warmup``:

* ``auto`` (default) -- GPU sessions preload this framework's kernel code objects
  (~40 ms, no launch).  Executor-pool workers (the multi-GPU canvas) additionally warm
  every family at pool start (``all``, on a private single-rank session: no collective);
  the Context widget asks for ``all`` too, from its worker thread -- the canvas's first
  fit is then warm.  A plain script pays a family's cold cost in its first fit instead of
  tiny fits of families it may never use;
* ``true`` / ``all`` or a comma list of :data:`FAMILIES` -- preload plus tiny fits of
  those families at session start, synchronously;
* ``lazy`` -- preload, then each family's tiny fit right before its first real fit;
* ``background`` -- preload, then the families' tiny fits on a background thread
  (private single-rank session, own HIP stream).  A user fit preempts the tiny fit in
  flight at its next iteration (progress / cancel hook) and the warm-up waits while user
  fits run (:func:`user_fit`), so module caches are never shared.  Measured: it only
  pays when the first fit comes > ~1.5 s after the session start (code-object loading
  in the background thread still delays the main thread's launches), hence opt-in;
* ``preload`` -- the code objects only;  ``false`` -- nothing.

Warm-up kernels, collectives and phases of a background or private-session fit are
invisible to fault injection, ``COMM_STATS`` and the trace.  ``Session.warmup_seconds``
reports the time per step."""
from __future__ import annotations

import contextlib
import threading
import time
import warnings

FAMILIES = ("trees", "glm", "kmeans", "als")
_DONE: set = set()                       # families warm in this process
_RUNNING: set = set()                    # a family's tiny fit must not warm itself again
_FAILED: set = set()                     # a failed warm-up is not retried at every fit
_PRELOADED: set = set()
_TL = threading.local()                  # .warming: this thread runs a warm-up fit


def plan(value) -> tuple:
    """Parse ``o3s.session.warmup`` -> (mode, families).  Raises ValueError on an unknown
    value (checked when the session is built, before it is published)."""
    v = str(value if value is not None else "auto").strip().lower()
    if v in ("false", "0", "no", "off", "none", ""):
        return ("off", ())
    if v in ("auto", "preload"):
        return ("preload", ())
    if v == "background":
        return ("background", FAMILIES)
    if v == "lazy":
        return ("lazy", ())
    if v in ("true", "1", "yes", "on", "all"):
        return ("eager", FAMILIES)
    fams = tuple(f.strip() for f in v.split(",") if f.strip())
    bad = [f for f in fams if f not in FAMILIES]
    if bad:
        raise ValueError(f"o3s.session.warmup: unknown value or families {bad} "
                         f"(auto, true, lazy, background, preload, false, or a list of {', '.join(FAMILIES)})")
    return ("eager", fams)


def _fit_trees(s):
    from ..ml.classification import GBTClassifier
    GBTClassifier(maxDepth=3, maxIter=2, stepSize=0.1, seed=0).fit(s.synthetic.trees(20_000, 16, seed=7))


def _fit_glm(s):
    from ..ml.classification import LogisticRegression
    LogisticRegression(maxIter=2).fit(s.synthetic.classification(20_000, 16, seed=7, cache=False))


def _fit_kmeans(s):
    from ..ml.clustering import KMeans
    KMeans(k=4, maxIter=2, seed=0).fit(s.synthetic.blobs(20_000, 16, 4, seed=7))


def _fit_als(s):
    from ..ml.recommendation import ALS
    df = s.synthetic.ratings(2_000, 500, 40_000, rank=4, seed=7, implicit=True)
    ALS(rank=32, maxIter=1, implicitPrefs=True, seed=0).fit(df)


_FIT = {"trees": _fit_trees, "glm": _fit_glm, "kmeans": _fit_kmeans, "als": _fit_als}


# ---------------------------------------------------------------- user-fit / warm-up gate
class _Gate:
    """Readers (user fits, any thread, nested) vs one writer (the background tiny fit)."""

    def __init__(self):
        self.cond = threading.Condition()
        self.users = 0
        self.waiting = 0                 # user fits blocked on a warm-up (it yields to them)
        self.warming = False

    def user_enter(self):
        with self.cond:
            if self.warming:
                self.waiting += 1
                try:
                    while self.warming:
                        self.cond.wait()
                finally:
                    self.waiting -= 1
            self.users += 1

    def user_exit(self):
        with self.cond:
            self.users -= 1
            self.cond.notify_all()

    def warm_enter(self):
        with self.cond:
            while self.users or self.warming:
                self.cond.wait()
            self.warming = True

    def warm_exit(self):
        with self.cond:
            self.warming = False
            self.cond.notify_all()


GATE = _Gate()


@contextlib.contextmanager
def user_fit(family):
    """Around every local fit (``ml/base.py``): waits for a background tiny fit in flight
    and keeps new ones out until the fit ends; the family counts as warm afterwards."""
    if getattr(_TL, "warming", False):   # the warm-up's own fit
        yield
        return
    GATE.user_enter()
    try:
        yield
    finally:
        GATE.user_exit()
        if family is not None and family not in _DONE:
            _DONE.add(family)            # its cold cost is paid: the background skips it


# ---------------------------------------------------------------- steps
def _preload(session, out: dict) -> None:
    dev = session.device
    if dev.type != "cuda" or dev in _PRELOADED:
        return
    from ..ops import _native
    t = time.perf_counter()
    try:
        _native.preload()
    except Exception as e:  # noqa: BLE001 - the first launches load them instead
        warnings.warn(f"o3s.session.warmup: kernel preload failed ({type(e).__name__}: {e})", RuntimeWarning)
        return
    _PRELOADED.add(dev)
    out["preload"] = round(time.perf_counter() - t, 4)


def _run_family(session, fam: str, out: dict, quiet: bool = False) -> bool:
    """One family's tiny fit.  ``quiet`` (the background thread): invisible to fault
    injection / counters, and it YIELDS to user fits -- a user fit that starts while it
    runs makes it stop at its next iteration (FitCancelled); returns False then."""
    from . import faults, progress
    from .tracing import TRACER, suppressed
    was = TRACER.enabled                 # the warm-up fits stay out of the user's trace
    if not quiet:
        TRACER.enabled = False
    _RUNNING.add(fam)
    _TL.warming = True
    t = time.perf_counter()
    scope = (progress.progress_scope(lambda _p: None, lambda: GATE.waiting > 0) if quiet
             else progress.detached())
    try:
        with scope, suppressed(), (faults.quiet() if quiet else contextlib.nullcontext()):
            _FIT[fam](session)
            if session.device.type == "cuda":
                import torch
                torch.cuda.current_stream(session.device).synchronize()
        out[fam] = round(time.perf_counter() - t, 4)
        _DONE.add(fam)
        return True
    except progress.FitCancelled:        # preempted by a user fit: retried later
        if session.device.type == "cuda":
            import torch
            torch.cuda.current_stream(session.device).synchronize()
        return False
    except Exception as e:               # a warm-up failure must not stop the session or fit
        warnings.warn(f"o3s.session.warmup: the {fam} warm-up fit failed ({type(e).__name__}: {e}); "
                      "its first real fit pays the one-time costs instead", RuntimeWarning)
        out[fam] = None
        _FAILED.add(fam)
        return True
    finally:
        _TL.warming = False
        _RUNNING.discard(fam)
        if not quiet:
            TRACER.enabled = was


def _private_session(session):
    """A single-rank session on the same device for the background fits: its comm is a
    LocalComm whose collectives bypass the traced / counted wrappers."""
    from ..parallel.comm import LocalComm
    from ..session import Session

    class _QuietComm(LocalComm):
        all_reduce = LocalComm.all_reduce.__wrapped__

    conf = (session.conf.copy().set("o3s.session.warmup", "false").set("o3s.trace", "false")
            .set("spark.master", "local[1]").set("spark.executor.instances", "1"))
    return Session(conf, comm=_QuietComm(session.device), device=session.device)


_THREAD = None
_STOP = threading.Event()


def _stop_background() -> None:
    """At interpreter exit: let the tiny fit in flight finish and start no other, before
    the HIP runtime is torn down under a daemon thread still inside a launch."""
    _STOP.set()
    wait_background(60)


import atexit  # noqa: E402

atexit.register(_stop_background)


def _background(session, fams) -> None:
    import torch
    try:
        priv = _private_session(session)
        torch.cuda.set_device(session.device)
        stream = torch.cuda.Stream(session.device)
    except Exception as e:  # noqa: BLE001
        warnings.warn(f"o3s.session.warmup: background warm-up not started ({e})", RuntimeWarning)
        return
    queue = list(fams)
    retries = {f: 2 for f in fams}
    while queue:
        fam = queue.pop(0)
        if fam in _DONE or fam in _FAILED or _STOP.is_set():
            continue
        GATE.warm_enter()
        try:
            if fam in _DONE or _STOP.is_set():      # a user fit of this family ran meanwhile
                continue
            out: dict = {}
            with torch.cuda.stream(stream):
                finished = _run_family(priv, fam, out, quiet=True)
            session.warmup_seconds.update(out)
            if not finished and retries[fam] > 0:   # preempted: try again after the others
                retries[fam] -= 1
                queue.append(fam)
        finally:
            GATE.warm_exit()


def wait_background(timeout: float | None = None) -> bool:
    """Join the background warm-up (tests, benchmarks); True when it has finished."""
    th = _THREAD
    if th is not None:
        th.join(timeout)
        return not th.is_alive()
    return True


def warmup(session, pool_worker: bool = False) -> dict:
    """Session-start warm-up: the preload (GPU), then the families -- synchronously
    (``eager``; every family for an executor-pool worker in ``auto`` mode) or on the
    background thread.  Returns seconds per step run now."""
    global _THREAD
    out: dict = {}
    value = session.conf.get("o3s.session.warmup", "auto")
    mode, fams = plan(value)
    if pool_worker and str(value).strip().lower() == "auto" and session.device.type == "cuda":
        mode, fams = "eager", FAMILIES    # the canvas's executors: warm before the first fit
    if mode == "off":
        return out
    _preload(session, out)                # GPU only
    if mode == "eager" and session.device.type != "cuda" and str(value).strip().lower() in (
            "true", "1", "yes", "on", "all"):
        return out                        # "all" (the Context widget's default) warms GPUs only
    if mode == "eager":                   # listed families: also on CPU (explicit request)
        # several ranks: each warms alone on a private single-rank session (no collective)
        target = _private_session(session) if session.comm.world_size > 1 else session
        for fam in fams:
            if fam not in _DONE:
                _run_family(target, fam, out, quiet=target is not session)
    elif mode == "background" and session.device.type == "cuda":
        todo = [f for f in fams if f not in _DONE and f not in _FAILED]
        if todo and (_THREAD is None or not _THREAD.is_alive()):
            _THREAD = threading.Thread(target=_background, args=(session, todo), name="o3s-warmup", daemon=True)
            _THREAD.start()
    return out


def before_fit(family: str) -> None:
    """``lazy`` mode: warm ``family`` once per process with a tiny fit right before its
    first real fit.  No-op in the other modes, after the first call and on CPU."""
    if family in _DONE or family in _RUNNING or family in _FAILED or getattr(_TL, "warming", False):
        return
    from ..session import Session
    s = Session.active()
    if s is None or s.device.type != "cuda":
        return
    mode, _ = plan(s.conf.get("o3s.session.warmup", "auto"))
    if mode != "lazy":
        return
    out = {}
    _preload(s, out)
    _run_family(s, family, out)
    s.warmup_seconds.update(out)
