"""Device warm-up: what a process's first fit would otherwise pay once.

The first fit of an estimator family in a process pays one-time costs that later fits do
not: the HIP code objects of this framework's kernels (one fatbin per ``csrc/*.hip`` file)
and of PyTorch's are loaded at their first launch, and first calls set up host-side state.
On the GBT config (500M x 64, depth 8, 5 trees) that was 0.31 s of a 1.01 s first fit
(``profiles/gbt_cold_fit_r5.json``).  The reference's estimators run on a JVM whose
executors are already started and JIT-warm when the Orange canvas fits its first model
(``orangecontrib/spark/base/spark_ml_estimator.py:22``, cluster started at
``widgets/data/spark_context.py:76``); here the session pays the equivalent up front.

Conf ``o3s.session.warmup``:

* ``auto`` (default) -- GPU sessions preload the kernel code objects (``preload``: no
  launch, no collective, so SPMD ranks and executor-pool workers do it too) and warm each
  estimator family lazily, once per process, right before that family's first fit
  (``lazy``); a family the graph never fits costs nothing;
* ``preload`` -- the code objects only;  ``lazy`` -- preload + the per-family lazy warm-up;
* ``true`` / ``all`` or a comma list of :data:`FAMILIES` -- tiny fits of those families
  at session start (round-5 behaviour), plus the preload;
* ``false`` -- nothing.

The lazy warm-up is a tiny fit of the same family on a few thousand synthetic rows,
issued on the ranks in lock step (the fit about to run is collective on every rank
anyway), so it is safe on SPMD ranks and pool workers.  ``Session.warmup_seconds``
reports the time per step."""
from __future__ import annotations

import time
import warnings

FAMILIES = ("trees", "glm", "kmeans", "als")
_DONE: set = set()
_RUNNING: set = set()                    # a family's tiny fit must not warm itself again
_FAILED: set = set()                     # lazy: a failed warm-up is not retried at every fit
_PRELOADED: set = set()


def plan(value) -> tuple:
    """Parse ``o3s.session.warmup`` -> (mode, families).  Raises ValueError on an unknown
    value (checked when the session is built, before it is published)."""
    v = str(value if value is not None else "auto").strip().lower()
    if v in ("false", "0", "no", "off", "none", ""):
        return ("off", ())
    if v in ("auto", "lazy"):
        return ("lazy", ())
    if v == "preload":
        return ("preload", ())
    if v in ("true", "1", "yes", "on", "all"):
        return ("eager", FAMILIES)
    fams = tuple(f.strip() for f in v.split(",") if f.strip())
    bad = [f for f in fams if f not in FAMILIES]
    if bad:
        raise ValueError(f"o3s.session.warmup: unknown value or families {bad} "
                         f"(auto, lazy, preload, true, false, or a list of {', '.join(FAMILIES)})")
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


def _run_family(session, fam: str, out: dict) -> None:
    from .tracing import TRACER
    from . import progress
    was = TRACER.enabled                 # the warm-up fits stay out of the user's trace
    TRACER.enabled = False
    _RUNNING.add(fam)
    t = time.perf_counter()
    try:
        with progress.detached():        # and out of the caller's progress / cancel scope
            _FIT[fam](session)
        if session.device.type == "cuda":
            import torch
            torch.cuda.synchronize(session.device)
        out[fam] = round(time.perf_counter() - t, 4)
        _DONE.add(fam)
    except Exception as e:               # a warm-up failure must not stop the session or fit
        warnings.warn(f"o3s.session.warmup: the {fam} warm-up fit failed ({type(e).__name__}: {e}); "
                      "its first real fit pays the one-time costs instead", RuntimeWarning)
        out[fam] = None
    finally:
        _RUNNING.discard(fam)
        TRACER.enabled = was


def warmup(session) -> dict:
    """Session-start warm-up: the preload (GPU) and, in ``eager`` mode, the listed
    families' tiny fits.  Returns seconds per step run now."""
    out: dict = {}
    mode, fams = plan(session.conf.get("o3s.session.warmup", "auto"))
    if mode == "off":
        return out
    _preload(session, out)                # GPU only
    for fam in fams:                      # listed families: also on CPU (explicit request)
        if fam not in _DONE:
            _run_family(session, fam, out)
    return out


def before_fit(family: str) -> None:
    """Called by each family's fit entry: warms the family once per process (``lazy``
    mode) with a tiny fit, so the cold cost lands on a few thousand rows instead of the
    user's data.  No-op after the first call, on CPU, and when warm-up is off."""
    if family in _DONE or family in _RUNNING or family in _FAILED:
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
    if out.get(family) is None:
        _FAILED.add(family)
    s.warmup_seconds.update(out)
