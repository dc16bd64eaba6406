"""Device warm-up at session start.

The first fit of an estimator family in a process pays one-time costs that later fits do
not: the HIP code objects of this framework's and PyTorch's kernels are loaded at their
first launch, and first calls set up host-side state.  On the GBT config (500M x 64, depth
8, 5 trees) that is 0.31 s of a 1.01 s first fit; one tiny fit beforehand (0.19 s) makes
the first real fit 0.699 s against 0.696 s warm (``profiles/gbt_cold_fit_r5.json``).  The
reference's estimators run on a JVM whose executors are already started and JIT-warm when
the Orange canvas fits its first model (``orangecontrib/spark/base/spark_ml_estimator.py:22``);
here the session does the equivalent once per process: a tiny fit of each estimator family
on synthetic rows, right after the device is selected.

Conf ``o3s.session.warmup``: ``auto`` (default: GPU sessions of one rank -- SPMD ranks skip
it, so no collective runs outside the user's program), ``true`` / ``false``, or a comma
list of families out of :data:`FAMILIES`.  ``Session.warmup_seconds`` reports the time per
family; each family is warmed at most once per process."""
from __future__ import annotations

import time
import warnings

FAMILIES = ("trees", "glm", "kmeans", "als")
_DONE: set = set()


def _families(session) -> tuple:
    v = str(session.conf.get("o3s.session.warmup", "auto")).strip().lower()
    if v in ("false", "0", "no", "off", "none", ""):
        return ()
    if v == "auto":
        on = session.device.type == "cuda" and session.comm.world_size == 1
        return FAMILIES if on else ()
    if v in ("true", "1", "yes", "on", "all"):
        return FAMILIES
    fams = tuple(f.strip() for f in v.split(",") if f.strip())
    bad = [f for f in fams if f not in FAMILIES]
    if bad:
        raise ValueError(f"o3s.session.warmup: unknown families {bad} (known: {', '.join(FAMILIES)})")
    return fams


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


def warmup(session) -> dict:
    """Run the configured families' tiny fits (once per process); returns seconds per
    family run now (None for a family whose fit raised: warned, not fatal)."""
    from .tracing import TRACER
    out = {}
    fams = [f for f in _families(session) if f not in _DONE]
    if not fams:
        return out
    was = TRACER.enabled                 # the warm-up fits stay out of the user's trace
    TRACER.enabled = False
    try:
        for fam in fams:
            t = time.perf_counter()
            try:
                _FIT[fam](session)
                if session.device.type == "cuda":
                    import torch
                    torch.cuda.synchronize(session.device)
            except Exception as e:        # a warm-up failure must not stop the session
                warnings.warn(f"o3s.session.warmup: the {fam} warm-up fit failed ({type(e).__name__}: {e}); "
                              "its first real fit pays the one-time costs instead", RuntimeWarning)
                out[fam] = None
                continue
            _DONE.add(fam)
            out[fam] = round(time.perf_counter() - t, 4)
    finally:
        TRACER.enabled = was
    return out
