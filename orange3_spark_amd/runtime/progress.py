"""Fit progress and cancellation (reference quirk Q14: ``fit`` ran synchronously on the Qt
main thread with no feedback, orangecontrib/spark/base/spark_ml_estimator.py:19-25).

The engine's iteration loops call :func:`report` with the fraction of the fit done
(per L-BFGS / SGD / IRLS iteration for the GLMs, per Lloyd iteration for KMeans, per ALS
iteration, per tree for GBT / RandomForest).  A caller that wants the values installs a
sink for the current thread -- ``Estimator.fit(df, progress=callback)``, or
``with progress_scope(callback):`` around any code that fits -- and gets monotonically
non-decreasing percentages 0..100.  The sink lives in a ``contextvars.ContextVar``, so
fits running on different threads (the widgets' worker threads) never see each other's
values, and a fit with no sink pays one ContextVar lookup per iteration.

``cancelled`` (optional, e.g. Orange's ``TaskState.is_interruption_requested``) is
polled at the same points; when it returns True the fit raises :class:`FitCancelled`.
Nested scopes (a Pipeline's stages, CrossValidator's folds) map the inner fit's 0..1
onto a sub-range of the outer one (:func:`sub_range`).
"""
from __future__ import annotations

import contextlib
import contextvars
from dataclasses import dataclass
from typing import Callable, Optional


class FitCancelled(RuntimeError):
    """Raised inside a fit whose caller asked to stop (the widget's task was cancelled)."""


@dataclass
class _Sink:
    callback: Callable[[float], None]
    cancelled: Optional[Callable[[], bool]]
    lo: float = 0.0
    hi: float = 100.0
    last: float = -1.0


_SINK: contextvars.ContextVar = contextvars.ContextVar("o3s_progress", default=None)


@contextlib.contextmanager
def progress_scope(callback: Callable[[float], None] | None, cancelled: Callable[[], bool] | None = None):
    """Report this thread's fit progress (percent, 0..100) to ``callback``."""
    if callback is None and cancelled is None:
        yield
        return
    tok = _SINK.set(_Sink(callback or (lambda _p: None), cancelled))
    try:
        yield
    finally:
        _SINK.reset(tok)


@contextlib.contextmanager
def sub_range(frac_lo: float, frac_hi: float):
    """Map nested reports (0..1) onto [frac_lo, frac_hi] of the enclosing scope's range."""
    s = _SINK.get()
    if s is None:
        yield
        return
    span = s.hi - s.lo
    inner = _Sink(s.callback, s.cancelled, s.lo + span * frac_lo, s.lo + span * frac_hi, s.last)
    tok = _SINK.set(inner)
    try:
        yield
    finally:
        _SINK.reset(tok)
        s.last = max(s.last, inner.last)


@contextlib.contextmanager
def detached():
    """No sink inside (a warm-up fit run on behalf of the engine, not the caller's fit)."""
    tok = _SINK.set(None)
    try:
        yield
    finally:
        _SINK.reset(tok)


def active() -> bool:
    return _SINK.get() is not None


def report(frac: float) -> None:
    """The current fit is ``frac`` (0..1) done; no-op without a sink.  Values never go
    backwards (a converged solver that reports fewer iterations than it budgeted)."""
    s = _SINK.get()
    if s is None:
        return
    if s.cancelled is not None and s.cancelled():
        raise FitCancelled("fit cancelled")
    f = min(1.0, max(0.0, float(frac)))
    p = s.lo + (s.hi - s.lo) * f
    if p > s.last:
        s.last = p
        s.callback(p)


def iteration(done: int, total: int) -> None:
    """``report(done / total)`` for an iteration counter."""
    if total > 0:
        report(done / total)


# ---------------------------------------------------------------- executor-pool relay
# A fit shipped to an executor pool (runtime/executors.py) runs in other processes: rank 0
# relays its percentages to the driver, which forwards them into the calling thread's sink
# (never raising there: the driver is in the middle of a pool command), and a cancel request
# travels the other way as a flag that the ranks OR together collectively at every report
# site, so all of them raise FitCancelled at the same iteration.

def watching() -> tuple:
    """(progress wanted, cancellation wanted) for the current thread's fit."""
    s = _SINK.get()
    return (s is not None, s is not None and s.cancelled is not None)


def forward(percent: float) -> None:
    """Feed a relayed percentage (0..100 of the remote fit) into this thread's sink without
    polling for cancellation."""
    s = _SINK.get()
    if s is None:
        return
    f = min(1.0, max(0.0, float(percent) / 100.0))
    p = s.lo + (s.hi - s.lo) * f
    if p > s.last:
        s.last = p
        s.callback(p)


def cancel_requested() -> bool:
    """Has this thread's caller asked to stop?  (Polls without raising.)"""
    s = _SINK.get()
    return bool(s is not None and s.cancelled is not None and s.cancelled())
