"""Tracing / profiling hooks (SURVEY §5 "Tracing / profiling"; the reference has none).

``trace(name)`` marks a phase -- an Estimator ``fit``, one solver iteration, a
collective, a kernel launch group -- in three places at once:

* a **roctx range** (``libroctx64``), so ``rocprofv3 --marker-trace`` / the ROCm timeline
  shows framework phases around the HIP kernels they launch;
* a ``torch.profiler.record_function`` scope when a torch profiler is active;
* the in-process :class:`Tracer` registry: call counts and wall time per phase, exported
  as a table or as Chrome-trace JSON (``chrome://tracing`` / Perfetto).

Disabled by default (one attribute test per call); enable with ``O3S_TRACE=1`` or the
session conf ``o3s.trace=true``.  ``O3S_TRACE_SYNC=1`` synchronises the device at range
boundaries so wall times equal device times (perturbs overlap; for analysis only).
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time
from collections import defaultdict


class _Roctx:
    def __init__(self):
        self.lib = None
        for cand in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(cand)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                self.lib = lib
                break
            except OSError:
                continue

    def push(self, name: str):
        if self.lib is not None:
            self.lib.roctxRangePushA(name.encode())

    def pop(self):
        if self.lib is not None:
            self.lib.roctxRangePop()

    def mark(self, name: str):
        if self.lib is not None:
            self.lib.roctxMarkA(name.encode())


class Tracer:
    """Process-wide phase registry (thread-safe)."""

    def __init__(self):
        self.enabled = os.environ.get("O3S_TRACE", "0") not in ("0", "", "false")
        self.sync = os.environ.get("O3S_TRACE_SYNC", "0") not in ("0", "", "false")
        self._lock = threading.Lock()
        self._stats = defaultdict(lambda: [0, 0.0])
        self._events: list = []
        self._roctx = None
        self._t0 = time.perf_counter()
        self.max_events = 200_000

    def enable(self, on: bool = True, sync: bool | None = None):
        self.enabled = bool(on)
        if sync is not None:
            self.sync = bool(sync)
        return self

    def reset(self):
        with self._lock:
            self._stats.clear()
            self._events.clear()
            self._t0 = time.perf_counter()

    @property
    def roctx(self) -> _Roctx:
        if self._roctx is None:
            self._roctx = _Roctx()
        return self._roctx

    def _sync(self):
        if self.sync:
            import torch
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                torch.cuda.synchronize()

    def record(self, name: str, t_start: float, dt: float, args: dict | None):
        with self._lock:
            s = self._stats[name]
            s[0] += 1
            s[1] += dt
            if len(self._events) < self.max_events:
                self._events.append((name, t_start - self._t0, dt, args or {}, threading.get_ident()))

    def summary(self) -> dict:
        """{phase: {"calls": n, "total_s": t, "mean_ms": m}} sorted by total time."""
        with self._lock:
            items = sorted(self._stats.items(), key=lambda kv: -kv[1][1])
            return {k: {"calls": c, "total_s": t, "mean_ms": 1e3 * t / max(c, 1)} for k, (c, t) in items}

    def table(self) -> str:
        rows = [f"{'phase':<48} {'calls':>7} {'total s':>10} {'mean ms':>10}"]
        for k, v in self.summary().items():
            rows.append(f"{k[:48]:<48} {v['calls']:>7} {v['total_s']:>10.4f} {v['mean_ms']:>10.3f}")
        return "\n".join(rows)

    def export_chrome(self, path: str, pid: int | None = None) -> str:
        """Write Chrome-trace JSON ("X" complete events, microseconds)."""
        pid = os.getpid() if pid is None else pid
        with self._lock:
            ev = [{"name": n, "ph": "X", "ts": ts * 1e6, "dur": dt * 1e6, "pid": pid, "tid": tid,
                   "args": {k: (v if isinstance(v, (int, float, str, bool)) else str(v)) for k, v in a.items()}}
                  for n, ts, dt, a, tid in self._events]
        with open(path, "w") as f:
            json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
        return path


TRACER = Tracer()
_OFF = threading.local()                 # per-thread suppression (the background warm-up)


@contextlib.contextmanager
def suppressed():
    """No phases are recorded from this thread inside (engine-internal work such as the
    warm-up fits stays out of the user's trace; other threads keep tracing)."""
    was = getattr(_OFF, "on", False)
    _OFF.on = True
    try:
        yield
    finally:
        _OFF.on = was


@contextlib.contextmanager
def trace(name: str, **args):
    """Mark a phase (no-op unless tracing is enabled)."""
    t = TRACER
    if not t.enabled or getattr(_OFF, "on", False):
        yield
        return
    t._sync()
    t.roctx.push(name)
    rf = None
    try:
        import torch.autograd.profiler as _p
        if _p._is_profiler_enabled:
            rf = _p.record_function(name)
            rf.__enter__()
    except Exception:  # noqa: BLE001 - profiler internals differ across versions
        rf = None
    t0 = time.perf_counter()
    try:
        yield
    finally:
        t._sync()
        dt = time.perf_counter() - t0
        if rf is not None:
            rf.__exit__(None, None, None)
        t.roctx.pop()
        t.record(name, t0, dt, args)


def traced(name: str | None = None):
    """Decorator form of :func:`trace`."""
    def deco(fn):
        label = name or fn.__qualname__

        def wrapper(*a, **k):
            if not TRACER.enabled or getattr(_OFF, "on", False):
                return fn(*a, **k)
            with trace(label):
                return fn(*a, **k)
        wrapper.__wrapped__ = fn
        wrapper.__name__ = fn.__name__
        wrapper.__doc__ = fn.__doc__
        return wrapper
    return deco


def mark(name: str):
    if TRACER.enabled and not getattr(_OFF, "on", False):
        TRACER.roctx.mark(name)
