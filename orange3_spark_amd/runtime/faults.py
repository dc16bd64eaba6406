"""Failure detection and fault injection (SURVEY §5 "Failure detection"; delegated to Spark
in the reference).

Single-node MI355X model: a fixed set of 1-8 ranks, so there is no elasticity -- a
failure must surface as a clear Python exception on every rank (which the widgets show
through ``self.error``) instead of a hang or a silent wrong answer.

* :class:`CommError` / :class:`DeviceError` wrap RCCL/gloo and HIP failures with the
  operation, rank and world size;
* collectives run under the process-group timeout (``o3s.comm.timeout``, default 30 min)
  and :func:`health_check` probes every rank over the CPU (gloo) side group with a short
  timeout;
* ``O3S_LAUNCH_BLOCKING=1`` synchronises after every native kernel launch so a faulting
  kernel is reported at its own call site;
* ``O3S_FAULT_INJECT="op:n[,op:n]"`` raises at the n-th call of ``op`` (e.g.
  ``comm.all_reduce:3``, ``kernel:10``) -- used by the tests to exercise the error paths.
"""
from __future__ import annotations

import contextlib
import os
import threading
from collections import Counter


class O3SError(RuntimeError):
    """Base class of framework runtime failures."""


class CommError(O3SError):
    def __init__(self, op: str, rank: int, world: int, backend: str, cause: BaseException | str):
        self.op, self.rank, self.world, self.backend = op, rank, world, backend
        super().__init__(f"collective {op} failed on rank {rank}/{world} ({backend}): {cause}")


class DeviceError(O3SError):
    def __init__(self, what: str, cause: BaseException | str):
        self.what = what
        super().__init__(f"device failure in {what}: {cause}")


class InjectedFault(O3SError):
    pass


class _Injector:
    def __init__(self):
        self._lock = threading.Lock()
        self.reset(os.environ.get("O3S_FAULT_INJECT", ""))

    def reset(self, spec: str = ""):
        with self._lock:
            self.plan = {}
            for item in filter(None, (s.strip() for s in spec.split(","))):
                op, _, n = item.rpartition(":")
                self.plan[op] = int(n)
            self.calls = Counter()

    def hit(self, op: str):
        if not self.plan or getattr(_QUIET, "on", False):
            return
        with self._lock:
            self.calls[op] += 1
            if self.plan.get(op) == self.calls[op]:
                raise InjectedFault(f"injected fault at {op} call #{self.calls[op]}")


INJECTOR = _Injector()
_QUIET = threading.local()               # engine-internal threads (warm-up) are not counted


@contextlib.contextmanager
def quiet():
    """Injection points reached by this thread inside are neither counted nor fired (the
    background warm-up's kernels and collectives are not the program under test)."""
    was = getattr(_QUIET, "on", False)
    _QUIET.on = True
    try:
        yield
    finally:
        _QUIET.on = was


def launch_blocking() -> bool:
    return os.environ.get("O3S_LAUNCH_BLOCKING", "0") not in ("0", "", "false")


def health_check(comm, timeout_s: float = 30.0) -> dict:
    """Probe all ranks: returns {"ok": bool, "world": n, "alive": [ranks]}.

    Uses a CPU-side gather with a timeout so a dead or hung rank is reported instead of
    blocking forever.  World size 1 is trivially healthy.
    """
    if comm.world_size == 1:
        return {"ok": True, "world": 1, "alive": [0]}
    import datetime

    import torch
    import torch.distributed as dist
    grp = getattr(comm, "_cpu_group", None) or getattr(comm, "group", None)
    buf = torch.zeros(comm.world_size, dtype=torch.int64)       # CPU tensor -> gloo side group
    buf[comm.rank] = 1
    try:
        h = dist.all_reduce(buf, group=grp, async_op=True)
        h.wait(timeout=datetime.timedelta(seconds=timeout_s))
    except Exception as e:  # noqa: BLE001
        return {"ok": False, "world": comm.world_size, "alive": [comm.rank], "error": str(e)}
    alive = [r for r in range(comm.world_size) if int(buf[r]) == 1]
    return {"ok": len(alive) == comm.world_size, "world": comm.world_size, "alive": alive}
