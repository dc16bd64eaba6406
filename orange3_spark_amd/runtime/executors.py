"""Driver + executor-pool runtime: one Orange (driver) process drives N GPU worker processes.

Reference: the Context widget sizes the cluster (``spark.executor.instances=8``,
orangecontrib/spark/widgets/data/spark_context.py:41-42,76) and every ``fit`` then runs on
all executors (orangecontrib/spark/base/spark_ml_estimator.py:19-25).  Spark does this with
a JVM driver, Py4J and YARN executors; the MI355X design is:

* ``Session(conf)`` with ``spark.executor.instances = N > 1`` (outside an SPMD launch)
  becomes a :class:`DriverSession`: the GUI / script process never touches a GPU; it
  ``spawn``-s N fresh worker processes (never ``exec``), worker r owns ``cuda:r`` and
  joins an N-rank RCCL group over xGMI (gloo on CPU).  Each worker holds an ordinary SPMD
  :class:`~orange3_spark_amd.session.Session` and 1/N of every DataFrame's rows.
* Every driver-side call is a **command** broadcast to all workers over a pipe; the
  workers execute it in lock step (so collectives inside line up) and rank 0 returns the
  result.  Results that are engine objects (DataFrames, column expressions, grouped data,
  readers, catalogs, RDDs, training summaries, ...) stay on the workers and come back as
  handles (:class:`RemoteObject` / :class:`RemoteDataFrame`, ``isinstance(h, DataFrame)``
  holds); plain values (counts, rows, pandas frames, fitted models with their host
  parameters) come back by value, device tensors moved to host memory.
* Estimator / Transformer / Evaluator calls on a handle ship the (pickled) stage to the
  workers (``ml/base.py`` hooks), so a fitted model arrives in the driver as a normal local
  model object -- widgets, ``model.coefficients`` and ``model.save`` work unchanged.
* ``createDataFrame(pandas)`` scatters: worker r receives only its row slice (host memory
  per worker ~ 1/N of the table) and copies it to its GPU through pinned memory.
* Handles are reference counted: when the driver drops the last handle, the workers free
  the object at the next command.  A command that fails on some ranks while others are
  stuck in a collective tears the pool down after a grace period instead of hanging the
  GUI; a rank that never answers after its peers did (``stragglerTimeout``) or a command
  that outlives the watchdog (``o3s.executor.timeout``) does the same.
* **Executor-resident models** (Spark keeps ALS factors as distributed DataFrames, reached
  through spark_ml_estimator.py:22 and spark_ml_model.py:53): a fitted model whose device
  state exceeds ``o3s.executor.residentModelBytes`` (16 MiB) stays on the executors and the
  driver receives a :class:`RemoteModel` -- ``isinstance(h, ALSModel)`` holds, it carries
  only the class and uid, and ``transform`` / ``recommendFor*`` / ``userFactors`` /
  ``save`` run on the executors (no factor byte crosses the driver pipes).  Small models
  (LR, SVC, KMeans, trees) still travel by value.
* **Lineage recovery** (Spark recomputes lost partitions from lineage): every handle
  remembers the command that produced it (a *recipe*: the pickled command plus the
  recipes of the handles it used).  When an executor dies the pool is torn down; the next
  call on any handle respawns a fresh pool (new subprocesses, never a re-exec) and
  replays the handle's recipe from its sources -- catalog tables, parquet readers,
  synthetic generators, ``createDataFrame`` from the driver-held host frame.  Temp-view
  registrations are replayed too.  A handle whose lineage is not replayable raises
  :class:`ExecutorLost` asking to re-run the upstream widgets.
"""
from __future__ import annotations

import io
import itertools
import logging
import os
import pickle
import socket
import threading
import time
import traceback
import weakref

log = logging.getLogger(__name__)

_REMOTE_MODULES = ("orange3_spark_amd.frame", "orange3_spark_amd.sql", "orange3_spark_amd.rdd",
                   "orange3_spark_amd.catalog", "orange3_spark_amd.io", "orange3_spark_amd.session",
                   "orange3_spark_amd.synthetic", "orange3_spark_amd.ml._summary")
_VALUE_MODULES = ("orange3_spark_amd.frame.types",)


class ExecutorError(RuntimeError):
    """A command failed on one or more executors (carries each failing rank's traceback)."""


class ExecutorLost(ExecutorError):
    """An executor died or a command did not finish on every rank: the pool is torn down."""


def _is_remote_kept(obj) -> bool:
    """Engine objects that stay on the workers (handles) rather than travel by value."""
    t = type(obj)
    mod = getattr(t, "__module__", "") or ""
    if not mod.startswith(_REMOTE_MODULES) or mod.startswith(_VALUE_MODULES):
        return False
    return not isinstance(obj, tuple)          # Row (a tuple subclass) travels by value


RESIDENT_MODEL_BYTES = 16 << 20               # default of o3s.executor.residentModelBytes


def _model_candidate(obj) -> bool:
    """A fitted model that may stay on the executors (PipelineModels never do: their large
    stages are kept one by one, the pipeline itself travels by value)."""
    mod = getattr(type(obj), "__module__", "") or ""
    if not mod.startswith("orange3_spark_amd.ml"):
        return False
    from ..ml.base import Model, PipelineModel
    return isinstance(obj, Model) and not isinstance(obj, PipelineModel)


def payload_bytes(obj, depth: int = 0, seen=None) -> int:
    """Bytes of array state (torch tensors, numpy arrays) reachable from ``obj`` through
    attributes, containers and engine dataclasses (depth-bounded)."""
    import numpy as np
    import torch
    if seen is None:
        seen = set()
    if id(obj) in seen or depth > 6:
        return 0
    seen.add(id(obj))
    if isinstance(obj, torch.Tensor):
        return obj.numel() * obj.element_size()
    if isinstance(obj, np.ndarray):
        return int(obj.nbytes)
    if isinstance(obj, (str, bytes, int, float, bool, type(None))):
        return 0
    if isinstance(obj, dict):
        return sum(payload_bytes(v, depth + 1, seen) for v in list(obj.values())[:4096])
    if isinstance(obj, (list, tuple, set, frozenset)):
        return sum(payload_bytes(v, depth + 1, seen) for v in list(obj)[:4096])
    mod = getattr(type(obj), "__module__", "") or ""
    if mod.startswith("orange3_spark_amd") and hasattr(obj, "__dict__"):
        return sum(payload_bytes(v, depth + 1, seen) for k, v in vars(obj).items() if k != "parent")
    return 0


def _resident_decision(session, obj) -> bool:
    """Keep ``obj`` on the executors?  The largest payload over the ranks decides, so every
    rank takes the same branch (the handle ids the ranks assign must stay in step)."""
    limit = float(session.conf.get("o3s.executor.residentModelBytes", str(RESIDENT_MODEL_BYTES)))
    nb = float(payload_bytes(obj))
    comm = session.comm
    if comm.world_size > 1:
        nb = float(comm.max_scalar(nb))
    return nb > limit


def _model_meta(obj) -> dict:
    t = type(obj)
    return {"cls": (t.__module__, t.__qualname__), "uid": getattr(obj, "uid", None)}


# =====================================================================================
# worker side
# =====================================================================================
class _Null:
    """Sink for the pickles of ranks != 0 (they only register objects): protocol 5 may
    hand large buffers over as PickleBuffer objects, which have no len()."""

    def write(self, b):
        return memoryview(b).nbytes


def _worker_pickler(objs: dict, ids: dict, counter, buf, session=None):
    """Pickler that keeps engine objects on this worker (registered under the next id of a
    counter every rank advances identically) and moves device tensors to host memory.
    Fitted models above the resident threshold are kept too (``kind`` "model")."""
    import cloudpickle
    import torch
    decided: dict = {}

    class P(cloudpickle.Pickler):
        def persistent_id(self, obj):
            k = ids.get(id(obj))
            known = k is not None and objs.get(k) is obj
            kind = None
            if _is_remote_kept(obj):
                kind = "frame" if _is_frame(obj) else "obj"
            elif _model_candidate(obj):
                if known:
                    kind = "model"
                elif session is not None:
                    keep = decided.get(id(obj))
                    if keep is None:
                        keep = decided[id(obj)] = _resident_decision(session, obj)
                    kind = "model" if keep else None
            if kind is None:
                return None
            if not known:
                k = next(counter)
                objs[k] = obj
                ids[id(obj)] = k
            return ("ref", k, type(obj).__name__, kind, _model_meta(obj) if kind == "model" else None)

        def reducer_override(self, obj):
            if isinstance(obj, torch.Tensor) and obj.device.type != "cpu":
                return obj.detach().cpu().__reduce_ex__(pickle.HIGHEST_PROTOCOL)
            if isinstance(obj, torch.device) and obj.type != "cpu":
                return (torch.device, ("cpu",))
            return super().reducer_override(obj)
    return P(buf, protocol=pickle.HIGHEST_PROTOCOL)


def _is_frame(obj) -> bool:
    from ..frame.dataframe import DataFrame
    return isinstance(obj, DataFrame)


def _worker_unpickler(objs: dict, data: bytes, slots=()):
    """Commands name executor objects by slot: ``("slot", i)`` is ``objs[slots[i]]`` (the
    slot table travels in the message header, so a recorded command can be replayed
    against the object ids of a respawned pool)."""
    class U(pickle.Unpickler):
        def persistent_load(self, pid):
            return objs[slots[pid[1]]] if pid[0] == "slot" else objs[pid[1]]
    return U(io.BytesIO(data)).load()


def _worker_entry(argv=None) -> int:
    """``python -m orange3_spark_amd.runtime.executors --connect HOST:PORT --rank R ...``:
    an executor process.  Started with subprocess (a fresh interpreter: the driver's main
    module is never re-imported, the driver never forks a process holding GPU state);
    authenticates to the driver's listener, receives the session conf, serves commands."""
    import argparse
    from multiprocessing.connection import Client
    ap = argparse.ArgumentParser()
    ap.add_argument("--connect", required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--dist-port", type=int, required=True)
    ap.add_argument("--gpu", type=int, default=1)
    ap.add_argument("--gloo", type=int, default=0)
    a = ap.parse_args(argv)
    host, port = a.connect.rsplit(":", 1)
    key = bytes.fromhex(os.environ.pop("O3S_EXECUTOR_AUTHKEY"))
    conn = Client((host, int(port)), authkey=key)
    conn.send_bytes(pickle.dumps(("hello", a.rank)))
    conf_pairs = pickle.loads(conn.recv_bytes())
    _worker_main(a.rank, a.world, a.dist_port, conf_pairs, conn, bool(a.gpu), bool(a.gloo))
    return 0


def _worker_main(rank: int, world: int, port: int, conf_pairs, conn, use_gpu: bool, gloo: bool):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if gloo:
        os.environ["O3S_DIST_BACKEND"] = "gloo"
    if not use_gpu:
        os.environ["HIP_VISIBLE_DEVICES"] = ""
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
    try:
        from ..conf import SessionConf
        from ..session import Session
        conf = SessionConf(False, conf_pairs).set("spark.master", "spmd")
        if not use_gpu:
            conf.set("o3s.device", "cpu")
        s = Session(conf)
        Session._active = s
        s._warmup(pool_worker=True)           # every family, before the first fit (runtime/warmup.py)
    except BaseException:  # noqa: BLE001 - reported to the driver
        conn.send_bytes(pickle.dumps(("error", rank, traceback.format_exc())))
        return
    conn.send_bytes(pickle.dumps(("ready", rank, str(s.device))))
    objs: dict = {0: s}
    ids: dict = {id(s): 0}
    counter = itertools.count(1)
    while True:
        try:
            msg = conn.recv_bytes()
        except (EOFError, OSError):
            break
        if msg == _CANCEL:                    # a cancel that arrived after its fit finished
            continue
        try:
            garbage, slots = pickle.loads(msg[8:_hdr_len(msg)])
        except Exception:  # noqa: BLE001
            garbage, slots = [], ()
        for k in garbage:
            o = objs.pop(k, None)
            if o is not None and ids.get(id(o)) == k:
                ids.pop(id(o), None)
        body = msg[_hdr_len(msg):]
        try:
            cmd = _worker_unpickler(objs, body, slots)
            kind = cmd[0]
            if kind == "stop":
                conn.send_bytes(pickle.dumps(("ok", rank, None)))
                break
            if kind == "watched":             # ("watched", inner, want_progress, want_cancel)
                with _watch_scope(s, conn, rank, cmd[2], cmd[3]):
                    result = _execute(s, cmd[1], objs)
            else:
                result = _execute(s, cmd, objs)
            buf = io.BytesIO() if rank == 0 else _Null()
            _worker_pickler(objs, ids, counter, buf, s).dump(result)
            conn.send_bytes(pickle.dumps(("ok", rank, buf.getvalue() if rank == 0 else None)))
        except BaseException as e:  # noqa: BLE001 - every failure goes back to the driver
            from .progress import FitCancelled
            st = "cancelled" if isinstance(e, FitCancelled) else "error"
            conn.send_bytes(pickle.dumps((st, rank, traceback.format_exc())))
    try:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass


# driver -> executors side message: stop the running fit (see _watch_scope)
_CANCEL = b"\xff" * 8 + b"o3s-cancel"


def _watch_scope(s, conn, rank: int, want_progress: bool, want_cancel: bool):
    """Progress / cancel scope of a fit shipped from the driver (``ExecutorPool.fit``).

    Rank 0 relays every percentage to the driver as a ``("progress", 0, p)`` side message
    (the driver forwards it into the calling thread's sink).  For cancellation each rank
    polls its pipe for :data:`_CANCEL` at every report site and the ranks OR their flags
    with one host collective (``Comm.any_flag``), so all of them raise ``FitCancelled`` at
    the same iteration -- a rank that stopped alone would leave its peers waiting in the
    next all-reduce.  Report sites run in lock step on every rank (SPMD loops), so the
    collective lines up."""
    from . import progress as P
    seen = [False]

    def relay(p):
        if rank == 0 and want_progress:
            conn.send_bytes(pickle.dumps(("progress", 0, float(p))))

    def cancelled():
        if not seen[0]:
            while conn.poll(0):
                if conn.recv_bytes() == _CANCEL:
                    seen[0] = True
        return s.comm.any_flag(seen[0])
    return P.progress_scope(relay, cancelled if want_cancel else None)


def _hdr_len(msg: bytes) -> int:
    return 8 + int.from_bytes(msg[:8], "little")


def _execute(s, cmd, objs=None):
    kind = cmd[0]
    if kind == "getattr":
        _, target, name = cmd
        v = getattr(target, name)
        if callable(v) and not isinstance(v, type) and hasattr(v, "__self__") and not _is_remote_kept(v):
            return _BoundMethod(name)
        return v
    if kind == "call":
        _, target, name, args, kwargs = cmd
        return getattr(target, name)(*args, **kwargs)
    if kind == "apply":                       # fn(*args, **kwargs) with a shipped callable
        _, fn, args, kwargs = cmd
        return fn(*args, **kwargs)
    if kind == "scatter_df":
        _, part, schema = cmd
        return s.createDataFrame(part, schema, _local=True)
    if kind == "info":
        import torch
        return {"device": str(s.device), "backend": s.comm.backend, "world": s.comm.world_size,
                "gpu": torch.cuda.get_device_name(s.device) if s.device.type == "cuda" else None,
                "objects": len(objs) if objs is not None else None}
    raise ValueError(f"unknown executor command {kind!r}")


class _BoundMethod:
    """Marker: the attribute is a method of the remote object (call it through the pool)."""

    def __init__(self, name):
        self.name = name


# =====================================================================================
# driver side
# =====================================================================================
def _free_port() -> int:
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    p = sk.getsockname()[1]
    sk.close()
    return p


class _Proc:
    """subprocess.Popen with the multiprocessing.Process surface the pool uses."""

    def __init__(self, popen):
        self.p = popen

    def is_alive(self) -> bool:
        return self.p.poll() is None

    @property
    def exitcode(self):
        return self.p.poll()

    def terminate(self):
        if self.is_alive():
            self.p.terminate()

    def kill(self):
        if self.is_alive():
            self.p.kill()

    def join(self, timeout=None):
        import subprocess
        try:
            self.p.wait(timeout)
        except subprocess.TimeoutExpired:
            pass


class _Recipe:
    """How a handle was produced (its lineage): replayed on a respawned pool.

    ``kind``: "session" (the executor session, id 0), "cmd" (``body`` = the pickled command
    whose executor objects are named by slot, ``slots`` = the recipes of those objects) or
    "scatter" (``body`` = (host pandas frame, schema) of a createDataFrame).  ``index``
    picks the handle among the command result's handles (unpickle order)."""

    __slots__ = ("kind", "body", "slots", "index", "_replayed", "__weakref__")

    def __init__(self, kind, body=None, slots=(), index=0):
        self.kind, self.body, self.slots, self.index = kind, body, tuple(slots), index
        self._replayed = None

    def at(self, index: int) -> "_Recipe":
        r = _Recipe(self.kind, self.body, self.slots, index)
        r._replayed = _Shared(self)
        return r


class _Shared:
    """Sibling recipes (several handles out of one command) share one replay."""

    __slots__ = ("root",)

    def __init__(self, root):
        self.root = root


_SESSION_RECIPE = _Recipe("session")
# calls whose effect lives in the executors' session state (replayed after a respawn)
_EFFECTS = frozenset(("createOrReplaceTempView", "createTempView", "createGlobalTempView",
                      "createOrReplaceGlobalTempView", "registerTempTable", "dropTempView",
                      "dropGlobalTempView", "setCheckpointDir", "setCurrentDatabase", "register"))


class ExecutorPool:
    """N worker processes in one RCCL (or gloo) group, driven by this process."""

    _pools: "weakref.WeakSet[ExecutorPool]" = weakref.WeakSet()

    def __init__(self, n: int, conf_pairs, use_gpu: bool | None = None, start_timeout: float = 600.0,
                 command_timeout: float | None = None, error_grace: float = 20.0,
                 straggler_timeout: float | None = None):
        import secrets
        import subprocess
        import sys
        from multiprocessing.connection import Listener
        import torch
        self.n = int(n)
        if self.n < 1:
            raise ValueError("an executor pool needs at least one executor")
        pairs = list(conf_pairs)
        dev_pref = dict(pairs).get("o3s.device", "auto").lower()
        ngpu = torch.cuda.device_count()          # counting does not initialise HIP here
        if use_gpu is None:
            use_gpu = dev_pref != "cpu" and ngpu > 0
        gloo = os.environ.get("O3S_DIST_BACKEND") == "gloo"
        if use_gpu and ngpu < self.n and not gloo:
            raise RuntimeError(f"spark.executor.instances={self.n} needs {self.n} GPUs, {ngpu} visible "
                               "(O3S_DIST_BACKEND=gloo shares GPUs between executors for testing)")
        self.use_gpu = bool(use_gpu)
        self.command_timeout = command_timeout
        self.error_grace = float(error_grace)
        self.straggler_timeout = straggler_timeout
        self._lock = threading.RLock()
        self._garbage: list = []
        self._proxies: dict = {}
        self._methods: set = set()
        self._watch = None                        # progress / cancel relay of a running fit
        self.alive = False
        self.lost_reason: str | None = None
        self._successor: "ExecutorPool | None" = None
        self._respawn = None                      # set by DriverSession: () -> new pool
        self.effects: list = []                   # replayable session-state commands
        self.bytes_sent = 0                       # command bytes driver -> executors (all ranks)
        self.bytes_received = 0                   # reply bytes executors -> driver
        self._conns, self._procs = [None] * self.n, []
        key = secrets.token_bytes(32)
        listener = Listener(("127.0.0.1", 0), authkey=key)
        host, lport = listener.address
        dist_port = _free_port()
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        # executors import what the driver can import (its sys.path: user modules whose
        # functions / classes are shipped by reference, like Spark's --py-files)
        paths = [root] + [p for p in sys.path if p and os.path.isdir(p)]
        paths += [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p]
        env = dict(os.environ, O3S_EXECUTOR_AUTHKEY=key.hex(), HSA_ENABLE_IPC_MODE_LEGACY="0",
                   PYTHONPATH=os.pathsep.join(dict.fromkeys(paths)))
        env.pop("WORLD_SIZE", None)
        for r in range(self.n):
            cmd = [sys.executable, "-m", "orange3_spark_amd.runtime.executors", "--connect", f"{host}:{lport}",
                   "--rank", str(r), "--world", str(self.n), "--dist-port", str(dist_port),
                   "--gpu", str(int(self.use_gpu)), "--gloo", str(int(gloo))]
            self._procs.append(_Proc(subprocess.Popen(cmd, env=env)))
        try:
            self._accept(listener, pairs, start_timeout)
        finally:
            listener.close()
        self.devices = [None] * self.n
        replies = self._gather(start_timeout, what="start")
        errs = [(r, d) for st, r, d in replies if st != "ready"]
        if errs:
            self._teardown()
            raise ExecutorLost("executor start failed:\n" + "\n".join(f"[rank {r}] {d}" for r, d in errs))
        for _, r, dev in replies:
            self.devices[r] = dev
        self.alive = True
        ExecutorPool._pools.add(self)

    @property
    def pids(self) -> list:
        return [p.p.pid for p in self._procs]

    def _accept(self, listener, pairs, timeout: float):
        """Accept the N executors' authenticated connections (in a helper thread, so a
        worker that dies before connecting is noticed) and send each the session conf."""
        got: list = []
        err: list = []

        def run():
            try:
                for _ in range(self.n):
                    c = listener.accept()
                    hello = pickle.loads(c.recv_bytes())
                    got.append((hello[1], c))
            except Exception as e:  # noqa: BLE001
                err.append(e)
        th = threading.Thread(target=run, daemon=True)
        th.start()
        deadline = time.monotonic() + timeout
        while th.is_alive():
            th.join(0.2)
            dead = [r for r, p in enumerate(self._procs) if not p.is_alive()]
            if dead or time.monotonic() > deadline:
                self._teardown()
                raise ExecutorLost(f"executor(s) {dead or 'all'} failed to connect "
                                   f"(exit codes {[self._procs[r].exitcode for r in dead]})")
        if err or len(got) != self.n:
            self._teardown()
            raise ExecutorLost(f"executor handshake failed: {err}")
        for r, c in got:
            self._conns[r] = c
            c.send_bytes(pickle.dumps(pairs))

    # ---------------------------------------------------------------- transport
    def _lost(self, msg: str):
        self.lost_reason = msg
        self._teardown()
        return ExecutorLost(msg)

    def _gather(self, timeout: float | None, what: str):
        """One reply per rank.  After the first error, the others get ``error_grace``
        seconds; after the first success, ``straggler_timeout`` (ranks of one command run
        in lock step: a rank still busy long after its peers finished is wedged).  Ranks
        that neither reply nor die in time mean the group is wedged (e.g. a collective
        waiting for a failed peer): the pool is torn down."""
        from multiprocessing.connection import wait
        pending = dict(enumerate(self._conns))
        out, first_err, first_ok = [], None, None
        deadline = None if timeout is None else time.monotonic() + timeout
        watch = self._watch
        while pending:
            if watch is not None and watch["cancel"] is not None and not watch["sent"] and watch["cancel"]():
                watch["sent"] = True              # every rank sees it at its next report site
                for c in self._conns:
                    try:
                        c.send_bytes(_CANCEL)
                    except (BrokenPipeError, OSError):
                        pass
            now = time.monotonic()
            limit = deadline
            if first_err is not None:
                g = first_err + self.error_grace
                limit = g if limit is None else min(limit, g)
            if first_ok is not None and self.straggler_timeout is not None:
                g = first_ok + self.straggler_timeout
                limit = g if limit is None else min(limit, g)
            if limit is not None and now > limit:
                why = "watchdog" if limit == deadline else ("error grace" if first_err is not None else "straggler")
                raise self._lost(f"executors {sorted(pending)} did not finish '{what}' ({why} timeout)"
                                 + (f"; errors: {self._fmt(out)}" if out else "") + " -- the pool was shut down")
            tick = 0.05 if watch is not None and watch["cancel"] is not None and not watch["sent"] else 1.0
            ready = wait(list(pending.values()), timeout=tick if limit is None else max(0.01, min(tick, limit - now)))
            for c in ready:
                r = next(k for k, v in pending.items() if v is c)
                try:
                    raw = c.recv_bytes()
                except (EOFError, OSError):
                    raise self._lost(f"executor {r} died during '{what}' (exit code "
                                     f"{self._procs[r].exitcode})") from None
                self.bytes_received += len(raw)
                msg = pickle.loads(raw)
                if msg[0] == "progress":          # side message of a watched fit (rank 0)
                    if watch is not None:
                        watch["progress"](msg[2])
                    continue
                pending.pop(r)
                out.append(msg)
                if msg[0] in ("error", "cancelled") and first_err is None:
                    first_err = time.monotonic()
                elif msg[0] not in ("error", "cancelled") and first_ok is None:
                    first_ok = time.monotonic()
            for r in list(pending):
                if not self._procs[r].is_alive():
                    raise self._lost(f"executor {r} exited with code {self._procs[r].exitcode} during '{what}'")
        return out

    @staticmethod
    def _fmt(replies):
        return "\n".join(f"[rank {r}] {d}" for st, r, d in replies if st in ("error", "cancelled"))

    def _driver_pickle(self, cmd):
        """Pickle ``cmd`` naming every handle by slot; returns (bytes, [handles by slot]).
        A handle of a dead pool is first rebuilt here from its recipe (lineage replay)."""
        import cloudpickle
        pool = self
        slots: list = []
        pos: dict = {}

        class P(cloudpickle.Pickler):
            def persistent_id(self, obj):
                if isinstance(obj, RemoteObject):
                    if obj._pool is not pool:
                        pool._adopt(obj)
                    i = pos.get(id(obj))
                    if i is None:
                        i = pos[id(obj)] = len(slots)
                        slots.append(obj)
                    return ("slot", i)
                return None
        buf = io.BytesIO()
        P(buf, protocol=pickle.HIGHEST_PROTOCOL).dump(cmd)
        return buf.getvalue(), slots

    def _driver_unpickle(self, data: bytes, recipe: "_Recipe | None", found: list | None = None):
        pool = self
        seq = itertools.count()

        class U(pickle.Unpickler):
            def persistent_load(self, pid):
                _, k, tname, kind, meta = pid
                i = next(seq)
                h = pool._proxy(k, tname, kind, meta, None if recipe is None else recipe.at(i))
                if found is not None:
                    found.append(h)
                return h
        return U(io.BytesIO(data)).load()

    def _proxy(self, k, tname, kind, meta=None, recipe=None):
        ref = self._proxies.get(k)
        obj = ref() if ref is not None else None
        if obj is None:
            if kind == "model":
                obj = RemoteModel(self, k, tname, meta)
            else:
                obj = (RemoteDataFrame if kind in ("frame", True) else RemoteObject)(self, k, tname)
            object.__setattr__(obj, "_recipe", recipe)
            self._proxies[k] = weakref.ref(obj)
            object.__setattr__(obj, "_fin", weakref.finalize(obj, self._release, k))
        return obj

    def _release(self, k):
        self._garbage.append(k)

    def _send_all(self, bodies, slot_ids):
        garbage, self._garbage = self._garbage, []
        for k in garbage:
            self._proxies.pop(k, None)
        hdr = pickle.dumps((garbage, slot_ids))
        head = len(hdr).to_bytes(8, "little") + hdr
        for r, c in enumerate(self._conns):
            msg = head + bodies[r]
            try:
                c.send_bytes(msg)
            except (BrokenPipeError, OSError):
                raise self._lost(f"executor {r} is gone") from None
            self.bytes_sent += len(msg)

    def _run(self, bodies, slot_ids, what, recipe, found=None):
        self._send_all(bodies, slot_ids)
        replies = self._gather(self.command_timeout, what)
        if replies and all(m[0] == "cancelled" for m in replies):
            from .progress import FitCancelled
            raise FitCancelled(f"{what} cancelled on all {self.n} executors")
        errs = [m for m in replies if m[0] != "ok"]
        if errs:
            raise ExecutorError("command failed on executor(s):\n" + self._fmt(replies))
        data = next(d for st, r, d in replies if r == 0)
        return self._driver_unpickle(data, recipe, found)

    def command(self, cmd, per_rank=None, what: str | None = None, recipe: "_Recipe | None" = None):
        """Run ``cmd`` on every executor (``per_rank[r]`` replaces it on rank r) and return
        rank 0's result.  On a dead pool the call moves to its respawned successor."""
        with self._lock:
            if self.alive:
                dead = [r for r, p in enumerate(self._procs) if not p.is_alive()]
                if dead:                          # lost between commands (killed, crashed)
                    self._lost(f"executor(s) {dead} exited (codes {[self._procs[r].exitcode for r in dead]})")
            if not self.alive:
                return self._revive().command(cmd, per_rank, what, recipe)
            what = what or str((cmd or per_rank[0])[0])
            if per_rank is None:
                body, slots = self._driver_pickle(cmd)
                bodies = [body] * self.n
                if recipe is None:
                    recipe = self._recipe_of(body, slots)
                    if recipe is not None and cmd[0] == "call" and cmd[2] in _EFFECTS:
                        self.effects.append(recipe)
            else:
                packed = [self._driver_pickle(c) for c in per_rank]
                bodies = [b for b, _ in packed]
                slots = packed[0][1]
                if any(sl != slots for _, sl in packed):
                    raise ValueError("per-rank commands must name the same handles")
            return self._run(bodies, [h._id for h in slots], what, recipe)

    @staticmethod
    def _recipe_of(body, slots):
        subs = []
        for h in slots:
            r = h._recipe
            if r is None:
                return None
            subs.append(r)
        return _Recipe("cmd", body, subs)

    # ---------------------------------------------------------------- lineage recovery
    def _revive(self) -> "ExecutorPool":
        """The live pool that replaces this dead one (respawning it if needed)."""
        p = self
        while not p.alive and p._successor is not None:
            p = p._successor
        if p.alive:
            return p
        if p._respawn is None:
            raise ExecutorLost("the executor pool is shut down"
                               + (f" ({p.lost_reason})" if p.lost_reason else ""))
        new = p._respawn(p)
        p._successor = new
        return new

    def _adopt(self, h: "RemoteObject") -> None:
        """Rebind handle ``h`` (of a dead predecessor pool) to an object of this pool,
        rebuilt by replaying its recipe."""
        old = h._pool
        q = old
        while q is not None and q is not self:
            q = q._successor
        if q is None:
            raise ValueError("a handle of another executor pool cannot be used here")
        if h._recipe is None:
            raise ExecutorLost(f"{h._tname} #{h._id} was lost with its executors and its lineage cannot be "
                               "replayed (it was not built from a table, file, generator or driver data): "
                               "re-run the upstream widgets")
        fresh = self._replay(h._recipe)
        fresh._fin.detach()
        object.__setattr__(h, "_pool", self)
        object.__setattr__(h, "_id", fresh._id)
        self._proxies[fresh._id] = weakref.ref(h)
        object.__setattr__(h, "_fin", weakref.finalize(h, self._release, fresh._id))

    def _replay(self, rec: "_Recipe") -> "RemoteObject":
        if rec.kind == "session":
            return self._proxy(0, "Session", "obj", None, _SESSION_RECIPE)
        root = rec._replayed.root if isinstance(rec._replayed, _Shared) else rec
        got = root._replayed if not isinstance(root._replayed, _Shared) else None
        # the cache holds executor ids only (no proxies): a replayed object that no live
        # handle holds is released like any other, and an id is reused only while a live
        # proxy of THIS pool still names it (an adopting handle takes over the id)
        if got is not None and got[0]() is self and rec.index < len(got[1]):
            live = self._live_proxy(got[1][rec.index])
            if live is not None:
                return live
        found: list = []
        if root.kind == "scatter":
            pdf, schema = root.body
            found.append(self.scatter_dataframe(pdf, schema))
        else:
            handles = [self._replay(r) for r in root.slots]
            self._run([root.body] * self.n, [h._id for h in handles], "replay", root, found)
            del handles
        root._replayed = (weakref.ref(self), [h._id for h in found])
        if rec.index >= len(found):
            raise ExecutorLost("lineage replay produced a different result shape")
        return found[rec.index]

    def _live_proxy(self, k):
        """The live proxy naming executor object ``k`` of this pool, or None if it was
        released (or is queued for release)."""
        ref = self._proxies.get(k)
        obj = ref() if ref is not None else None
        if obj is None or k in self._garbage or getattr(obj, "_id", None) != k:
            return None
        return obj

    def replay_effects(self, effects) -> None:
        for rec in effects:
            try:
                handles = [self._replay(r) for r in rec.slots]
                self._run([rec.body] * self.n, [h._id for h in handles], "replay effect", None)
                self.effects.append(rec)
            except (ExecutorError, ExecutorLost) as e:
                log.warning("could not replay a session effect after respawn: %s", e)

    # ---------------------------------------------------------------- API used by proxies
    def getattr(self, obj: "RemoteObject", name: str):
        key = (obj._tname, name)
        if key in self._methods:                 # known method: no round trip until it is called
            return RemoteMethod(obj, name)
        v = self.command(("getattr", obj, name), what=f"{obj._tname}.{name}")
        if isinstance(v, _BoundMethod):
            self._methods.add(key)
            return RemoteMethod(obj, name)
        return v

    def call(self, obj, name: str, args=(), kwargs=None):
        return self.command(("call", obj, name, tuple(args), dict(kwargs or {})),
                            what=f"{getattr(obj, '_tname', type(obj).__name__)}.{name}")

    def apply(self, fn, *args, **kwargs):
        return self.command(("apply", fn, args, kwargs), what=getattr(fn, "__name__", "apply"))

    def apply_watched(self, fn, *args, **kwargs):
        """``apply`` for a fit, relaying the calling thread's progress sink and cancel
        request (runtime/progress.py) to the executors: rank 0's percentages come back as
        side messages while the command runs, and a cancel makes every rank raise
        ``FitCancelled`` at the same iteration -- the pool stays usable."""
        from . import progress as P
        want_p, want_c = P.watching()
        if not (want_p or want_c):
            return self.apply(fn, *args, **kwargs)
        with self._lock:
            pool = self._revive()                 # a respawned successor runs it if this one died
            pool._watch = {"progress": P.forward, "cancel": P.cancel_requested if want_c else None, "sent": False}
            try:
                return pool.command(("watched", ("apply", fn, args, kwargs), want_p, want_c),
                                    what=getattr(fn, "__name__", "apply"))
            finally:
                pool._watch = None

    def scatter_dataframe(self, pdf, schema=None):
        """Row slice r of a host pandas frame -> executor r (only that slice is sent).  The
        driver keeps a reference to the host frame as the handle's lineage (Spark's
        ``parallelize`` keeps its local collection the same way)."""
        n = len(pdf)
        parts = [pdf.iloc[(n * r) // self.n:(n * (r + 1)) // self.n] for r in range(self.n)]
        return self.command(None, per_rank=[("scatter_df", p, schema) for p in parts], what="createDataFrame",
                            recipe=_Recipe("scatter", (pdf, schema)))

    def info(self):
        return self.command(("info",))

    # ---------------------------------------------------------------- lifecycle
    def shutdown(self, timeout: float = 30.0):
        with self._lock:
            self._respawn = None
            if not self.alive:
                return
            self.alive = False
            hdr = pickle.dumps(([], ()))
            for c in self._conns:
                try:
                    c.send_bytes(len(hdr).to_bytes(8, "little") + hdr + pickle.dumps(("stop",)))
                except (BrokenPipeError, OSError):
                    pass
            for p in self._procs:
                p.join(timeout)
            self._teardown()

    def _teardown(self):
        self.alive = False
        for p in self._procs:
            if p.is_alive():
                p.terminate()
        for p in self._procs:
            p.join(10)
            if p.is_alive():
                p.kill()
                p.join(5)
        for c in self._conns:
            try:
                if c is not None:
                    c.close()
            except OSError:
                pass

    def __del__(self):
        try:
            self._teardown()
        except Exception:  # noqa: BLE001
            pass


def _shutdown_all():
    for p in list(ExecutorPool._pools):
        try:
            p.shutdown(timeout=10)
        except Exception:  # noqa: BLE001
            pass


import atexit  # noqa: E402

atexit.register(_shutdown_all)


# =====================================================================================
# handles
# =====================================================================================
_BINOPS = ("__add__", "__radd__", "__sub__", "__rsub__", "__mul__", "__rmul__", "__truediv__", "__rtruediv__",
           "__floordiv__", "__mod__", "__rmod__", "__pow__", "__rpow__", "__lt__", "__le__", "__gt__", "__ge__",
           "__and__", "__rand__", "__or__", "__ror__", "__eq__", "__ne__", "__getitem__", "__contains__")
_UNOPS = ("__neg__", "__invert__", "__abs__")


class RemoteObject:
    """Driver-side handle of an object that lives on every executor (same id on each).
    ``_recipe`` is its lineage (how to rebuild it on a respawned pool), ``_fin`` the
    finaliser that frees the executor object when the handle dies."""

    __slots__ = ("_pool", "_id", "_tname", "_recipe", "_fin", "__weakref__")

    def __init__(self, pool: ExecutorPool, k: int, tname: str):
        object.__setattr__(self, "_pool", pool)
        object.__setattr__(self, "_id", k)
        object.__setattr__(self, "_tname", tname)
        object.__setattr__(self, "_recipe", None)
        object.__setattr__(self, "_fin", None)

    def __getattr__(self, name):
        if name.startswith("__") and name.endswith("__"):
            raise AttributeError(name)
        return self._pool.getattr(self, name)

    def __setattr__(self, name, value):
        self._pool.call(_Setattr(), "set", (self, name, value))

    def __call__(self, *args, **kwargs):
        return self._pool.call(self, "__call__", args, kwargs)

    def __repr__(self):
        return f"<remote {self._tname} #{self._id} on {self._pool.n} executors>"

    def __hash__(self):
        return hash((id(self._pool), self._id))

    def __bool__(self):
        return True

    def __iter__(self):
        return iter(self._pool.apply(_to_list, self))

    def __len__(self):
        return int(self._pool.apply(_global_len, self))

    def __reduce__(self):
        raise TypeError("executor handles cannot be pickled outside their pool")


def _make_op(name):
    def op(self, *args):
        return self._pool.call(self, name, args)
    op.__name__ = name
    return op


for _n in _BINOPS + _UNOPS:
    setattr(RemoteObject, _n, _make_op(_n))


class _Setattr:
    """Shipped helper: setattr on the executor-side object."""

    @staticmethod
    def set(obj, name, value):
        setattr(obj, name, value)


def _to_list(obj):
    return list(obj)


def _global_len(obj):
    cnt = getattr(obj, "count", None)
    if callable(cnt):
        try:
            v = cnt()
            if isinstance(v, int):
                return v
        except TypeError:
            pass
    return len(obj)


class RemoteMethod:
    __slots__ = ("_obj", "_name")

    def __init__(self, obj, name):
        self._obj, self._name = obj, name

    def __call__(self, *args, **kwargs):
        return self._obj._pool.call(self._obj, self._name, args, kwargs)

    def __repr__(self):
        return f"<remote method {self._obj._tname}.{self._name}>"


def _dataframe_class():
    from ..frame.dataframe import DataFrame
    return DataFrame


class RemoteDataFrame(RemoteObject):
    """Handle of a row-sharded DataFrame held by the executors.  ``isinstance(h, DataFrame)``
    is true (``__class__`` reports DataFrame) so widget channels typed DataFrame accept it;
    every DataFrame method runs on the executors."""

    __slots__ = ()

    @property
    def __class__(self):
        return _dataframe_class()

    @property
    def pool(self):
        return self._pool

    def __repr__(self):
        try:
            cols = self._pool.getattr(self, "columns")
        except Exception:  # noqa: BLE001
            cols = "?"
        return f"DataFrame[{cols}] (on {self._pool.n} executors)"


class RemoteModel(RemoteObject):
    """Handle of a fitted model held by the executors (its device state exceeded
    ``o3s.executor.residentModelBytes``).  ``isinstance(h, <ModelClass>)`` holds and ``uid``
    is local; every other attribute / method (``transform``, ``recommendForAllUsers``,
    ``userFactors``, params) runs on the executors.  ``save`` / ``write().save`` write from
    the executors: no model byte goes through the driver."""

    __slots__ = ("_cls", "uid")

    def __init__(self, pool: ExecutorPool, k: int, tname: str, meta: dict | None = None):
        super().__init__(pool, k, tname)
        meta = meta or {}
        cls = None
        if meta.get("cls"):
            import importlib
            mod, qual = meta["cls"]
            cls = importlib.import_module(mod)
            for part in qual.split("."):
                cls = getattr(cls, part)
        object.__setattr__(self, "_cls", cls)
        object.__setattr__(self, "uid", meta.get("uid"))

    @property
    def __class__(self):
        return self._cls or RemoteModel

    @property
    def pool(self):
        return self._pool

    def write(self):
        return _RemoteWriter(self)

    def save(self, path: str) -> None:
        self.write().save(path)

    def __repr__(self):
        return f"{self._tname}: uid={self.uid} (resident on {self._pool.n} executors)"


class _RemoteWriter:
    """``MLWriter`` of an executor-resident model: the ranks write (rank 0 the metadata and
    its data parts), the driver only sends the path."""

    def __init__(self, h):
        self._h, self._overwrite, self._opts = h, False, {}

    def overwrite(self):
        self._overwrite = True
        return self

    def option(self, k, v):
        self._opts[k] = v
        return self

    def session(self, s):
        return self

    def save(self, path: str) -> None:
        self._h._pool.apply(_exec_save, self._h, os.path.abspath(path), self._overwrite, self._opts)

    def saveImpl(self, path: str) -> None:
        self._h._pool.apply(_exec_save_impl, self._h, os.path.abspath(path))


def _exec_save(model, path, overwrite, opts):
    w = model.write()
    if overwrite:
        w.overwrite()
    for k, v in opts.items():
        w.option(k, v)
    w.save(path)


def _exec_save_impl(model, path):
    model.write().saveImpl(path)


_HANDLE_TYPES = (RemoteObject, RemoteDataFrame, RemoteModel)


def is_remote(obj) -> bool:
    return type(obj) in _HANDLE_TYPES


def remote_pool_of(*objs):
    """The executor pool of the first handle among ``objs`` (recursing into lists/dicts)."""
    for o in objs:
        if type(o) in _HANDLE_TYPES:
            return o._pool
        if isinstance(o, (list, tuple)):
            p = remote_pool_of(*o)
            if p is not None:
                return p
        if isinstance(o, dict):
            p = remote_pool_of(*o.values())
            if p is not None:
                return p
    return None


def ship(fn):
    """Decorator for free functions taking DataFrames (stat tests, correlation, ...): called
    with executor handles, the function itself runs on the executors."""
    import functools

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        pool = remote_pool_of(args, kwargs)
        if pool is not None:
            return pool.apply(fn, *args, **kwargs)
        return fn(*args, **kwargs)
    return wrapper


if __name__ == "__main__":
    # run the entry from the package module (not this __main__ copy), so every class the
    # executor pickles back (_BoundMethod, ...) is the driver's class
    import sys as _sys
    from orange3_spark_amd.runtime import executors as _executors
    _sys.exit(_executors._worker_entry())
