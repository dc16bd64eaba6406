"""Iteration checkpoints for the iterative estimators (SURVEY §5 "Checkpoint / resume").

Spark's ``checkpointInterval`` truncates RDD lineage; on one MI355X node the useful
equivalent is *resume*: every ``interval`` iterations an estimator persists its solver
state (centres, factor shards, coefficients, finished trees) under the session's
checkpoint directory (``spark.checkpoint.dir`` / ``SparkContext.setCheckpointDir``), and
a later ``fit`` of the same estimator configuration on the same data continues from
the last checkpoint instead of iteration 0 -- e.g. after a crashed or interrupted run.

Format (no pickle): ``<dir>/<key>/step-<n>/rank-<r>.npz`` (numpy arrays, loaded with
``allow_pickle=False``) + ``meta.json``; rank-sharded state (ALS factors) writes one file
per rank, replicated state is written by rank 0 only.  The key hashes the estimator
class, its params and a data fingerprint, so a changed configuration never resumes from
a stale state.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil

import numpy as np


def fingerprint(*parts) -> str:
    h = hashlib.sha1()
    for p in parts:
        h.update(repr(p).encode())
    return h.hexdigest()[:16]


def checkpoint_dir(session) -> str | None:
    if session is None:
        return None
    conf = getattr(session, "conf", None)
    d = conf.get("spark.checkpoint.dir", None) if conf is not None else None
    return d or None


class Checkpointer:
    """Save/restore solver state every ``interval`` iterations (no-op if disabled)."""

    def __init__(self, root: str | None, key: str, interval: int, comm, sharded: bool = False, keep: int = 1):
        self.root = os.path.join(root, key) if root else None
        self.interval = int(interval or 0)
        self.comm = comm
        self.sharded = sharded
        self.keep = keep

    @property
    def enabled(self) -> bool:
        return self.root is not None and self.interval > 0

    def due(self, step: int) -> bool:
        return self.enabled and step > 0 and step % self.interval == 0

    def _step_dir(self, step: int) -> str:
        return os.path.join(self.root, f"step-{step:08d}")

    def save(self, step: int, state: dict, meta: dict | None = None) -> None:
        if not self.enabled:
            return
        d = self._step_dir(step)
        rank = self.comm.rank if self.comm is not None else 0
        os.makedirs(d, exist_ok=True)
        if self.sharded or rank == 0:
            arrays = {k: np.asarray(v) for k, v in state.items()}
            tmp = os.path.join(d, f".rank-{rank}.tmp.npz")
            np.savez(tmp, **arrays)
            os.replace(tmp, os.path.join(d, f"rank-{rank}.npz"))
        if self.comm is not None:
            self.comm.barrier()
        if rank == 0:
            with open(os.path.join(d, "meta.json"), "w") as f:
                json.dump({"step": step, "world": self.comm.world_size if self.comm else 1,
                           "sharded": self.sharded, **(meta or {})}, f)
            self._prune(step)
        if self.comm is not None:
            self.comm.barrier()
        from .faults import INJECTOR
        INJECTOR.hit("checkpoint.saved")      # lets tests crash a fit right after a checkpoint

    def _prune(self, step: int) -> None:
        steps = sorted(int(n.split("-")[1]) for n in os.listdir(self.root) if n.startswith("step-"))
        for s in steps[:-self.keep]:
            shutil.rmtree(self._step_dir(s), ignore_errors=True)

    def latest(self) -> tuple[int, dict, dict] | None:
        """(step, state, meta) of the newest complete checkpoint, or None."""
        if not self.enabled or not os.path.isdir(self.root):
            return None
        rank = self.comm.rank if self.comm is not None else 0
        world = self.comm.world_size if self.comm is not None else 1
        for name in sorted((n for n in os.listdir(self.root) if n.startswith("step-")), reverse=True):
            d = os.path.join(self.root, name)
            mp = os.path.join(d, "meta.json")
            if not os.path.exists(mp):
                continue
            with open(mp) as f:
                meta = json.load(f)
            if meta.get("sharded") and meta.get("world") != world:
                continue                      # sharded state only resumes on the same world size
            fp = os.path.join(d, f"rank-{rank if meta.get('sharded') else 0}.npz")
            if not os.path.exists(fp):
                continue
            with np.load(fp, allow_pickle=False) as z:
                state = {k: z[k] for k in z.files}
            return int(meta["step"]), state, meta
        return None

    def clear(self) -> None:
        if self.enabled and (self.comm is None or self.comm.rank == 0):
            shutil.rmtree(self.root, ignore_errors=True)


def for_estimator(est, df, sharded: bool = False, extra=()) -> Checkpointer:
    """Checkpointer for ``est.fit(df)``: enabled when the session has a checkpoint dir and
    the estimator's ``checkpointInterval`` (or conf ``o3s.checkpoint.interval``) is > 0."""
    session = getattr(df, "session", None)
    root = checkpoint_dir(session)
    interval = 0
    if root:
        if est.hasParam("checkpointInterval") and est.isDefined(est.getParam("checkpointInterval")):
            interval = int(est.getOrDefault(est.getParam("checkpointInterval")))
        else:
            interval = int(session.conf.get("o3s.checkpoint.interval", "0") or 0)
    params = sorted((p.name, repr(v)) for p, v in est.extractParamMap().items()
                    if p.name not in ("checkpointInterval",))
    n = df.comm.sum_scalar(len(df)) if root else 0
    key = f"{type(est).__name__}-{fingerprint(type(est).__name__, params, n, extra)}"
    return Checkpointer(root, key, interval, df.comm, sharded=sharded)
