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
class, its params and a digest of every input column's rows (all ranks, in rank order),
so a changed configuration or changed data never resumes from a stale state, and a
completed fit clears its checkpoints.
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
        """Drop every checkpoint of this key: called once a fit has COMPLETED, so a later
        fit never resumes from a finished run's state."""
        if not self.enabled:
            return
        if self.comm is not None:
            self.comm.barrier()
        if self.comm is None or self.comm.rank == 0:
            shutil.rmtree(self.root, ignore_errors=True)
        if self.comm is not None:
            self.comm.barrier()


# --------------------------------------------------------------------------- data fingerprint
_FP_CHUNK = 1 << 26          # int32 words per device reduction chunk (int64 temporaries: 512 MB)


def _tensor_digest(t) -> tuple:
    """Order-sensitive digest of a tensor's bytes, computed where the tensor lives.

    The bytes are read as int32 words w_i and folded into two wrapping int64 sums,
    sum(w_i) and sum(w_i * m_i) with m_i an odd multiplicative hash of the word position,
    so a changed value or a permutation of rows changes the digest.  One streaming pass
    (chunked so the int64 temporaries stay bounded); only runs when checkpointing is on.
    """
    import torch
    if t is None:
        return ("none",)
    t = t.detach()
    if not t.is_contiguous():
        t = t.contiguous()
    b = t.reshape(-1).view(torch.uint8) if t.numel() else t.new_empty(0, dtype=torch.uint8)
    nw = b.numel() // 4
    words = b[: nw * 4].view(torch.int32)
    s0 = torch.zeros((), dtype=torch.int64, device=t.device)
    s1 = torch.zeros((), dtype=torch.int64, device=t.device)
    for lo in range(0, nw, _FP_CHUNK):
        w = words[lo: lo + _FP_CHUNK].to(torch.int64)
        pos = torch.arange(lo, lo + w.numel(), dtype=torch.int64, device=t.device)
        m = ((pos * 0x9E3779B1) & 0x7FFFFFFF) | 1
        s0 += w.sum()
        s1 += (w * m).sum()
    tail = bytes(b[nw * 4:].cpu().tolist())
    return (str(t.dtype), tuple(t.shape), int(s0), int(s1), tail)


def column_digest(col) -> tuple:
    """Digest of one column's local rows (device columns on device, host columns on host)."""
    from ..frame import column as C
    try:
        from ..synthetic import LineageVectorColumn
    except ImportError:          # pragma: no cover
        LineageVectorColumn = ()
    if LineageVectorColumn and isinstance(col, LineageVectorColumn):
        # rows past the resident prefix are a pure function of (seed, global row)
        sp = col.spec
        return ("lineage", sp.seed, sp.d, sp.ld, len(col), col.row0, float(sp.btrue),
                _tensor_digest(sp.wtrue), _tensor_digest(col.data))
    if isinstance(col, C.NumericColumn):
        return ("num", _tensor_digest(col.data), _tensor_digest(col.valid))
    if isinstance(col, C.VectorColumn):
        return ("vec", col.size, _tensor_digest(col.data))
    if isinstance(col, C.SparseVectorColumn):
        return ("csr", col.size, _tensor_digest(col.indptr), _tensor_digest(col.indices),
                _tensor_digest(col.values))
    if isinstance(col, C.HostColumn):
        h = hashlib.sha1()
        for v in col.values:
            h.update(repr(v).encode())
            h.update(b"\x00")
        return ("host", len(col), h.hexdigest())
    return (type(col).__name__, len(col))


def _input_columns(est, df) -> list[str]:
    """Columns the estimator reads: every ``*Col`` / ``*Cols`` param naming a column of df."""
    names = []
    for p in est.params:
        if not (p.name.endswith("Col") or p.name.endswith("Cols")) or not est.isDefined(p):
            continue
        v = est.getOrDefault(p)
        for c in (v if isinstance(v, (list, tuple)) else [v]):
            if isinstance(c, str) and c in df.columns and c not in names:
                names.append(c)
    return names


def data_fingerprint(est, df) -> str:
    """Fingerprint of the rows ``est`` would train on, identical on every rank: the global
    row count plus the rank-ordered digests of every input column's local rows."""
    local = fingerprint(len(df), [(c, column_digest(df.column_data(c))) for c in _input_columns(est, df)])
    comm = df.comm
    parts = comm.all_gather_object(local) if comm is not None and comm.world_size > 1 else [local]
    return fingerprint(parts)


def for_estimator(est, df, sharded: bool = False, extra=()) -> Checkpointer:
    """Checkpointer for ``est.fit(df)``: enabled when the session has a checkpoint dir and
    the estimator's ``checkpointInterval`` (or conf ``o3s.checkpoint.interval``) is > 0.

    The key hashes the estimator class, its params, a digest of the training data
    (:func:`data_fingerprint`) and ``extra`` (e.g. ALS user/item counts), so only a fit of
    the same configuration on the same data resumes; solvers call ``clear()`` once a fit
    completes."""
    session = getattr(df, "session", None)
    root = checkpoint_dir(session)
    interval = 0
    if root:
        if est.hasParam("checkpointInterval") and est.isDefined(est.getParam("checkpointInterval")):
            interval = int(est.getOrDefault(est.getParam("checkpointInterval")))
        else:
            interval = int(session.conf.get("o3s.checkpoint.interval", "0") or 0)
    if not root or interval <= 0:
        return Checkpointer(None, "", 0, df.comm, sharded=sharded)
    params = sorted((p.name, repr(v)) for p, v in est.extractParamMap().items()
                    if p.name not in ("checkpointInterval",))
    data = data_fingerprint(est, df)
    key = f"{type(est).__name__}-{fingerprint(type(est).__name__, params, data, extra)}"
    return Checkpointer(root, key, interval, df.comm, sharded=sharded)
