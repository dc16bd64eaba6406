"""Collective communication for row-sharded (data-parallel) training.

Replaces Spark's ``treeAggregate`` / broadcast / shuffle between YARN executors
(SURVEY §2.9).  Design, MI355X-first:

* one process per GPU (``torchrun``-style env: RANK / LOCAL_RANK / WORLD_SIZE);
* ``torch.distributed`` with backend ``"nccl"`` -- on ROCm that *is* RCCL running over
  the xGMI point-to-point links -- for device tensors, ``gloo`` for CPU tensors and
  the multi-process CPU tests;
* estimators aggregate **one flat buffer per step** (gradient + loss + weight sum in a
  single fp64 vector, KMeans sums+counts, histogram slabs): xGMI rings are per-link
  bound and small messages are latency bound, so fewer larger collectives win
  (:meth:`Comm.all_reduce_coalesced` packs several tensors into one launch);
* :class:`LocalComm` is the world_size==1 fast path (all collectives are identity).
"""
from __future__ import annotations

import datetime
import os
import pickle
from typing import Any, Sequence

import torch
import torch.distributed as dist


class Comm:
    """Interface.  All methods are collective: every rank must call them in order."""

    rank: int = 0
    world_size: int = 1
    device: torch.device = torch.device("cpu")
    backend: str = "local"

    # -- tensor collectives (in place unless stated) --------------------------------
    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        raise NotImplementedError

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate equally-sized shards along dim 0 (rank order)."""
        raise NotImplementedError

    def all_gather_v(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate variable-length shards along dim 0 (rank order)."""
        raise NotImplementedError

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor, async_op: bool = False):
        """Equal shards gathered straight into ``out`` ([world * t.shape[0], ...], rank
        order): no staging buffer, no concatenation.  ``async_op=True`` returns a handle
        whose ``wait()`` orders the caller's stream after the transfer (RCCL runs it on
        its own stream, so the caller's kernels overlap it); None when already done."""
        raise NotImplementedError

    def reduce_scatter(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def all_to_all_v(self, send: torch.Tensor, send_counts: Sequence[int]) -> tuple[torch.Tensor, list[int]]:
        """Exchange row blocks: rows [sum(c[:r]), sum(c[:r+1])) go to rank r."""
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError

    # -- python objects ---------------------------------------------------------
    def all_gather_object(self, obj: Any) -> list:
        raise NotImplementedError

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        raise NotImplementedError

    def all_to_all_object(self, objs: Sequence[Any]) -> list:
        """``objs[r]`` goes to rank r; returns the objects received, in source-rank order.
        Pickled into one byte buffer on the comm device -> a single all_to_all_v (the
        objects are this job's own data, never files).  The receive side unpickles straight
        from the received buffer (no intermediate bytes copy), so receiving a slice of a
        table costs about the slice once in host memory."""
        if self.world_size == 1:
            return [objs[0]]
        import pickle
        blobs = [pickle.dumps(o, protocol=pickle.HIGHEST_PROTOCOL) for o in objs]
        sizes = [len(b) for b in blobs]
        flat = torch.empty(sum(sizes), dtype=torch.uint8)
        if sizes and sum(sizes):
            fv = flat.numpy()
            off = 0
            for b in blobs:
                fv[off:off + len(b)] = memoryview(b)
                off += len(b)
        del blobs
        recv, counts = self.all_to_all_v(flat.to(self.device), sizes)
        del flat
        raw = memoryview(recv.cpu().numpy())
        out, off = [], 0
        for c in counts:
            out.append(pickle.loads(raw[off:off + c]))
            off += c
        return out

    # -- helpers ----------------------------------------------------------------
    def all_reduce_coalesced(self, tensors: Sequence[torch.Tensor], op: str = "sum") -> list[torch.Tensor]:
        """Pack tensors of one dtype/device into a single buffer -> one collective."""
        if self.world_size == 1 or not tensors:
            return list(tensors)
        flat = torch.cat([t.reshape(-1) for t in tensors])
        self.all_reduce(flat, op)
        out, off = [], 0
        for t in tensors:
            k = t.numel()
            t.copy_(flat[off:off + k].view_as(t))
            out.append(t)
            off += k
        return out

    def sum_scalar(self, x: float | int) -> float | int:
        if self.world_size == 1:
            return x
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.all_reduce(t)
        v = t.item()
        return int(round(v)) if isinstance(x, int) else v

    def max_scalar(self, x: float) -> float:
        if self.world_size == 1:
            return x
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.all_reduce(t, "max")
        return t.item()

    def any_flag(self, flag: bool) -> bool:
        """Collective OR of one host boolean (a stop decision every rank must take at the
        same point).  Runs on the host (gloo) group: no device allocation or sync."""
        return bool(flag)

    @property
    def is_driver(self) -> bool:
        return self.rank == 0


class LocalComm(Comm):
    """Single process, single device: every collective is the identity."""

    def __init__(self, device: torch.device | str = "cpu"):
        self.device = torch.device(device)
        self.rank, self.world_size, self.backend = 0, 1, "local"

    def all_reduce(self, t, op="sum"):
        return t

    def all_gather(self, t):
        return t

    def all_gather_v(self, t):
        return t

    def all_gather_into(self, out, t, async_op=False):
        out.copy_(t)
        return None

    def reduce_scatter(self, t):
        return t

    def broadcast(self, t, src=0):
        return t

    def all_to_all_v(self, send, send_counts):
        return send, [int(send.shape[0])]

    def barrier(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def all_gather_object(self, obj):
        return [obj]

    def broadcast_object(self, obj, src=0):
        return obj


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
        "prod": dist.ReduceOp.PRODUCT}


# "ring": RCCL's all_gather (rings over xGMI); "mesh": grouped peer-to-peer transfers to
# every peer at once (TorchComm._all_gather_mesh).  tools/bench_comm.py times both.
ALLGATHER_ALGO = os.environ.get("O3S_ALLGATHER", "ring")
# O3S_COMM_STRICT=1: GPU sessions refuse host tensors in tensor collectives instead of
# staging them through the device (TorchComm._host)
COMM_STRICT = os.environ.get("O3S_COMM_STRICT", "0") == "1"


class _Works:
    """Handle of several outstanding point-to-point transfers (wait() waits for all)."""

    def __init__(self, reqs):
        self.reqs = list(reqs)

    def wait(self):
        for q in self.reqs:
            q.wait()
        self.reqs = []
        return True

    def is_completed(self):
        return all(q.is_completed() for q in self.reqs)


class TorchComm(Comm):
    """torch.distributed process group: RCCL (backend "nccl") on GPU, gloo on CPU.

    On a GPU node a second gloo group is created for CPU-side object traffic so python
    object collectives never allocate device memory.
    """

    def __init__(self, device: torch.device, backend: str | None = None, group=None, timeout_s: int = 1800):
        self.device = torch.device(device)
        if not dist.is_initialized():
            init_process_group(self.device, backend, timeout_s)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self._cpu_group = None
        if self.backend != "gloo":
            # the same ranks as ``group`` (a subgroup's host collectives must not span the world)
            ranks = None if group is None else dist.get_process_group_ranks(group)
            self._cpu_group = dist.new_group(ranks=ranks, backend="gloo")

    def _host(self, t) -> bool:
        """True when a GPU session's collective got a host tensor.  RCCL takes device
        tensors only (gloo, the one-GPU multi-rank rehearsal, takes both), so such tensors
        are staged through the session device and the result goes back to the host;
        O3S_COMM_STRICT=1 raises instead, to find the call sites."""
        if self.device.type != "cuda" or t.device.type == "cuda":
            return False
        if COMM_STRICT:
            raise RuntimeError(f"host tensor {tuple(t.shape)} {t.dtype} passed to a device collective")
        return True

    def all_reduce(self, t, op="sum"):
        if self.world_size > 1:
            if self._host(t):
                d = t.to(self.device)
                dist.all_reduce(d, op=_OPS[op], group=self.group)
                t.copy_(d.cpu())
            else:
                dist.all_reduce(t, op=_OPS[op], group=self.group)
        return t

    def all_gather(self, t):
        if self.world_size == 1:
            return t
        if self._host(t):
            return self.all_gather(t.to(self.device)).cpu()
        t = t.contiguous()
        out = torch.empty((self.world_size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def all_gather_v(self, t):
        if self.world_size == 1:
            return t
        sizes = self.all_gather_object(int(t.shape[0]))
        m = max(sizes)
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        full = self.all_gather(pad)
        parts = [full[r * m: r * m + s] for r, s in enumerate(sizes)]
        return torch.cat(parts) if parts else t

    def all_gather_into(self, out, t, async_op=False):
        if self.world_size == 1:
            out.copy_(t)
            return None
        if self._host(out) or self._host(t):
            out.copy_(self.all_gather(t.to(self.device)).to(out.device))
            return None
        if ALLGATHER_ALGO == "mesh":
            return self._all_gather_mesh(out, t.contiguous(), async_op)
        return dist.all_gather_into_tensor(out, t.contiguous(), group=self.group, async_op=async_op)

    def _all_gather_mesh(self, out, t, async_op):
        """All-gather as W-1 concurrent peer transfers per rank (one grouped batch of
        isend/irecv): on xGMI every GPU pair has its own link, so each rank's shard leaves
        on all 7 links at once instead of hopping around a ring.  Rank r's
        shard lands at out[r k : (r + 1) k] on every rank, like all_gather_into_tensor."""
        W, r, k = self.world_size, self.rank, t.shape[0]
        out[r * k:(r + 1) * k].copy_(t)
        glob = (lambda q: q) if self.group is None else (lambda q: dist.get_global_rank(self.group, q))
        ops = []
        for d in range(1, W):
            to, frm = (r + d) % W, (r - d) % W
            ops.append(dist.P2POp(dist.isend, t, glob(to), group=self.group))
            ops.append(dist.P2POp(dist.irecv, out[frm * k:(frm + 1) * k], glob(frm), group=self.group))
        reqs = dist.batch_isend_irecv(ops)
        work = _Works(reqs)
        if async_op:
            return work
        work.wait()
        return None

    def reduce_scatter(self, t):
        if self.world_size == 1:
            return t
        if self._host(t):
            return self.reduce_scatter(t.to(self.device)).cpu()
        k = t.shape[0] // self.world_size
        out = torch.empty((k,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, t.contiguous(), group=self.group)
        return out

    def broadcast(self, t, src=0):
        if self.world_size > 1:
            if self._host(t):
                d = t.to(self.device)
                dist.broadcast(d, src=src, group=self.group)
                t.copy_(d.cpu())
                return t
            dist.broadcast(t, src=src, group=self.group)
        return t

    def all_to_all_v(self, send, send_counts):
        if self.world_size == 1:
            return send, [int(send.shape[0])]
        counts = torch.tensor(list(send_counts), dtype=torch.int64)
        all_counts = self.all_gather_object(counts.tolist())
        recv_counts = [all_counts[r][self.rank] for r in range(self.world_size)]
        if self._host(send):
            out = torch.empty((sum(recv_counts),) + tuple(send.shape[1:]), dtype=send.dtype, device=self.device)
            dist.all_to_all_single(out, send.to(self.device).contiguous(), output_split_sizes=recv_counts,
                                   input_split_sizes=list(map(int, send_counts)), group=self.group)
            return out.cpu(), recv_counts
        out = torch.empty((sum(recv_counts),) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        dist.all_to_all_single(out, send.contiguous(), output_split_sizes=recv_counts,
                               input_split_sizes=list(map(int, send_counts)), group=self.group)
        return out, recv_counts

    def barrier(self):
        if self.world_size > 1:
            if self.device.type == "cuda" and self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def all_gather_object(self, obj):
        if self.world_size == 1:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self._cpu_group or self.group)
        return out

    def broadcast_object(self, obj, src=0):
        if self.world_size == 1:
            return obj
        buf = [obj]
        dist.broadcast_object_list(buf, src=src, group=self._cpu_group or self.group)
        return buf[0]

    def any_flag(self, flag):
        if self.world_size == 1:
            return bool(flag)
        t = torch.tensor([1 if flag else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._cpu_group or self.group)
        return bool(t.item())


def env_world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from torchrun-style environment variables."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world


def init_process_group(device: torch.device, backend: str | None = None, timeout_s: int = 1800) -> None:
    if dist.is_initialized():
        return
    rank, _, world = env_world()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        # O3S_DIST_BACKEND=gloo rehearses multi-rank runs with several ranks on one GPU
        # (RCCL refuses two ranks per device); production GPU runs use RCCL ("nccl").
        backend = os.environ.get("O3S_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
    kw = dict(backend=backend, rank=rank, world_size=world,
              timeout=datetime.timedelta(seconds=timeout_s))
    if device.type == "cuda" and backend == "nccl":
        kw["device_id"] = device
    dist.init_process_group(**kw)


def make_comm(device: torch.device | str, world_size: int | None = None, timeout_s: int = 1800) -> Comm:
    device = torch.device(device)
    _, _, world = env_world()
    if world_size is not None:
        world = world_size
    if world <= 1 and not dist.is_initialized():
        return LocalComm(device)
    return TorchComm(device, timeout_s=timeout_s)


# ------------------------------------------------------------ tracing + failure wrapping
COMM_STATS: dict = {}        # op -> [calls, bytes of the first tensor argument], process-wide
def _guard(name, fn):
    """Trace a collective, apply fault injection, and turn backend exceptions into
    CommError carrying op/rank/world (runtime/faults.py)."""
    from ..runtime.faults import INJECTOR, CommError, O3SError
    from ..runtime.tracing import trace
    op = "comm." + name

    def wrapper(self, *a, **k):
        INJECTOR.hit(op)
        st = COMM_STATS.setdefault(name, [0, 0])          # always-on: calls, tensor bytes (no sync)
        st[0] += 1
        if a and isinstance(a[0], torch.Tensor):
            st[1] += a[0].numel() * a[0].element_size()
        with trace(op):
            try:
                return fn(self, *a, **k)
            except O3SError:
                raise
            except Exception as e:  # noqa: BLE001 - RCCL/gloo raise RuntimeError/DistBackendError/...
                raise CommError(name, self.rank, self.world_size, self.backend, e) from e
    wrapper.__name__, wrapper.__doc__, wrapper.__wrapped__ = fn.__name__, fn.__doc__, fn
    return wrapper


for _n in ("all_reduce", "all_gather", "all_gather_v", "all_gather_into", "reduce_scatter", "broadcast", "all_to_all_v", "barrier",
           "all_gather_object", "broadcast_object", "any_flag"):
    setattr(TorchComm, _n, _guard(_n, TorchComm.__dict__[_n]))
LocalComm.all_reduce = _guard("all_reduce", LocalComm.__dict__["all_reduce"])
