"""MEMORY_AND_DISK storage: feature rows beyond the HBM budget live in pinned host memory
and stream through the GPU on every pass.

Reference: ``df.cache()`` (orangecontrib/spark/widgets/data/spark_df_cache.py:39) and the
estimators' repeated passes (spark_ml_estimator.py:22).  Spark's default storage level
spills partitions that do not fit in executor memory and streams them back on each use;
on MI355X the "memory" tier is 288 GB of HBM3E per GPU and the "disk" tier is pinned host
DRAM behind PCIe.  Design:

* :class:`SpilledVectorColumn` -- a vector column whose first ``resident_rows`` rows are
  a device matrix and whose remaining rows are one pinned host matrix.
* :class:`HostStreamer` -- double-buffered H2D streaming of the host rows in fixed-size
  chunks on a dedicated copy stream: chunk i+1 is copied while the consumer's kernels run
  on chunk i; copies and kernels are ordered by HIP events only (no host synchronisation
  per chunk), and a staging buffer is refilled only after the kernels that read it
  finished (``free`` event).  Consumers: the GLM pass (models/glm.py) and the KMeans
  assign/update pass (models/kmeans.py).
* :func:`spill_to_budget` -- ``DataFrame.persist(MEMORY_AND_DISK)``: moves the rows of
  device vector columns beyond the HBM budget (``o3s.storage.hbmBudget`` bytes, default
  the session's ``o3s.memory.fraction`` of free HBM) to pinned host memory.
* out-of-core ingest (:func:`host_resident`): a table read from parquet / the catalog /
  pandas / Arrow whose numeric columns exceed the budget keeps them on the host from the
  start, zero copy over the Arrow / numpy buffers (nothing is materialised on the device);
  ``VectorAssembler`` stages them through pinned buffers in row chunks into the assemble
  kernel, straight into a SpilledVectorColumn (:func:`assemble_streamed`), whose resident
  prefix fills the budget; GLM / KMeans / tree fits and the scalers consume it chunk by
  chunk (tree binning writes resident uint8 bins per chunk).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import column as C

CHUNK_BYTES = int(os.environ.get("O3S_SPILL_CHUNK_MB", "512")) << 20


class SpilledVectorColumn(C.VectorColumn):
    """Dense vectors: rows [0, resident) on the device (``data``), rows [resident, n) in
    pinned host memory (``host``), same dtype and leading dimension."""

    max_materialise_bytes = 32 << 30

    def __init__(self, resident: torch.Tensor, host: torch.Tensor, size: int | None = None):
        super().__init__(resident, size)
        if host.dim() != 2 or host.shape[1] != resident.shape[1] or host.dtype != resident.dtype:
            raise ValueError("host rows must match the resident rows' width and dtype")
        self.host = host

    def __len__(self):
        return int(self.data.shape[0] + self.host.shape[0])

    @property
    def resident_rows(self) -> int:
        return int(self.data.shape[0])

    @property
    def spilled_rows(self) -> int:
        return int(self.host.shape[0])

    def full(self) -> torch.Tensor:
        nbytes = len(self) * self.ld * self.data.element_size()
        if nbytes > self.max_materialise_bytes and self.data.is_cuda:
            raise MemoryError(f"materialising {nbytes / 2**30:.1f} GiB of spilled rows on the device; consume "
                              "this column with a streaming op (GLM / KMeans fits) or sample / limit first")
        return torch.cat([self.data, self.host.to(self.data.device)])

    def dense(self):
        f = self.full()
        return f if self.size == self.ld else f[:, : self.size]

    def take(self, idx):
        idx = idx.to(torch.int64)
        dev = self.data.device
        out = torch.empty((idx.numel(), self.ld), dtype=self.data.dtype, device=dev)
        nr = self.resident_rows
        idx_d = idx.to(dev)
        on_dev = idx_d < nr
        if bool(on_dev.any()):
            out[on_dev] = self.data[idx_d[on_dev]]
        off = ~on_dev
        if bool(off.any()):
            hi = (idx_d[off] - nr).cpu()
            out[off] = self.host[hi].to(dev)
        return C.VectorColumn(out, self.size)

    def mask_select(self, mask):
        """Rows where ``mask`` holds, keeping the layout: the selected resident rows stay a
        device prefix and the selected host rows a pinned host suffix (nothing of the
        column's length is materialised on the device -- ``filter`` / handleInvalid
        "skip" on an out-of-core frame)."""
        nr = self.resident_rows
        m = mask.reshape(-1)
        res = self.data[m[:nr].to(self.data.device)]
        hm = m[nr:].cpu()
        host = self.host[hm]
        if self.host.is_pinned() and not host.is_pinned() and host.numel():
            host = host.pin_memory()
        if host.shape[0] == 0:
            return C.VectorColumn(res, self.size)
        return SpilledVectorColumn(res, host, self.size)

    def slice(self, start, end):
        n = len(self)
        start, end = max(0, start), min(n, end)
        nr = self.resident_rows
        if end <= nr:
            return C.VectorColumn(self.data[start:end], self.size)
        if start >= nr:
            return SpilledVectorColumn(self.data[:0], self.host[start - nr:end - nr], self.size)
        return SpilledVectorColumn(self.data[start:nr], self.host[: end - nr], self.size)

    def to_numpy(self):
        a = torch.cat([self.data.detach().cpu(), self.host])[:, : self.size]
        if a.dtype in (torch.bfloat16, torch.float16):
            a = a.float()
        return a.numpy().astype(np.float64)

    def nbytes(self):
        return (self.data.numel() + self.host.numel()) * self.data.element_size()

    @staticmethod
    def concat(cols):
        """Row concatenation WITHOUT materialising on the device (``DataFrame.union`` of
        out-of-core frames): the first column's resident rows stay resident, every later row
        goes to one pinned host matrix (a resident prefix plus a host suffix is the only
        layout the streaming consumers read).  Width / dtype follow the first column."""
        first = cols[0]
        dev, dt, ld, size = first.data.device, first.data.dtype, first.ld, first.size
        res = first.data
        tail = [first.host] if isinstance(first, SpilledVectorColumn) else []
        for c in cols[1:]:
            tail.append(_fit_ld(c.data, ld, dt, size))
            if isinstance(c, SpilledVectorColumn):
                tail.append(_fit_ld(c.host, ld, dt, size))
        tail = [t for t in tail if t.shape[0]]
        if not tail:
            return C.VectorColumn(res, size)
        host = _pinned_cat(tail, pin=dev.type == "cuda")
        return SpilledVectorColumn(res, host, size)

    def streamer(self, chunk_bytes: int | None = None) -> "HostStreamer":
        s = getattr(self, "_streamer", None)
        if s is None or (chunk_bytes is not None and s.chunk_bytes != chunk_bytes):
            s = self._streamer = HostStreamer(self.host, self.data.device, chunk_bytes)
        return s


class HostStreamer:
    """Double-buffered host -> device streaming of a pinned [n, ld] matrix in row chunks."""

    def __init__(self, host: torch.Tensor, device, chunk_bytes: int | None = None):
        self.host = host
        self.device = torch.device(device)
        self.chunk_bytes = int(chunk_bytes or CHUNK_BYTES)
        row_bytes = max(1, host.shape[1] * host.element_size())
        self.chunk_rows = max(1, self.chunk_bytes // row_bytes)
        n = int(host.shape[0])
        self.ranges = [(a, min(n, a + self.chunk_rows)) for a in range(0, n, self.chunk_rows)]
        self.bytes_streamed = 0
        if self.device.type == "cuda" and self.ranges:
            rows = min(self.chunk_rows, n)
            self.buf = [torch.empty((rows, host.shape[1]), dtype=host.dtype, device=self.device) for _ in range(2)]
            self.stream = torch.cuda.Stream(self.device)
            self.ready = [torch.cuda.Event(), torch.cuda.Event()]
            self.free = [torch.cuda.Event(), torch.cuda.Event()]
            self._free_recorded = [False, False]

    def __len__(self):
        return len(self.ranges)

    def _issue_copy(self, i: int):
        a, b = self.ranges[i]
        k = i & 1
        cs = self.stream
        if self._free_recorded[k]:
            cs.wait_event(self.free[k])           # the kernels of chunk i-2 are done with buf[k]
        with torch.cuda.stream(cs):
            self.buf[k][: b - a].copy_(self.host[a:b], non_blocking=True)
        self.ready[k].record(cs)

    def run(self, fn) -> None:
        """``fn(chunk, row_offset)`` for every chunk, in order, on the current stream.

        GPU: copy i+1 is issued before ``fn(i)`` runs (prefetch depth 1, whatever ``fn``
        does on the host), ``fn``'s kernels wait only for their chunk's copy event, and
        a staging buffer is refilled only after the kernels that read it finished.  The
        chunk view is valid until ``fn`` returns (enqueue-wise)."""
        if not self.ranges:
            return
        if self.device.type != "cuda":
            for a, b in self.ranges:
                fn(self.host[a:b], a)
            return
        main = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(main)                # the consumer's inputs (e.g. coefficients) are ready
        self._issue_copy(0)
        for i, (a, b) in enumerate(self.ranges):
            if i + 1 < len(self.ranges):
                self._issue_copy(i + 1)
            k = i & 1
            main.wait_event(self.ready[k])
            fn(self.buf[k][: b - a], a)
            self.free[k].record(main)
            self._free_recorded[k] = True
            self.bytes_streamed += (b - a) * self.host.shape[1] * self.host.element_size()


def map_rows(col: "SpilledVectorColumn", fn) -> torch.Tensor:
    """``fn`` (device rows -> per-row tensor) over the resident rows and then every
    streamed chunk; the pieces are concatenated in row order (e.g. a model's margins)."""
    outs = [fn(col.data)] if col.resident_rows or not col.spilled_rows else []
    col.streamer().run(lambda X, off: outs.append(fn(X)))
    return torch.cat(outs) if len(outs) > 1 else outs[0]


class RowBlocks:
    """The rows of a spilled vector column as a sequence of device blocks -- the resident
    matrix, then every streamed chunk -- each passed through ``prep`` (dtype / layout /
    normalisation the consumer needs).  ``run(fn)`` calls ``fn(block, first_row)``."""

    def __init__(self, col: "SpilledVectorColumn", prep=None):
        self.col = col
        self.prep = prep or (lambda X: X)
        self.n = len(col)
        self.nres = col.resident_rows
        self.D = col.size
        self.device = col.data.device
        self._res = self.prep(col.data[:, : col.size]) if self.nres else None

    @property
    def shape(self):
        return (self.n, self.D)

    def run(self, fn) -> None:
        if self.nres:
            fn(self._res, 0)
        if self.col.spilled_rows:
            self.col.streamer().run(lambda X, off: fn(self.prep(X[:, : self.D]), self.nres + off))

    def rows(self, idx: torch.Tensor) -> torch.Tensor:
        """Rows at local indices ``idx`` (device tensor, prepared)."""
        return self.prep(self.col.take(idx).data[:, : self.D])


def _fit_ld(t: torch.Tensor, ld: int, dt, size: int) -> torch.Tensor:
    """``t`` with leading dimension ``ld`` and dtype ``dt`` (columns of one vector size can
    differ in padding / dtype: fp64 unpadded vs bf16 padded)."""
    if t.shape[1] == ld and t.dtype == dt:
        return t
    out = torch.zeros((t.shape[0], ld), dtype=dt, device=t.device)
    out[:, :size] = t[:, :size].to(dt)
    return out


def map_blocks(col: "SpilledVectorColumn", fn, chunk_bytes: int | None = None,
               budget: int | None = None) -> "SpilledVectorColumn":
    """A row-wise map over an out-of-core vector column into a NEW spilled column
    (feature transformers on frames larger than HBM).  ``fn``: fp64 rows [m, size] ->
    fp64 rows [m, size].  Resident rows are mapped in bounded chunks (no fp64 copy of the
    whole prefix); host rows stream through the device and are written back to pinned
    memory asynchronously on the consumer stream.

    Output storage: the column's own dtype and padding (bf16 on the GPU).  An out-of-core
    table is by definition larger than HBM, so its derived columns stay in the compact
    storage dtype -- fp64 (what a resident transform returns, as Spark's double vectors)
    would take 4x the HBM and pinned host bytes; the map itself is computed in fp64.

    Output split: the input's resident prefix already holds its share of HBM, so the
    output's device prefix takes at most ``budget`` bytes (default: what the device can
    allocate now, less working room for the fp64 chunks, times ``o3s.memory.fraction``);
    rows beyond it go to the pinned host part like the streamed ones."""
    dt, ld, D, dev = col.data.dtype, col.ld, col.size, col.data.device
    cuda = dev.type == "cuda"
    step = max(1, int(chunk_bytes or CHUNK_BYTES) // max(1, ld * 8))
    row_bytes = ld * col.data.element_size()
    if budget is None and cuda:
        from ..session import Session
        s = Session.active()
        frac = s.conf.memory_fraction() if s is not None else 0.85
        work = 4 * step * ld * 8 + (256 << 20)       # fp64 chunk, its map, the cast, slack
        budget = int(max(0, device_free_bytes(dev) - work) * frac)
    keep = col.resident_rows if budget is None else min(col.resident_rows, max(0, int(budget) // max(1, row_bytes)))

    def apply(X):
        y = fn(X[:, :D].to(torch.float64))
        if y.shape != (X.shape[0], D):
            raise ValueError("map_blocks: fn must keep the row count and the vector size")
        out = torch.zeros((X.shape[0], ld), dtype=dt, device=X.device) if ld != D else None
        if out is None:
            return y.to(dt)
        out[:, :D] = y.to(dt)
        return out

    res = torch.empty((keep, ld), dtype=dt, device=dev)
    spill = col.resident_rows - keep                # input-resident rows whose output goes to the host
    host = torch.empty((spill + col.spilled_rows, ld), dtype=dt, pin_memory=cuda and torch.cuda.is_available())
    for a in range(0, col.resident_rows, step):
        b = min(col.resident_rows, a + step)
        y = apply(col.data[a:b])
        r = max(0, min(b, keep) - a)
        if r:
            res[a:a + r] = y[:r]
        if b - a - r:
            host[a + r - keep:b - keep].copy_(y[r:], non_blocking=cuda)

    def sink(X, off):
        for a in range(0, X.shape[0], step):
            b = min(X.shape[0], a + step)
            host[spill + off + a:spill + off + b].copy_(apply(X[a:b]), non_blocking=cuda)
    col.streamer(chunk_bytes).run(sink)
    if cuda:
        torch.cuda.synchronize(dev)
    return SpilledVectorColumn(res, host, D)


def block_moments(col: "SpilledVectorColumn"):
    """(sum, sum of squares, count, max |x| (finite), min, max) of every vector slot over
    the resident rows and every streamed chunk, fp64 -- the column summary the scalers fit
    on, without materialising the column."""
    D, dev = col.size, col.data.device
    z = torch.zeros(D, dtype=torch.float64, device=dev)
    acc = {"s": z.clone(), "ss": z.clone(), "mx": z.clone(),
           "lo": torch.full((D,), float("inf"), dtype=torch.float64, device=dev),
           "hi": torch.full((D,), float("-inf"), dtype=torch.float64, device=dev)}
    step = max(1, CHUNK_BYTES // max(1, D * 8))

    def add(X, _off=0):
        for a in range(0, X.shape[0], step):
            x = X[a:a + step, :D].to(torch.float64)
            acc["s"] += x.sum(0)
            acc["ss"] += (x * x).sum(0)
            acc["mx"] = torch.maximum(acc["mx"], torch.where(torch.isfinite(x), x, torch.zeros_like(x)).abs().max(0).values)
            acc["lo"] = torch.minimum(acc["lo"], x.min(0).values)
            acc["hi"] = torch.maximum(acc["hi"], x.max(0).values)
    if col.resident_rows:
        add(col.data)
    col.streamer().run(add)
    return acc["s"], acc["ss"], float(len(col)), acc["mx"], acc["lo"], acc["hi"]


def _pinned_copy(src: torch.Tensor) -> torch.Tensor:
    """Device rows -> a pinned host matrix, in bounded chunks (no full-size staging)."""
    return _pinned_cat([src], pin=src.is_cuda)


def _pinned_cat(parts, pin: bool = True) -> torch.Tensor:
    """Row-concatenation of device and/or host matrices into ONE pinned host matrix
    (``torch.cat`` of pinned tensors returns pageable memory, which would halve the
    streaming rate), copied in bounded chunks."""
    parts = [p for p in parts if p is not None]
    ld, dt = parts[0].shape[1], parts[0].dtype
    n = sum(int(p.shape[0]) for p in parts)
    out = torch.empty((n, ld), dtype=dt, pin_memory=pin and torch.cuda.is_available())
    step = max(1, (256 << 20) // max(1, ld * parts[0].element_size()))
    off = 0
    for p in parts:
        for a in range(0, p.shape[0], step):
            b = min(p.shape[0], a + step)
            out[off + a:off + b].copy_(p[a:b])
        off += int(p.shape[0])
    return out


def device_free_bytes(dev) -> int:
    """Bytes a new device allocation can take now: free HBM plus the caching allocator's
    reserved-but-unused blocks."""
    dev = torch.device(dev)
    if dev.type != "cuda":
        return 1 << 62
    free, _ = torch.cuda.mem_get_info(dev)
    return int(free + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev))


def ingest_budget(session) -> int | None:
    """Device bytes the numeric columns of a NEW table may take (out-of-core ingest:
    read.parquet / catalog tables / createDataFrame): ``o3s.storage.hbmBudget`` when set,
    else on the GPU the session's ``o3s.memory.fraction`` of the allocatable HBM; None on
    the CPU with no explicit budget (no limit)."""
    v = session.conf.get("o3s.storage.hbmBudget", None)
    if v not in (None, "", "auto"):
        return int(float(v))
    if session.device.type != "cuda":
        return None
    return int(device_free_bytes(session.device) * session.conf.memory_fraction())


def host_resident(session, nbytes: int) -> bool:
    """True when a new table of ``nbytes`` numeric bytes must stay in host memory (its
    columns are then streamed to the device by the consumers: VectorAssembler into a
    SpilledVectorColumn, labels moved on use)."""
    b = ingest_budget(session)
    return b is not None and nbytes > b and session.device.type == "cuda"


def pinned(t: torch.Tensor) -> torch.Tensor:
    """A pinned host copy (plain host tensor when no GPU is present)."""
    t = t.detach()
    if t.device.type != "cpu":
        t = t.cpu()
    return t.pin_memory() if torch.cuda.is_available() else t.contiguous()


def host_array(a: np.ndarray) -> torch.Tensor:
    """Zero-copy host tensor over a numpy array (out-of-core ingest: Arrow / pandas column
    buffers are read-only and stay where they are -- no writable copy, no pinned copy; the
    consumer stages row chunks through pinned buffers, see :func:`assemble_streamed`).
    The engine never writes into a source column in place."""
    import warnings
    a = np.ascontiguousarray(a)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)       # "non-writable NumPy array"
        return torch.from_numpy(a)


def hbm_budget(session) -> int:
    v = session.conf.get("o3s.storage.hbmBudget", None)
    if v not in (None, "", "auto"):
        return int(float(v))
    dev = session.device
    if dev.type != "cuda":
        return 1 << 62
    free, _ = torch.cuda.mem_get_info(dev)
    return int(free * session.conf.memory_fraction())


def spill_to_budget(df, budget: int | None = None, disk_only: bool = False) -> int:
    """Move rows of ``df``'s dense vector columns beyond ``budget`` bytes (largest column
    first; every column's resident prefix counts against the budget) to pinned host memory,
    in place.  Returns the bytes moved.  ``disk_only``: every row of those columns."""
    budget = hbm_budget(df.session) if budget is None else int(budget)
    vec = [(k, c) for k, c in df._cols.items()
           if type(c) is C.VectorColumn or isinstance(c, SpilledVectorColumn)]
    vec.sort(key=lambda kc: -kc[1].nbytes())
    moved = 0
    left = 0 if disk_only else budget
    while vec:
        k, c = vec.pop(0)
        row_bytes = c.ld * c.data.element_size()
        n = len(c)
        keep = min(n, max(0, left // max(row_bytes, 1)))
        nres = c.resident_rows if isinstance(c, SpilledVectorColumn) else n
        if keep >= nres:
            left -= nres * row_bytes
            continue
        old_host = c.host if isinstance(c, SpilledVectorColumn) else None
        size, dev = c.size, c.data.device
        host = _pinned_cat([c.data[keep:], old_host])
        moved += (nres - keep) * row_bytes
        if keep * row_bytes + (64 << 20) <= device_free_bytes(dev):
            res = c.data[:keep].clone()
        else:
            # the new resident prefix does not fit NEXT TO the old column (the auto budget
            # counts the column's own bytes as available): stage the prefix through pinned
            # host memory, drop the device column, then re-allocate what is actually free
            # (less if another frame still shares the old buffer)
            pre = _pinned_cat([c.data[:keep]])
            df._cols[k] = SpilledVectorColumn(torch.empty((0, c.ld), dtype=c.data.dtype, device=dev), host, size)
            del c
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            fit = max(0, (device_free_bytes(dev) - (64 << 20)) // max(row_bytes, 1))
            k2 = min(keep, fit)
            res = pre[:k2].to(dev)
            if k2 < keep:
                host = _pinned_cat([pre[k2:], host])
            del pre
            moved += (keep - k2) * row_bytes
            keep = k2
        df._cols[k] = SpilledVectorColumn(res, host, size)
        left -= keep * row_bytes
    return moved


def assemble_streamed(sources, n: int, session, budget: int | None, chunk_bytes: int | None = None,
                      want_bad: bool = False):
    """VectorAssembler over host-resident (and/or device) columns, in row chunks.

    ``sources``: list of (tensor [n] or [n, w], valid [n] | None, width) -- host tensors
    may be pageable (zero-copy Arrow / numpy buffers).  GPU pipeline per chunk c:
    the host rows of chunk c+1 are copied into one of two pinned staging sets (CPU, while
    the GPU works) and sent on a copy stream; chunk c is assembled by the bf16 gather kernel
    on the current stream once its copy event fired; rows beyond the budget go back to the
    pinned host block on a third stream (H2D and D2H overlap on the full-duplex link); the
    invalid-row count stays on the device until the end.  CPU: torch, chunk by chunk.
    Returns (SpilledVectorColumn | VectorColumn, invalid count), plus the per-row invalid
    flags (bool [n] on the device) when ``want_bad`` (handleInvalid "skip")."""
    from ..ops import assemble as A
    from ..ops.glm import padded_width
    dev = session.device
    vdt = session.vector_dtype()
    D = sum(int(w) for _, _, w in sources)
    ld = padded_width(D) if vdt == torch.bfloat16 else D
    esz = torch.empty((), dtype=vdt).element_size()
    keep = n if budget is None else max(0, min(n, budget // max(1, ld * esz)))
    in_row = sum(t.element_size() * (1 if t.dim() == 1 else t.shape[1]) for t, _, _ in sources) or 1
    rows = max(1024, int(chunk_bytes or CHUNK_BYTES) // in_row)
    cuda = dev.type == "cuda"
    import time as _time
    _t0 = _time.perf_counter()
    res = torch.empty((keep, ld), dtype=vdt, device=dev)
    host = torch.empty((n - keep, ld), dtype=vdt, pin_memory=cuda and torch.cuda.is_available())
    _t_alloc = _time.perf_counter() - _t0
    bounds = [(a, min(n, a + rows)) for a in range(0, n, rows)]
    bad_all = torch.zeros(n, dtype=torch.bool, device=dev) if want_bad else None
    if not cuda:
        nbad = 0
        for a, b in bounds:
            out, nb = _assemble_chunk_torch([(t[a:b], None if v is None else v[a:b], w) for t, v, w in sources],
                                            b - a, D, ld, vdt)
            nbad += nb
            if want_bad and nb:
                bad_all[a:b] = torch.isnan(out[:, :D].float()).any(1)
            r = max(0, min(b, keep) - a)
            res[a:a + r] = out[:r]
            host[a + r - keep:b - keep] = out[r:]
        col = SpilledVectorColumn(res, host, D) if n > keep else C.VectorColumn(res, D)
        return (col, nbad, bad_all) if want_bad else (col, nbad)
    copy, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)
    # two pinned staging sets for the host-side sources (pageable -> pinned on the CPU)
    def _stage_buf(t):
        shape = (rows,) + tuple(t.shape[1:])
        return torch.empty(shape, dtype=t.dtype, pin_memory=True)
    _t1 = _time.perf_counter()
    stg = [[(None if t.is_cuda else _stage_buf(t), None if (v is None or v.is_cuda) else _stage_buf(v))
            for t, v, _ in sources] for _ in range(2)]
    sent = [None, None]                         # copy event of the chunk that last used set k
    stats = {"chunks": len(bounds), "host_wait_s": 0.0, "host_copy_s": 0.0, "out_alloc_s": _t_alloc,
             "staging_alloc_s": _time.perf_counter() - _t1}
    LAST_ASSEMBLE_STATS.clear()
    LAST_ASSEMBLE_STATS.update(stats)

    def stage(i):
        a, b = bounds[i]
        m = b - a
        k = i & 1
        t0 = _time.perf_counter()
        if sent[k] is not None:
            sent[k].synchronize()               # the H2D of chunk i-2 has drained set k
        t1 = _time.perf_counter()
        LAST_ASSEMBLE_STATS["host_wait_s"] += t1 - t0
        out, copies = [], []
        for (t, v, w), (tb, vb) in zip(sources, stg[k]):
            tt, vv = t[a:b], None if v is None else v[a:b]
            if tb is not None:
                copies.append((tb[:m], tt))
                tt = tb[:m]
            if vb is not None:
                copies.append((vb[:m], vv))
                vv = vb[:m]
            out.append((tt, vv, w))
        _parallel_copy(copies)                  # pageable -> pinned, on host threads
        LAST_ASSEMBLE_STATS["host_copy_s"] += _time.perf_counter() - t1
        with torch.cuda.stream(copy):
            out = [(tt.to(dev, non_blocking=True), None if vv is None else vv.to(dev, non_blocking=True), w)
                   for tt, vv, w in out]
        ev = torch.cuda.Event()
        ev.record(copy)
        sent[k] = ev
        return out, ev

    nbad_d = torch.zeros(1, dtype=torch.int64, device=dev)
    nxt = stage(0) if bounds else None
    for i, (a, b) in enumerate(bounds):
        cur, ev = nxt
        if i + 1 < len(bounds):
            nxt = stage(i + 1)                  # CPU staging + H2D of chunk i+1 overlap chunk i
        main.wait_event(ev)
        for t, v, _ in cur:
            t.record_stream(main)
            if v is not None:
                v.record_stream(main)
        m = b - a
        if vdt == torch.bfloat16 and all(A.supported(t) for t, _, _ in cur):
            out, badf, nb, _ = A.assemble_bf16(cur, m, dev)
            nbad_d += nb.to(torch.int64)
            if want_bad:
                bad_all[a:b] = badf.bool()
        else:
            out, nb = _assemble_chunk_torch(cur, m, D, ld, vdt)
            nbad_d += nb
            if want_bad:
                bad_all[a:b] = torch.isnan(out[:, :D].float()).any(1)
        r = max(0, min(b, keep) - a)
        if r:
            res[a:a + r].copy_(out[:r])
        if m - r:
            d2h.wait_stream(main)
            with torch.cuda.stream(d2h):
                host[a + r - keep:b - keep].copy_(out[r:], non_blocking=True)
            out.record_stream(d2h)
    t2 = _time.perf_counter()
    LAST_ASSEMBLE_STATS["loop_s"] = t2 - _t0
    torch.cuda.synchronize(dev)
    LAST_ASSEMBLE_STATS["final_sync_s"] = _time.perf_counter() - t2
    col = SpilledVectorColumn(res, host, D) if n > keep else C.VectorColumn(res, D)
    return (col, int(nbad_d.item()), bad_all) if want_bad else (col, int(nbad_d.item()))


_COPY_POOL = None
LAST_ASSEMBLE_STATS: dict = {}      # host-side time split of the last streamed assembly (GPU)


def _parallel_copy(pairs, piece_bytes: int = 8 << 20) -> None:
    """dst.copy_(src) for host tensor pairs, split into ~8 MB row pieces over a thread pool
    (numpy copies release the GIL): one thread copies pageable memory at ~10 GB/s, far
    below the PCIe rate the staged chunks then move at."""
    global _COPY_POOL
    tasks = []
    for dst, src in pairs:
        d, s_ = dst.numpy(), src.numpy()
        row = max(1, d[:1].nbytes)
        step = max(1, piece_bytes // row)
        tasks += [(d[i:i + step], s_[i:i + step]) for i in range(0, d.shape[0], step)]
    if len(tasks) <= 1:
        for d, s_ in tasks:
            np.copyto(d, s_)
        return
    if _COPY_POOL is None:
        import concurrent.futures as cf
        _COPY_POOL = cf.ThreadPoolExecutor(max_workers=max(1, min(16, (os.cpu_count() or 2) // 2)))
    list(_COPY_POOL.map(lambda ds: np.copyto(ds[0], ds[1]), tasks))


def _assemble_chunk_torch(cur, m, D, ld, vdt):
    """(rows [m, ld] of dtype vdt, invalid count) of one chunk by torch (CPU, or GPU
    sources the kernel does not take)."""
    mats = []
    for t, v, w in cur:
        if t.dim() == 1:
            x = t.to(torch.float64)
            if v is not None:
                x = torch.where(v, x, torch.full_like(x, float("nan")))
            mats.append(x[:, None])
        else:
            mats.append(t[:, :int(w)].to(torch.float64))
    mat = torch.cat(mats, 1)
    nb = int(torch.isnan(mat).any(1).sum()) if not mat.is_cuda else torch.isnan(mat).any(1).sum()
    out = torch.zeros((m, ld), dtype=vdt, device=mat.device)
    out[:, :D] = mat.to(vdt)
    return out, nb


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
