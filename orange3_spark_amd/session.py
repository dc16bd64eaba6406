"""Session: the engine entry point (replaces SparkContext + HiveContext/SparkSession).

In the reference a single process-global pair ``sc``/``hc`` is created by the Context
widget (orangecontrib/spark/widgets/data/spark_context.py:68-78) and shared through
class attributes (orangecontrib/spark/base/shared_spark_context.py:9-27).  Here:

* a Session owns the device of this process (``cuda:LOCAL_RANK`` on MI355X, else CPU),
  the communicator (RCCL via torch.distributed when WORLD_SIZE > 1), the catalog
  ("Hive" tables in a parquet warehouse) and the SQL engine;
* one process per GPU: under ``torchrun --nproc-per-node 8`` every rank creates the
  same Session and holds 1/8 of every DataFrame's rows (SPMD, like Spark executors but
  with the driver program replicated);
* ``Session.getOrCreate()`` / ``Session.active()`` give the process-global instance
  the widgets share (``SharedSession`` mixin in the add-on).
"""
from __future__ import annotations

import logging
import threading
from collections import OrderedDict

import numpy as np
import torch

from .conf import SessionConf
from .frame import column as C
from .frame.dataframe import DataFrame, Row
from .parallel.comm import LocalComm, env_world, make_comm

log = logging.getLogger("orange3_spark_amd")

__version__ = "0.1.0"


def resolve_executors(value) -> int:
    """``spark.executor.instances``: an integer, or ``auto`` = every visible GPU (at least 1).
    Counting devices does not initialise HIP (the driver process never touches a GPU)."""
    v = str(value if value is not None else "auto").strip().lower()
    if v in ("", "auto", "*", "all"):
        return max(1, torch.cuda.device_count())
    return int(float(v))


def _wants_pool(conf) -> bool:
    """``spark.executor.instances = N > 1`` (``auto``: N = visible GPUs) outside an SPMD
    launch -> driver + N executors; ``o3s.executor.pool = true`` asks for a pool even at
    N = 1 (the GUI process then never touches the GPU).  ``spark.master`` ``local`` /
    ``local[1]`` keeps everything in this process."""
    import os
    if conf is None or os.environ.get("WORLD_SIZE") not in (None, "", "1"):
        return False
    master = conf.master().lower()
    if master in ("spmd", "local", "local[1]"):
        return False
    try:
        n = resolve_executors(conf.get("spark.executor.instances", "auto"))
    except (TypeError, ValueError):
        return False
    forced = str(conf.get("o3s.executor.pool", "false")).lower() in ("1", "true", "yes")
    return n > 1 or (forced and n >= 1)


class Session:
    _active: "Session | None" = None
    _lock = threading.RLock()

    def __new__(cls, conf: SessionConf | None = None, comm=None, device=None):
        if cls is Session and comm is None and device is None and _wants_pool(conf):
            return object.__new__(DriverSession)
        return object.__new__(cls)

    def __init__(self, conf: SessionConf | None = None, comm=None, device=None):
        self.conf = conf.copy() if conf is not None else SessionConf()
        self.device = torch.device(device) if device is not None else self._pick_device()
        if comm is None:
            master = self.conf.master().lower()
            rank, local, world = env_world()
            comm = make_comm(self.device, timeout_s=int(float(self.conf.get("o3s.comm.timeout", "1800")))) \
                if (world > 1 or master == "spmd") else LocalComm(self.device)
        self.comm = comm
        if self.conf.get("spark.master", "").lower() == "spmd":
            inst = self.conf.get("spark.executor.instances", "auto")
            want = self.comm.world_size if str(inst).lower() in ("auto", "", "*", "all") else int(float(inst))
            if want not in (1, self.comm.world_size):
                raise ValueError(f"spark.executor.instances={want} but this SPMD launch has "
                                 f"WORLD_SIZE={self.comm.world_size} ranks")
        from .catalog import Catalog
        self.catalog = Catalog(self)
        self._stopped = False
        self.version = __version__
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        if str(self.conf.get("o3s.trace", "false")).lower() in ("1", "true", "yes"):
            from .runtime.tracing import TRACER
            TRACER.enable(sync=str(self.conf.get("o3s.trace.sync", "false")).lower() in ("1", "true"))
        self.warmup_seconds: dict = {}
        from .runtime.warmup import plan
        plan(self.conf.get("o3s.session.warmup", "auto"))     # a bad value fails before publication

    def _warmup(self, pool_worker: bool = False) -> None:
        """Kernel code-object preload and (conf) tiny fits of the estimator families once
        per process (``runtime/warmup.py``; conf ``o3s.session.warmup``), so the user's
        first fit does not pay the one-time kernel-loading costs."""
        from .runtime.warmup import warmup
        self.warmup_seconds = warmup(self, pool_worker)

    # ------------------------------------------------------------------ lifecycle
    def _pick_device(self) -> torch.device:
        pref = self.conf.device_pref()
        if pref == "cpu":
            return torch.device("cpu")
        if torch.cuda.is_available():
            _, local, _ = env_world()
            return torch.device("cuda", local % max(1, torch.cuda.device_count()))
        if pref == "cuda":
            raise RuntimeError("o3s.device=cuda but no GPU is visible")
        return torch.device("cpu")

    @classmethod
    def getOrCreate(cls, conf: SessionConf | None = None) -> "Session":
        created = False
        with cls._lock:
            if cls._active is None or cls._active._stopped:
                cls._active = Session(conf)
                created = True
            elif conf is not None:
                for k, v in conf.getAll():
                    cls._active.conf.set(k, v)
            s = cls._active
        if created:            # outside the lock: a warm-up fit may look the session up itself
            s._warmup()
        return s

    @classmethod
    def active(cls) -> "Session | None":
        return cls._active if cls._active is not None and not cls._active._stopped else None

    getActiveSession = active

    def stop(self) -> None:
        self._stopped = True
        if Session._active is self:
            Session._active = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()

    @property
    def rank(self) -> int:
        return self.comm.rank

    @property
    def world_size(self) -> int:
        return self.comm.world_size

    @property
    def defaultParallelism(self) -> int:
        return self.comm.world_size

    @property
    def sparkContext(self):
        """The SparkContext view (RDDs, broadcast, accumulators; rdd.py)."""
        ctx = self.__dict__.get("_sc_view")
        if ctx is None:
            from .rdd import Context
            ctx = self.__dict__["_sc_view"] = Context(self)
        return ctx

    @property
    def udf(self):
        """``spark.udf.register(name, f, returnType)`` -> callable from SQL (sql/udf.py)."""
        from .sql.udf import UDFRegistration
        return UDFRegistration()

    def parallelize(self, c, numSlices=None):
        return self.sparkContext.parallelize(c, numSlices)

    @property
    def appName(self):
        return self.conf.get("spark.app.name")

    # ------------------------------------------------------------------ runtime services
    def setCheckpointDir(self, dirName: str) -> None:
        """Enable iteration checkpoints / resume for iterative estimators
        (runtime/checkpoint.py; SparkContext.setCheckpointDir)."""
        self.conf.set("spark.checkpoint.dir", str(dirName))

    def getCheckpointDir(self):
        return self.conf.get("spark.checkpoint.dir", None)

    def health_check(self, timeout_s: float = 30.0) -> dict:
        """Probe every rank (runtime/faults.py)."""
        from .runtime.faults import health_check
        return health_check(self.comm, timeout_s)

    @property
    def tracer(self):
        """Process tracer (runtime/tracing.py): ``session.tracer.enable()``, ``.table()``."""
        from .runtime.tracing import TRACER
        return TRACER

    def local_view(self) -> "Session":
        """A view of this session whose collectives are local (replicated compute)."""
        v = object.__new__(Session)
        v.__dict__.update(self.__dict__)
        v.comm = LocalComm(self.device)
        return v

    # ------------------------------------------------------------------ dtype policy
    def vector_dtype(self) -> torch.dtype:
        pref = self.conf.vector_dtype()
        if pref == "auto":
            return torch.bfloat16 if self.device.type == "cuda" else torch.float64
        return {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float32": torch.float32,
                "float": torch.float32, "float64": torch.float64, "double": torch.float64}[pref]

    # ------------------------------------------------------------------ creation
    def _shard_bounds(self, n: int) -> tuple[int, int]:
        r, w = self.comm.rank, self.comm.world_size
        return (n * r) // w, (n * (r + 1)) // w

    def createDataFrame(self, data, schema=None, samplingRatio=None, verifySchema=True, _local=False,
                        scatter_from: int | None = None) -> DataFrame:
        """Create a row-sharded DataFrame from host data.

        Accepts a pandas DataFrame, a pyarrow Table, a list of Rows/tuples/dicts, a
        2-D numpy array, a dict of column arrays, or an Orange-style Table (anything
        with ``domain``/``X``).  SPMD: by default every rank is given the same host data and
        keeps its contiguous slice; ``scatter_from=r`` means only rank r holds the table
        (the others pass None) and each rank receives just its slice (host memory per rank
        ~ 1/N).  ``_local``: the data already is this rank's slice (executor scatter).
        Numeric columns reach the GPU through pinned staging buffers.
        """
        if scatter_from is not None and self.comm.world_size > 1:
            return self._scatter_create(data, schema, int(scatter_from))
        from .io import arrow_to_columns
        from .utils import data_utils
        import pandas as pd
        try:
            import pyarrow as pa
        except ImportError:  # pragma: no cover
            pa = None
        from .rdd import RDD
        if isinstance(data, RDD):
            return data.toDF(schema)
        names = _schema_names(schema)
        if hasattr(data, "domain") and hasattr(data, "X"):
            data = data_utils.orange_to_pandas(data)
        if pa is not None and isinstance(data, pa.Table):
            n = data.num_rows
            lo, hi = (0, n) if _local else self._shard_bounds(n)
            cols = arrow_to_columns(data.slice(lo, hi - lo), self)
            return DataFrame(self, cols, hi - lo)
        if isinstance(data, dict):
            data = pd.DataFrame(data)
        if isinstance(data, np.ndarray):
            if data.ndim == 1:
                data = data[:, None]
            data = pd.DataFrame(data, columns=names or [f"_{i + 1}" for i in range(data.shape[1])])
            names = None
        if isinstance(data, (list, tuple)):
            data = _rows_to_pandas(list(data), names)
            names = None
        if not isinstance(data, pd.DataFrame):
            raise TypeError(f"cannot create a DataFrame from {type(data).__name__}")
        if names:
            data = data.copy()
            data.columns = names
        n = len(data)
        lo, hi = (0, n) if _local else self._shard_bounds(n)
        part = data.iloc[lo:hi]
        cols = OrderedDict()
        from .frame import spill
        nb = sum(part[k].to_numpy().nbytes for k in part.columns if part[k].dtype.kind in "fiub")
        host = spill.host_resident(self, nb)          # out-of-core: numeric columns stay on the host
        for k in part.columns:
            arr = part[k].to_numpy()
            if host and arr.dtype.kind in "fiub" and arr.ndim == 1:
                a = arr.astype(np.int64) if arr.dtype.kind == "u" else arr
                cols[str(k)] = C.NumericColumn(spill.host_array(a))
            else:
                cols[str(k)] = C.from_numpy(arr, self.device)
        df = DataFrame(self, cols, hi - lo)
        if schema is not None and not isinstance(schema, (list, tuple)) and hasattr(schema, "fields"):
            for f in schema.fields:
                from .frame.types import NumericType
                if f.name in df.columns and isinstance(f.dataType, NumericType):
                    df = df.withColumn(f.name, df[f.name].cast(f.dataType))
        return df

    def _scatter_create(self, data, schema, src: int) -> DataFrame:
        """Rank ``src`` splits its host table into per-rank row slices and sends slice r to
        rank r (one object all-to-all); no rank but ``src`` ever holds the whole table."""
        from .utils import data_utils
        import pandas as pd
        w = self.comm.world_size
        parts = [None] * w
        if self.comm.rank == src:
            if hasattr(data, "domain") and hasattr(data, "X"):
                data = data_utils.orange_to_pandas(data)
            elif isinstance(data, dict):
                data = pd.DataFrame(data)
            elif isinstance(data, (list, tuple)):
                data = _rows_to_pandas(list(data), _schema_names(schema))
            elif isinstance(data, np.ndarray):
                data = pd.DataFrame(data if data.ndim == 2 else data[:, None])
            n = len(data)
            parts = [data.iloc[(n * r) // w:(n * (r + 1)) // w] for r in range(w)]
        send = parts if self.comm.rank == src else [None] * w
        got = self.comm.all_to_all_object(send)
        part = got[src]
        del parts, send, got, data
        return self.createDataFrame(part, schema, _local=True)

    def range(self, start: int, end: int | None = None, step: int = 1, numPartitions=None) -> DataFrame:
        if end is None:
            start, end = 0, start
        n = max(0, (end - start + step - 1) // step) if step > 0 else max(0, (start - end - step - 1) // (-step))
        lo, hi = self._shard_bounds(n)
        ids = torch.arange(lo, hi, dtype=torch.int64, device=self.device) * step + start
        return DataFrame(self, OrderedDict(id=C.NumericColumn(ids)), hi - lo)

    def emptyDataFrame(self) -> DataFrame:
        return DataFrame(self, OrderedDict(), 0)

    # ------------------------------------------------------------------ catalog / sql
    def table(self, name: str) -> DataFrame:
        return self.catalog.table(name)

    def sql(self, query: str) -> DataFrame:
        from .sql.engine import execute
        return execute(self, query)

    def tableNames(self, dbName: str | None = None) -> list[str]:
        return self.catalog.tableNames(dbName)

    def tables(self, dbName: str | None = None) -> DataFrame:
        names = self.tableNames(dbName)
        db = dbName or self.catalog.currentDatabase()
        return self.createDataFrame({"database": [db] * len(names), "tableName": names,
                                     "isTemporary": [n in self.catalog._temp for n in names]})

    @property
    def read(self):
        from .io import DataFrameReader
        return DataFrameReader(self)

    @property
    def synthetic(self):
        from .synthetic import SyntheticData
        return SyntheticData(self)

    def __repr__(self):
        return (f"Session(app={self.appName!r}, device={self.device}, rank={self.rank}/"
                f"{self.world_size}, backend={self.comm.backend})")


class DriverSession(Session):
    """Driver of an executor pool (runtime/executors.py): this process keeps no rows and
    never touches a GPU; ``spark.executor.instances`` worker processes (one per MI355X, an
    RCCL group over xGMI) hold the data and run every operation.  DataFrames are handles
    (``RemoteDataFrame``); small fitted models come back by value, large ones stay on the
    executors (``RemoteModel``).  When an executor dies the pool is respawned on the next
    call and handles are rebuilt from their lineage (``events`` records it; listeners
    registered with :meth:`add_listener` -- the Context widget -- are told).  Canvas
    defaults are hang-free: collectives time out after ``o3s.executor.commTimeout`` (120 s),
    a rank still busy ``o3s.executor.stragglerTimeout`` (600 s) after its peers answered, or
    a command running past ``o3s.executor.timeout`` (6 h), tears the pool down instead of
    blocking the GUI.  Reference: the Context widget's executor sizing
    (orangecontrib/spark/widgets/data/spark_context.py:41-42,76)."""

    def __init__(self, conf: SessionConf | None = None, comm=None, device=None):
        self.conf = conf.copy() if conf is not None else SessionConf()
        self.device = torch.device("cpu")
        self.comm = LocalComm(self.device)
        self.n_executors = resolve_executors(self.conf.get("spark.executor.instances", "auto"))
        self.events: list = []
        self._listeners: list = []
        self._stopped = False
        self.version = __version__
        self._attach(self._spawn())

    def _pool_conf(self):
        pairs = OrderedDict(self.conf.getAll())
        pairs["spark.executor.instances"] = str(self.n_executors)
        if not self.conf.contains("o3s.comm.timeout"):
            pairs["o3s.comm.timeout"] = self.conf.get("o3s.executor.commTimeout", "120")
        return list(pairs.items())

    def _spawn(self):
        from .runtime.executors import ExecutorPool

        def _f(key, default):
            v = self.conf.get(key, default)
            return None if v in (None, "", "0", "none", "None") else float(v)
        pool = ExecutorPool(self.n_executors, self._pool_conf(),
                            command_timeout=_f("o3s.executor.timeout", "21600"),
                            error_grace=float(self.conf.get("o3s.executor.errorGrace", "20")),
                            straggler_timeout=_f("o3s.executor.stragglerTimeout", "600"))
        pool._respawn = self._respawn
        return pool

    def _attach(self, pool):
        from .runtime.executors import _SESSION_RECIPE
        self.pool = pool
        self._remote = pool._proxy(0, "Session", "obj", None, _SESSION_RECIPE)
        self.catalog = self._remote.catalog

    def _respawn(self, dead):
        """A fresh pool replacing ``dead`` (new subprocesses; never a re-exec of a process
        that touched a GPU), with the dead pool's session effects replayed."""
        if self._stopped or str(self.conf.get("o3s.executor.respawn", "true")).lower() in ("0", "false", "no"):
            from .runtime.executors import ExecutorLost
            raise ExecutorLost("the executor pool is shut down" + (f" ({dead.lost_reason})" if dead.lost_reason else ""))
        import time as _t
        t0 = _t.time()
        new = self._spawn()
        ev = {"event": "executors respawned", "reason": dead.lost_reason, "executors": new.n,
              "devices": list(new.devices), "seconds": None, "time": t0}
        self._attach(new)
        new.replay_effects(dead.effects)
        ev["seconds"] = _t.time() - t0
        self.events.append(ev)
        log.warning("executor pool respawned after: %s", dead.lost_reason)
        for cb in list(self._listeners):
            try:
                cb(ev)
            except Exception:  # noqa: BLE001 - a listener must not break recovery
                log.exception("executor event listener failed")
        return new

    def add_listener(self, cb) -> None:
        """``cb(event_dict)`` on pool events (respawn after an executor loss)."""
        self._listeners.append(cb)

    def restart_executors(self):
        """Replace the pool now (what the next call does after an executor loss)."""
        old = self.pool
        if old.alive:
            old.lost_reason = "restart requested"
            old._teardown()
        return old._revive()

    # --- lifecycle ------------------------------------------------------------------
    def stop(self) -> None:
        if not self._stopped:
            self._stopped = True
            self.pool.shutdown()
        super().stop()

    @property
    def live_pool(self):
        """The current pool, respawned first if the last one was lost."""
        if not self.pool.alive:
            self.pool._revive()
        return self.pool

    @property
    def executors(self) -> int:
        return self.pool.n

    @property
    def world_size(self) -> int:
        return self.pool.n

    @property
    def defaultParallelism(self) -> int:
        return self.pool.n

    def executor_info(self) -> dict:
        pool = self.live_pool
        d = pool.info()
        d["devices"] = list(pool.devices)
        d["respawns"] = len(self.events)
        return d

    def __repr__(self):
        devs = self.pool.devices
        span = devs[0] if len(set(devs)) == 1 else f"{devs[0]}..{devs[-1]}"
        return (f"Session(app={self.appName!r}, executors={self.pool.n} [{span}], driver=cpu, "
                f"alive={self.pool.alive})")

    # --- data sources (all executed on the executors) ---------------------------------
    def createDataFrame(self, data, schema=None, samplingRatio=None, verifySchema=True, **_):
        """Host data -> executors: executor r receives only its row slice (scatter)."""
        from .rdd import RDD  # noqa: F401 - type check below
        from .runtime.executors import is_remote
        from .utils import data_utils
        import pandas as pd
        if is_remote(data):                       # an executor RDD / frame
            return self._remote.createDataFrame(data, schema)
        if hasattr(data, "domain") and hasattr(data, "X"):
            data = data_utils.orange_to_pandas(data)
        try:
            import pyarrow as pa
            if isinstance(data, pa.Table):
                data = data.to_pandas()
        except ImportError:  # pragma: no cover
            pass
        names = _schema_names(schema)
        if isinstance(data, dict):
            data = pd.DataFrame(data)
        if isinstance(data, np.ndarray):
            data = pd.DataFrame(data if data.ndim == 2 else data[:, None],
                                columns=names or [f"_{i + 1}" for i in range(data.shape[1] if data.ndim == 2 else 1)])
            names = None
        if isinstance(data, (list, tuple)):
            data = _rows_to_pandas(list(data), names)
            names = None
        if not isinstance(data, pd.DataFrame):
            raise TypeError(f"cannot create a DataFrame from {type(data).__name__}")
        return self.live_pool.scatter_dataframe(data, schema)

    def range(self, start, end=None, step=1, numPartitions=None):
        return self._remote.range(start, end, step, numPartitions)

    def emptyDataFrame(self):
        return self._remote.emptyDataFrame()

    def table(self, name):
        return self._remote.table(name)

    def sql(self, query):
        return self._remote.sql(query)

    def tableNames(self, dbName=None):
        return self._remote.tableNames(dbName)

    def tables(self, dbName=None):
        return self._remote.tables(dbName)

    @property
    def read(self):
        return self._remote.read

    @property
    def synthetic(self):
        return self._remote.synthetic

    @property
    def sparkContext(self):
        return self._remote.sparkContext

    @property
    def udf(self):
        return self._remote.udf

    def parallelize(self, c, numSlices=None):
        return self._remote.parallelize(c, numSlices)

    def setCheckpointDir(self, dirName):
        super().setCheckpointDir(dirName)
        self._remote.setCheckpointDir(dirName)

    def health_check(self, timeout_s: float = 30.0) -> dict:
        return self._remote.health_check(timeout_s)

    def local_view(self):
        raise RuntimeError("the driver of an executor pool holds no rows (use the executors' session)")


SparkSession = Session


class _Builder:
    def __init__(self):
        self._conf = SessionConf()

    def config(self, key=None, value=None, conf=None):
        if conf is not None:
            for k, v in conf.getAll():
                self._conf.set(k, v)
        if key is not None:
            self._conf.set(key, value)
        return self

    def appName(self, name):
        return self.config("spark.app.name", name)

    def master(self, m):
        return self.config("spark.master", m)

    def enableHiveSupport(self):
        return self

    def getOrCreate(self) -> Session:
        return Session.getOrCreate(self._conf)


class _BuilderDescriptor:
    def __get__(self, obj, owner):
        return _Builder()


Session.builder = _BuilderDescriptor()


def _schema_names(schema):
    if schema is None:
        return None
    if isinstance(schema, (list, tuple)):
        return [s if isinstance(s, str) else s.name for s in schema]
    if hasattr(schema, "names"):
        return list(schema.names)
    if isinstance(schema, str):
        return [p.strip().split(" ")[0].split(":")[0] for p in schema.split(",")]
    return None


def _rows_to_pandas(rows: list, names):
    import pandas as pd
    if not rows:
        return pd.DataFrame(columns=names or [])
    first = rows[0]
    if isinstance(first, Row) and first.__fields__:
        return pd.DataFrame([tuple(r) for r in rows], columns=names or first.__fields__)
    if isinstance(first, dict):
        return pd.DataFrame(rows, columns=names)
    if not isinstance(first, (list, tuple)):
        rows = [(r,) for r in rows]
        first = rows[0]
    names = names or [f"_{i + 1}" for i in range(len(first))]
    cols = list(zip(*rows))
    data = OrderedDict()
    for k, vals in zip(names, cols):
        if any(hasattr(v, "toArray") for v in vals):
            data[k] = pd.Series(list(vals), dtype=object)
        else:
            data[k] = list(vals)
    return pd.DataFrame(data)
