"""SessionConf: string-keyed engine configuration (replaces ``pyspark.SparkConf``).

The reference's Context widget edits a SparkConf as key/value rows with these defaults
(orangecontrib/spark/widgets/data/spark_context.py:38-47): app name, master
``yarn-client``, 8 executors x 4 cores x 8g, driver 4 cores/2g, ``spark.logConf``,
``spark.app.id``.  We keep the same editor UX and accept every ``spark.*`` key, and
map the ones that mean something on one MI355X node:

=============================  ========================================================
key                            meaning here
=============================  ========================================================
``spark.app.name``             session name (logs, trace ranges)
``spark.master``               ``local`` / ``local[*]`` (one process, GPU 0 or CPU),
                               ``spmd`` (one process per GPU launched by torchrun);
                               ``yarn-client`` and other cluster URLs map to auto
``spark.executor.instances``   executors = GPUs: ``auto`` (default, every visible GPU --
                               the reference's 8-executor default on an 8-GPU node) or N;
                               N > 1 outside SPMD spawns a driver + N-executor pool
                               (runtime/executors.py); checked against WORLD_SIZE in SPMD
``o3s.executor.*``             pool knobs: ``pool`` (true: a pool even for 1 GPU),
                               ``timeout`` (per-command watchdog, 21600 s), ``commTimeout``
                               (executor collectives, 120 s), ``stragglerTimeout`` (600 s),
                               ``errorGrace`` (20 s), ``residentModelBytes`` (16 MiB),
                               ``respawn`` (true)
``o3s.device``                 ``auto`` | ``cuda`` | ``cpu``
``o3s.vector.dtype``           feature-matrix storage: ``auto`` (bf16 on GPU, f64 on
                               CPU) | ``bfloat16`` | ``float32`` | ``float64``
``o3s.memory.fraction``        share of free HBM the DataFrame cache may pin (0.85)
``spark.sql.warehouse.dir``    catalog ("Hive") root directory
``o3s.seed``                   default RNG seed (sample/randomSplit/estimators)
=============================  ========================================================
"""
from __future__ import annotations

import os
from collections import OrderedDict

DEFAULTS = OrderedDict([
    ("spark.app.name", "OrangeSpark-AMD"),
    ("spark.master", "local[*]"),
    ("spark.executor.instances", "auto"),
    ("spark.executor.cores", "1"),
    ("spark.executor.memory", "288g"),
    ("spark.driver.cores", "4"),
    ("spark.driver.memory", "16g"),
    ("spark.logConf", "false"),
    ("spark.app.id", "o3s"),
    ("spark.sql.warehouse.dir", "spark-warehouse"),
    ("o3s.device", "auto"),
    ("o3s.vector.dtype", "auto"),
    ("o3s.memory.fraction", "0.85"),
    ("o3s.seed", "42"),
    ("o3s.trace", "false"),                 # runtime/tracing.py phase tracer + roctx ranges
    ("o3s.session.warmup", "auto"),         # runtime/warmup.py: kernel preload; pool workers warm every family
    ("o3s.checkpoint.interval", "0"),       # iterations between checkpoints (needs spark.checkpoint.dir)
    # o3s.comm.timeout (unset): seconds before a hung collective raises -- 1800 for SPMD
    # launches (benchmarks), o3s.executor.commTimeout (120) inside an executor pool
])


def env_key(name: str) -> str:
    """Configuration key of an ``O3S_CONF_<key>`` environment variable: ``__`` separates
    the key's parts (``.``).  A suffix written all in upper case (the shell convention,
    ``O3S_CONF_SPARK__EXECUTOR__INSTANCES``) is lower-cased; any other suffix keeps its
    case, so camelCase keys survive (``O3S_CONF_o3s__executor__commTimeout`` ->
    ``o3s.executor.commTimeout``)."""
    k = name[len("O3S_CONF_"):]
    if k.upper() == k:
        k = k.lower()
    return k.replace("__", ".")


class SessionConf:
    """Mutable string->string map with SparkConf's method names."""

    def __init__(self, loadDefaults: bool = True, _pairs=None):
        self._d: OrderedDict[str, str] = OrderedDict()
        if loadDefaults:
            self._d.update(DEFAULTS)
            for k, v in os.environ.items():
                if k.startswith("O3S_CONF_"):
                    self._d[env_key(k)] = v
        if _pairs:
            for k, v in _pairs:
                self._d[str(k)] = str(v)

    # SparkConf API ------------------------------------------------------------
    def set(self, key: str, value) -> "SessionConf":
        self._d[str(key)] = str(value)
        return self

    def setIfMissing(self, key, value) -> "SessionConf":
        self._d.setdefault(str(key), str(value))
        return self

    def setAll(self, pairs) -> "SessionConf":
        for k, v in pairs:
            self.set(k, v)
        return self

    def setAppName(self, name) -> "SessionConf":
        return self.set("spark.app.name", name)

    def setMaster(self, master) -> "SessionConf":
        return self.set("spark.master", master)

    def get(self, key: str, defaultValue=None):
        return self._d.get(key, defaultValue)

    def getAll(self) -> list[tuple[str, str]]:
        return list(self._d.items())

    def contains(self, key) -> bool:
        return key in self._d

    def remove(self, key) -> "SessionConf":
        self._d.pop(key, None)
        return self

    def toDebugString(self) -> str:
        return "\n".join(f"{k}={v}" for k, v in self._d.items())

    def copy(self) -> "SessionConf":
        return SessionConf(False, self._d.items())

    # typed accessors ----------------------------------------------------------
    def seed(self) -> int:
        return int(self.get("o3s.seed", "42"))

    def memory_fraction(self) -> float:
        return float(self.get("o3s.memory.fraction", "0.85"))

    def master(self) -> str:
        return self.get("spark.master", "local[*]")

    def device_pref(self) -> str:
        return self.get("o3s.device", "auto").lower()

    def vector_dtype(self) -> str:
        return self.get("o3s.vector.dtype", "auto").lower()

    def warehouse(self) -> str:
        return self.get("spark.sql.warehouse.dir", "spark-warehouse")


SparkConf = SessionConf
