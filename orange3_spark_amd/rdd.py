"""RDD API: the ``SparkContext`` half of the session (parallelize / textFile / broadcast /
accumulators) and resilient distributed datasets of Python objects.

The reference hands scripts a live ``SparkContext`` (``sc``) next to the HiveContext
(``hc``): the PySpark Script widget injects both into its console
(orangecontrib/spark/widgets/data/pyspark_script_console.py:331) and its script library is
plain PySpark, so RDD code (``sc.parallelize(...).map(...).reduceByKey(...)``) is part of
what a user of the reference runs.  Spark executes those closures on executors and moves
shuffle blocks over its Netty block manager *(external)*.

Here the driver program runs SPMD on every rank (one process per GPU).  An RDD has
``numPartitions`` partitions; partition ``p`` lives on the rank ``owner(p)`` (``p mod
world`` for source RDDs).  Narrow transformations are lazy per-partition iterator chains
(pipelined, no intermediate lists, errors surface at the action like Spark).  Wide
transformations (``reduceByKey``, ``groupByKey``, ``join``, ``sortBy``, ``distinct``,
``repartition`` ...) hash- or range-partition records and exchange them with ONE
``all_to_all`` of pickled buckets over the communicator (RCCL / gloo), with map-side
combining where Spark does it.  Actions combine per-rank results with an all-gather, so
every rank sees the driver's answer.  Keys are hashed with a process-independent hash
(Python's ``hash(str)`` is salted per process).

These are host-side Python records (the GPU path for tabular data is the columnar
DataFrame; ``DataFrame.rdd`` / ``RDD.toDF`` convert between the two).
"""
from __future__ import annotations

import bisect
import heapq
import itertools
import math
import os
import pickle
import random
import zlib
from collections import defaultdict
from typing import Any, Callable, Iterable, Iterator

__all__ = ["Context", "RDD", "Broadcast", "Accumulator", "AccumulatorParam", "StatCounter", "portable_hash"]


# ----------------------------------------------------------------------------- hashing
def portable_hash(x) -> int:
    """Hash that is identical in every process (ranks must agree on key placement)."""
    if x is None:
        return 0
    if isinstance(x, bool):
        return int(x)
    if isinstance(x, int):
        return x & 0x7FFFFFFFFFFFFFFF
    if isinstance(x, float):
        if x.is_integer():
            return int(x) & 0x7FFFFFFFFFFFFFFF
        return hash(x) & 0x7FFFFFFFFFFFFFFF          # float hashing is not salted
    if isinstance(x, str):
        return zlib.crc32(x.encode("utf-8", "surrogatepass"))
    if isinstance(x, (bytes, bytearray)):
        return zlib.crc32(bytes(x))
    if isinstance(x, tuple):
        h = 0x345678
        for v in x:
            h = ((h ^ portable_hash(v)) * 1000003) & 0xFFFFFFFFFFFF
        return h ^ len(x)
    if isinstance(x, frozenset):
        return sum(portable_hash(v) for v in x) & 0xFFFFFFFFFFFF
    return zlib.crc32(pickle.dumps(x, protocol=4))


# ----------------------------------------------------------------------------- stats
class StatCounter:
    """Count / mean / variance (Welford, mergeable) / min / max of numbers."""

    def __init__(self, values: Iterable = ()):
        self.n = 0
        self.mu = 0.0
        self.m2 = 0.0
        self.maxValue = float("-inf")
        self.minValue = float("inf")
        for v in values:
            self.merge(v)

    def merge(self, value) -> "StatCounter":
        delta = value - self.mu
        self.n += 1
        self.mu += delta / self.n
        self.m2 += delta * (value - self.mu)
        self.maxValue = max(self.maxValue, value)
        self.minValue = min(self.minValue, value)
        return self

    def mergeStats(self, other: "StatCounter") -> "StatCounter":
        if other.n == 0:
            return self
        if self.n == 0:
            self.n, self.mu, self.m2 = other.n, other.mu, other.m2
            self.maxValue, self.minValue = other.maxValue, other.minValue
            return self
        delta = other.mu - self.mu
        n = self.n + other.n
        self.mu += delta * other.n / n
        self.m2 += other.m2 + delta * delta * self.n * other.n / n
        self.n = n
        self.maxValue = max(self.maxValue, other.maxValue)
        self.minValue = min(self.minValue, other.minValue)
        return self

    def count(self):
        return self.n

    def mean(self):
        return self.mu if self.n else float("nan")

    def sum(self):
        return self.n * self.mu

    def min(self):
        return self.minValue

    def max(self):
        return self.maxValue

    def variance(self):
        return self.m2 / self.n if self.n else float("nan")

    def sampleVariance(self):
        return self.m2 / (self.n - 1) if self.n > 1 else float("nan")

    def stdev(self):
        return math.sqrt(self.variance())

    def sampleStdev(self):
        return math.sqrt(self.sampleVariance())

    def asDict(self, sample=False):
        return {"count": self.count(), "mean": self.mean(), "sum": self.sum(), "min": self.min(),
                "max": self.max(), "stdev": self.sampleStdev() if sample else self.stdev(),
                "variance": self.sampleVariance() if sample else self.variance()}

    def __repr__(self):
        return "(count: %s, mean: %s, stdev: %s, max: %s, min: %s)" % (
            self.count(), self.mean(), self.stdev(), self.max(), self.min())


# ----------------------------------------------------------------------------- shared variables
class Broadcast:
    """Read-only value shared by every task.  SPMD: every rank's driver program already
    holds it, so the value is broadcast from rank 0 once to guarantee agreement."""

    def __init__(self, ctx: "Context", value):
        self._ctx = ctx
        self._value = ctx.comm.broadcast_object(value, 0) if ctx.comm.world_size > 1 else value
        self._alive = True

    @property
    def value(self):
        if not self._alive:
            raise RuntimeError("Broadcast variable has been destroyed")
        return self._value

    def unpersist(self, blocking=False):
        pass

    def destroy(self, blocking=False):
        self._alive = False
        self._value = None


class AccumulatorParam:
    def zero(self, value):
        return type(value)() if not isinstance(value, (int, float, complex)) else 0 * value

    def addInPlace(self, value1, value2):
        value1 += value2
        return value1


class Accumulator:
    """Add-only shared variable: tasks ``add`` on the rank that runs them; reading
    ``value`` (a collective, like every driver-side action here) merges all ranks."""

    def __init__(self, ctx: "Context", value, accum_param: AccumulatorParam | None = None):
        self._ctx = ctx
        self._param = accum_param or AccumulatorParam()
        self._initial = value
        self._local = self._param.zero(value)

    def add(self, term):
        self._local = self._param.addInPlace(self._local, term)

    def __iadd__(self, term):
        self.add(term)
        return self

    @property
    def value(self):
        parts = self._ctx.comm.all_gather_object(self._local) if self._ctx.comm.world_size > 1 else [self._local]
        v = _copy(self._initial)
        for p in parts:
            v = self._param.addInPlace(v, p)
        return v

    @value.setter
    def value(self, v):
        self._initial = v
        self._local = self._param.zero(v)

    def __repr__(self):
        return f"Accumulator<value={self._initial}+local {self._local}>"


# ----------------------------------------------------------------------------- RDD
_RDD_IDS = itertools.count()


class RDD:
    """A partitioned collection of Python objects (see module docstring)."""

    def __init__(self, ctx: "Context", num_partitions: int, compute: Callable[[int], Iterable],
                 owner: Callable[[int], int] | None = None, deps: tuple = (), prepare: Callable | None = None,
                 partitioner=None):
        self.ctx = ctx
        self._n = int(num_partitions)
        self._compute = compute
        w = ctx.comm.world_size
        self._owner = owner or (lambda p: p % w)
        self._deps = deps
        self._prep = prepare
        self._prepared = prepare is None
        self.partitioner = partitioner
        self._cached = None
        self._id = next(_RDD_IDS)
        self._name = None

    # -- plumbing ----------------------------------------------------------------------
    @property
    def context(self):
        return self.ctx

    def id(self):
        return self._id

    def name(self):
        return self._name

    def setName(self, name):
        self._name = name
        return self

    def getNumPartitions(self) -> int:
        return self._n

    def _local_pids(self) -> list[int]:
        r = self.ctx.comm.rank
        return [p for p in range(self._n) if self._owner(p) == r]

    def _prepare(self):
        for d in self._deps:
            d._prepare()
        if not self._prepared:
            self._prep()
            self._prepared = True

    def _iter(self, pid: int) -> Iterator:
        if self._cached is not None:
            return iter(self._cached[pid])
        return iter(self._compute(pid))

    def _local_partitions(self) -> dict[int, list]:
        self._prepare()
        return {p: list(self._iter(p)) for p in self._local_pids()}

    def _gather(self, local_result):
        c = self.ctx.comm
        return c.all_gather_object(local_result) if c.world_size > 1 else [local_result]

    def _derive(self, f: Callable[[int, Iterator], Iterable], preserves_partitioning=False) -> "RDD":
        parent = self
        return RDD(self.ctx, self._n, lambda p: f(p, parent._iter(p)), self._owner, (self,),
                   partitioner=self.partitioner if preserves_partitioning else None)

    # -- persistence (partitions are host lists; cache materialises them once) ------------
    def cache(self):
        self._prepare()
        if self._cached is None:
            self._cached = {p: list(self._compute(p)) for p in self._local_pids()}
        return self

    def persist(self, storageLevel=None):
        return self.cache()

    def unpersist(self, blocking=False):
        self._cached = None
        return self

    @property
    def is_cached(self):
        return self._cached is not None

    def checkpoint(self):
        self.cache()

    def localCheckpoint(self):
        self.cache()

    def isCheckpointed(self):
        return self._cached is not None

    def getStorageLevel(self):
        return "MEMORY_ONLY" if self._cached is not None else "NONE"

    def toDebugString(self):
        return f"({self._n}) RDD[{self._id}] {self._name or ''} deps={[d._id for d in self._deps]}".encode()

    # -- narrow transformations ------------------------------------------------------------
    def map(self, f, preservesPartitioning=False):
        return self._derive(lambda p, it: map(f, it), preservesPartitioning)

    def flatMap(self, f, preservesPartitioning=False):
        return self._derive(lambda p, it: itertools.chain.from_iterable(map(f, it)), preservesPartitioning)

    def filter(self, f):
        return self._derive(lambda p, it: filter(f, it), True)

    def mapPartitions(self, f, preservesPartitioning=False):
        return self._derive(lambda p, it: f(it), preservesPartitioning)

    def mapPartitionsWithIndex(self, f, preservesPartitioning=False):
        return self._derive(f, preservesPartitioning)

    mapPartitionsWithSplit = mapPartitionsWithIndex

    def glom(self):
        return self._derive(lambda p, it: [list(it)])

    def mapValues(self, f):
        return self._derive(lambda p, it: ((k, f(v)) for k, v in it), True)

    def flatMapValues(self, f):
        return self._derive(lambda p, it: ((k, x) for k, v in it for x in f(v)), True)

    def keys(self):
        return self.map(lambda kv: kv[0])

    def values(self):
        return self.map(lambda kv: kv[1])

    def keyBy(self, f):
        return self.map(lambda x: (f(x), x))

    def zipWithUniqueId(self):
        n = self._n
        return self._derive(lambda p, it: ((x, i * n + p) for i, x in enumerate(it)))

    def zipWithIndex(self):
        """Global index in partition order (one count job, like Spark)."""
        sizes = self._partition_sizes()
        offs = [0] * (self._n + 1)
        for p in range(self._n):
            offs[p + 1] = offs[p] + sizes[p]
        return self._derive(lambda p, it: ((x, offs[p] + i) for i, x in enumerate(it)))

    def _partition_sizes(self) -> list[int]:
        local = {p: sum(1 for _ in self._iter(p)) for p in self._local_pids_prepared()}
        sizes = [0] * self._n
        for part in self._gather(local):
            for p, c in part.items():
                sizes[p] = c
        return sizes

    def _local_pids_prepared(self):
        self._prepare()
        return self._local_pids()

    def sample(self, withReplacement, fraction, seed=None):
        seed = random.randrange(1 << 30) if seed is None else seed

        def f(p, it):
            rng = random.Random(seed * 1000003 + p)
            for x in it:
                if withReplacement:
                    k = _poisson(rng, fraction)
                    for _ in range(k):
                        yield x
                elif rng.random() < fraction:
                    yield x
        return self._derive(f, True)

    def randomSplit(self, weights, seed=None):
        s = float(sum(weights))
        bounds = list(itertools.accumulate(w / s for w in weights))
        seed = random.randrange(1 << 30) if seed is None else seed
        out = []
        for i in range(len(weights)):
            lo = bounds[i - 1] if i else 0.0
            hi = bounds[i]

            def f(p, it, lo=lo, hi=hi):
                rng = random.Random(seed * 1000003 + p)
                for x in it:
                    u = rng.random()
                    if lo <= u < hi:
                        yield x
            out.append(self._derive(f, True))
        return out

    def union(self, other: "RDD") -> "RDD":
        a, b = self, other
        na = a._n
        return RDD(self.ctx, a._n + b._n, lambda p: a._iter(p) if p < na else b._iter(p - na),
                   lambda p: a._owner(p) if p < na else b._owner(p - na), (a, b))

    def __add__(self, other):
        return self.union(other)

    def cartesian(self, other: "RDD") -> "RDD":
        state = {}
        parent = self

        def prep():
            state["other"] = [x for part in other._gather(list(itertools.chain.from_iterable(
                other._local_partitions().values()))) for x in part]
        return RDD(self.ctx, self._n, lambda p: ((x, y) for x in parent._iter(p) for y in state["other"]),
                   self._owner, (self, other), prep)

    def pipe(self, command, env=None, checkCode=False):
        import subprocess

        def f(p, it):
            data = "".join(f"{x}\n" for x in it).encode()
            r = subprocess.run(command, shell=True, input=data, capture_output=True, env=env)
            if checkCode and r.returncode:
                raise RuntimeError(f"pipe command exited with {r.returncode}")
            return r.stdout.decode().splitlines()
        return self._derive(f)

    # -- shuffles ------------------------------------------------------------------------
    def _shuffle(self, num_partitions: int, records: Callable[[int, Iterator], Iterable[tuple[int, Any]]],
                 partitioner=None) -> "RDD":
        """Route ``records(pid, it) -> (target_pid, record)`` to ``target_pid``'s owner with one
        all-to-all; the result's partition p holds its records in source-partition order."""
        ctx, parent, n = self.ctx, self, int(num_partitions)
        w, r = ctx.comm.world_size, ctx.comm.rank
        state = {}

        def prep():
            buckets = [defaultdict(list) for _ in range(w)]
            for p in parent._local_pids():
                for tp, rec in records(p, parent._iter(p)):
                    buckets[tp % w][tp].append(rec)
            recv = ctx.comm.all_to_all_object([dict(b) for b in buckets]) if w > 1 else [dict(buckets[0])]
            parts = defaultdict(list)
            for src in recv:
                for tp, recs in src.items():
                    parts[tp].extend(recs)
            state["parts"] = parts
            state["rank"] = r
        return RDD(ctx, n, lambda p: state["parts"].get(p, ()), None, (self,), prep, partitioner)

    def partitionBy(self, numPartitions, partitionFunc=portable_hash):
        n = int(numPartitions)
        return self._shuffle(n, lambda p, it: ((partitionFunc(kv[0]) % n, kv) for kv in it), ("hash", n))

    def repartition(self, numPartitions):
        n = int(numPartitions)
        return self._shuffle(n, lambda p, it: (((p + i) % n, x) for i, x in enumerate(it)))

    def coalesce(self, numPartitions, shuffle=False):
        n = max(1, int(numPartitions))
        if n >= self._n and not shuffle:
            return self
        return self._shuffle(n, lambda p, it: ((p * n // max(self._n, 1), x) for x in it))

    def combineByKey(self, createCombiner, mergeValue, mergeCombiners, numPartitions=None,
                     partitionFunc=portable_hash):
        n = int(numPartitions or self._n)

        def local_combine(p, it):
            acc = {}
            for k, v in it:
                acc[k] = mergeValue(acc[k], v) if k in acc else createCombiner(v)
            return ((partitionFunc(k) % n, (k, c)) for k, c in acc.items())
        shuffled = self._shuffle(n, local_combine, ("hash", n))

        def merge(p, it):
            acc = {}
            for k, c in it:
                acc[k] = mergeCombiners(acc[k], c) if k in acc else c
            return iter(acc.items())
        return shuffled._derive(merge, True)

    def reduceByKey(self, func, numPartitions=None, partitionFunc=portable_hash):
        return self.combineByKey(lambda v: v, func, func, numPartitions, partitionFunc)

    def reduceByKeyLocally(self, func):
        out = {}
        for k, v in self.reduceByKey(func).collect():
            out[k] = v
        return out

    def foldByKey(self, zeroValue, func, numPartitions=None, partitionFunc=portable_hash):
        return self.combineByKey(lambda v: func(_copy(zeroValue), v), func, func, numPartitions, partitionFunc)

    def aggregateByKey(self, zeroValue, seqFunc, combFunc, numPartitions=None, partitionFunc=portable_hash):
        return self.combineByKey(lambda v: seqFunc(_copy(zeroValue), v), seqFunc, combFunc, numPartitions,
                                 partitionFunc)

    def groupByKey(self, numPartitions=None, partitionFunc=portable_hash):
        n = int(numPartitions or self._n)
        shuffled = self.partitionBy(n, partitionFunc)

        def group(p, it):
            acc = {}
            for k, v in it:
                acc.setdefault(k, []).append(v)
            return iter(acc.items())
        return shuffled._derive(group, True)

    def groupBy(self, f, numPartitions=None, partitionFunc=portable_hash):
        return self.map(lambda x: (f(x), x)).groupByKey(numPartitions, partitionFunc)

    def countByKey(self):
        return dict(self.map(lambda kv: (kv[0], 1)).reduceByKey(lambda a, b: a + b).collect())

    def countByValue(self):
        return dict(self.map(lambda x: (x, 1)).reduceByKey(lambda a, b: a + b).collect())

    def distinct(self, numPartitions=None):
        return self.map(lambda x: (x, None)).reduceByKey(lambda a, b: a, numPartitions).keys()

    def cogroup(self, *others, numPartitions=None):
        rdds = (self,) + tuple(others)
        n = int(numPartitions or max(r._n for r in rdds))
        tagged = None
        for i, r in enumerate(rdds):
            t = r.map(lambda kv, i=i: (kv[0], (i, kv[1])))
            tagged = t if tagged is None else tagged.union(t)
        shuffled = tagged.partitionBy(n)
        m = len(rdds)

        def group(p, it):
            acc = {}
            for k, (i, v) in it:
                acc.setdefault(k, tuple([] for _ in range(m)))[i].append(v)
            return iter(acc.items())
        return shuffled._derive(group, True)

    def groupWith(self, other, *others):
        return self.cogroup(other, *others)

    def join(self, other, numPartitions=None):
        return self.cogroup(other, numPartitions=numPartitions).flatMapValues(
            lambda vs: [(a, b) for a in vs[0] for b in vs[1]])

    def leftOuterJoin(self, other, numPartitions=None):
        return self.cogroup(other, numPartitions=numPartitions).flatMapValues(
            lambda vs: [(a, b) for a in vs[0] for b in (vs[1] or [None])])

    def rightOuterJoin(self, other, numPartitions=None):
        return self.cogroup(other, numPartitions=numPartitions).flatMapValues(
            lambda vs: [(a, b) for a in (vs[0] or [None]) for b in vs[1]])

    def fullOuterJoin(self, other, numPartitions=None):
        return self.cogroup(other, numPartitions=numPartitions).flatMapValues(
            lambda vs: [(a, b) for a in (vs[0] or [None]) for b in (vs[1] or [None])])

    def subtractByKey(self, other, numPartitions=None):
        return self.cogroup(other, numPartitions=numPartitions).filter(
            lambda kv: kv[1][0] and not kv[1][1]).flatMapValues(lambda vs: vs[0])

    def subtract(self, other, numPartitions=None):
        return self.map(lambda x: (x, True)).subtractByKey(other.map(lambda x: (x, True)), numPartitions).keys()

    def intersection(self, other):
        return self.map(lambda x: (x, None)).cogroup(other.map(lambda x: (x, None))).filter(
            lambda kv: kv[1][0] and kv[1][1]).keys()

    def sortByKey(self, ascending=True, numPartitions=None, keyfunc=lambda k: k):
        """Range partitioning from a key sample (bounds agreed by all ranks), then a local sort."""
        n = int(numPartitions or self._n)
        parent = self
        state = {}

        def prep_bounds():
            sample = []
            for p in parent._local_pids():
                part = [keyfunc(kv[0]) for kv in parent._iter(p)]
                step = max(1, len(part) // 64)
                sample.extend(part[::step])
            allk = sorted(itertools.chain.from_iterable(parent._gather(sample)))
            state["bounds"] = [allk[len(allk) * (i + 1) // n] for i in range(n - 1)] if allk and n > 1 else []

        bounded = RDD(self.ctx, self._n, self._iter, self._owner, (self,), prep_bounds)

        def route(p, it):
            b = state["bounds"]
            for kv in it:
                i = bisect.bisect_left(b, keyfunc(kv[0]))
                yield (i if ascending else n - 1 - i), kv
        shuffled = bounded._shuffle(n, route, ("range", n))
        return shuffled._derive(lambda p, it: iter(sorted(it, key=lambda kv: keyfunc(kv[0]), reverse=not ascending)),
                                True)

    def sortBy(self, keyfunc, ascending=True, numPartitions=None):
        return self.keyBy(keyfunc).sortByKey(ascending, numPartitions).values()

    # -- actions -------------------------------------------------------------------------
    def collect(self) -> list:
        local = self._local_partitions()
        merged = {}
        for part in self._gather(local):
            merged.update(part)
        return [x for p in range(self._n) for x in merged.get(p, ())]

    def collectAsMap(self) -> dict:
        return dict(self.collect())

    def toLocalIterator(self, prefetchPartitions=False):
        return iter(self.collect())

    def count(self) -> int:
        self._prepare()
        return sum(self._gather(sum(sum(1 for _ in self._iter(p)) for p in self._local_pids())))

    def countApprox(self, timeout, confidence=0.95):
        return self.count()

    def isEmpty(self) -> bool:
        return self.count() == 0

    def first(self):
        r = self.take(1)
        if not r:
            raise ValueError("RDD is empty")
        return r[0]

    def take(self, num: int) -> list:
        self._prepare()
        local = {p: list(itertools.islice(self._iter(p), num)) for p in self._local_pids()}
        merged = {}
        for part in self._gather(local):
            merged.update(part)
        out = []
        for p in range(self._n):
            out.extend(merged.get(p, ()))
            if len(out) >= num:
                break
        return out[:num]

    def top(self, num, key=None):
        self._prepare()
        local = heapq.nlargest(num, (x for p in self._local_pids() for x in self._iter(p)), key=key)
        return heapq.nlargest(num, itertools.chain.from_iterable(self._gather(local)), key=key)

    def takeOrdered(self, num, key=None):
        self._prepare()
        local = heapq.nsmallest(num, (x for p in self._local_pids() for x in self._iter(p)), key=key)
        return heapq.nsmallest(num, itertools.chain.from_iterable(self._gather(local)), key=key)

    def takeSample(self, withReplacement, num, seed=None):
        data = self.collect()
        rng = random.Random(seed)
        if withReplacement:
            return [rng.choice(data) for _ in range(num)] if data else []
        return rng.sample(data, min(num, len(data)))

    def reduce(self, f):
        self._prepare()
        sentinel = object()
        local = sentinel
        for p in self._local_pids():
            for x in self._iter(p):
                local = x if local is sentinel else f(local, x)
        vals = [v for v in self._gather(None if local is sentinel else (local,)) if v is not None]
        if not vals:
            raise ValueError("Can not reduce() empty RDD")
        acc = vals[0][0]
        for v in vals[1:]:
            acc = f(acc, v[0])
        return acc

    def treeReduce(self, f, depth=2):
        return self.reduce(f)

    def fold(self, zeroValue, op):
        self._prepare()
        local = [_fold(op, _copy(zeroValue), self._iter(p)) for p in self._local_pids()]
        return _fold(op, zeroValue, itertools.chain.from_iterable(self._gather(local)))

    def aggregate(self, zeroValue, seqOp, combOp):
        self._prepare()
        local = [_fold(seqOp, _copy(zeroValue), self._iter(p)) for p in self._local_pids()]
        return _fold(combOp, zeroValue, itertools.chain.from_iterable(self._gather(local)))

    def treeAggregate(self, zeroValue, seqOp, combOp, depth=2):
        return self.aggregate(zeroValue, seqOp, combOp)

    def sum(self):
        return self.fold(0, lambda a, b: a + b)

    def stats(self) -> StatCounter:
        self._prepare()
        local = StatCounter(x for p in self._local_pids() for x in self._iter(p))
        out = StatCounter()
        for s in self._gather(local):
            out.mergeStats(s)
        return out

    def mean(self):
        return self.stats().mean()

    def variance(self):
        return self.stats().variance()

    def stdev(self):
        return self.stats().stdev()

    def sampleVariance(self):
        return self.stats().sampleVariance()

    def sampleStdev(self):
        return self.stats().sampleStdev()

    def max(self, key=None):
        return self.reduce(lambda a, b: b if (key(b) if key else b) > (key(a) if key else a) else a)

    def min(self, key=None):
        return self.reduce(lambda a, b: b if (key(b) if key else b) < (key(a) if key else a) else a)

    def histogram(self, buckets):
        if isinstance(buckets, int):
            st = self.stats()
            lo, hi = st.min(), st.max()
            if lo == hi:
                edges = [lo, hi]
            else:
                edges = [lo + (hi - lo) * i / buckets for i in range(buckets)] + [hi]
        else:
            edges = list(buckets)
        nb = len(edges) - 1

        def count(it):
            c = [0] * nb
            for x in it:
                if edges[0] <= x <= edges[-1]:
                    i = min(bisect.bisect_right(edges, x) - 1, nb - 1)
                    c[i] += 1
            return c
        self._prepare()
        local = count(x for p in self._local_pids() for x in self._iter(p))
        tot = [0] * nb
        for c in self._gather(local):
            tot = [a + b for a, b in zip(tot, c)]
        return edges, tot

    def lookup(self, key):
        return self.filter(lambda kv: kv[0] == key).values().collect()

    def foreach(self, f):
        self._prepare()
        for p in self._local_pids():
            for x in self._iter(p):
                f(x)

    def foreachPartition(self, f):
        self._prepare()
        for p in self._local_pids():
            f(self._iter(p))

    def saveAsTextFile(self, path, compressionCodecClass=None):
        """One ``part-NNNNN`` file per partition, written by the partition's owner, plus
        ``_SUCCESS`` (Hadoop layout)."""
        self._prepare()
        os.makedirs(path, exist_ok=True)
        for p in self._local_pids():
            with open(os.path.join(path, f"part-{p:05d}"), "w") as f:
                for x in self._iter(p):
                    f.write(f"{x}\n")
        self.ctx.comm.barrier()
        if self.ctx.comm.rank == 0:
            open(os.path.join(path, "_SUCCESS"), "w").close()

    def saveAsPickleFile(self, path, batchSize=10):
        self._prepare()
        os.makedirs(path, exist_ok=True)
        for p in self._local_pids():
            with open(os.path.join(path, f"part-{p:05d}.pkl"), "wb") as f:
                pickle.dump(list(self._iter(p)), f, protocol=4)
        self.ctx.comm.barrier()

    # -- DataFrame bridge ------------------------------------------------------------------
    def toDF(self, schema=None, sampleRatio=None):
        """This rank's records become this rank's rows of a DataFrame (no data movement)."""
        import pandas as pd
        from .frame.dataframe import DataFrame, Row
        from .session import _rows_to_pandas, _schema_names
        rows = [x for part in self._local_partitions().values() for x in part]
        names = _schema_names(schema)
        if names is None:
            probe = next((x for x in rows[:1]), None)
            seen = [n for n in self._gather(list(probe._fields) if isinstance(probe, Row) and hasattr(probe, "_fields")
                                            else (list(probe.keys()) if isinstance(probe, dict) else
                                                  (len(probe) if isinstance(probe, (tuple, list)) else None)))
                    if n is not None]
            first = seen[0] if seen else None
            names = first if isinstance(first, list) else ([f"_{i + 1}" for i in range(first)] if first else None)
        if not rows:
            if not names:
                return DataFrame(self.ctx.session, {}, 0)
            pdf = pd.DataFrame({n: pd.Series([], dtype=float) for n in names})
        else:
            pdf = _rows_to_pandas(rows, names)
        local = self.ctx.session.local_view().createDataFrame(pdf, schema if not isinstance(schema, (list, tuple))
                                                              else None)
        return DataFrame(self.ctx.session, local._cols, len(local))

    def __repr__(self):
        return f"RDD[{self._id}] ({self._n} partitions)"


def _copy(v):
    import copy
    return copy.deepcopy(v)


def _fold(op, zero, it):
    acc = zero
    for x in it:
        acc = op(acc, x)
    return acc


def _poisson(rng: random.Random, lam: float) -> int:
    l, k, p = math.exp(-lam), 0, 1.0
    while True:
        p *= rng.random()
        if p <= l:
            return k
        k += 1


# ----------------------------------------------------------------------------- context
class Context:
    """``SparkContext`` view of a Session (``session.sparkContext``; the widgets' ``sc``).
    Unknown attributes fall through to the session, so ``sc.sql`` etc. keep working."""

    def __init__(self, session):
        self.session = session

    @property
    def comm(self):
        return self.session.comm

    def __getattr__(self, item):
        if item == "session":
            raise AttributeError(item)
        return getattr(self.session, item)

    # -- configuration ------------------------------------------------------------------
    @property
    def defaultParallelism(self) -> int:
        return max(2, self.comm.world_size * 2)

    @property
    def defaultMinPartitions(self) -> int:
        return min(self.defaultParallelism, 2)

    @property
    def version(self):
        from . import __version__
        return __version__

    @property
    def master(self):
        return self.session.conf.get("spark.master")

    @property
    def appName(self):
        return self.session.conf.get("spark.app.name")

    @property
    def applicationId(self):
        return self.session.conf.get("spark.app.id", "o3s-app")

    @property
    def startTime(self):
        return getattr(self.session, "_start_time", 0)

    def getConf(self):
        return self.session.conf

    def setLogLevel(self, logLevel: str):
        import logging
        logging.getLogger("orange3_spark_amd").setLevel(getattr(logging, str(logLevel).upper(), logging.INFO))

    def setJobGroup(self, groupId, description, interruptOnCancel=False):
        pass

    def setLocalProperty(self, key, value):
        self.session.conf.set(key, value)

    def getLocalProperty(self, key):
        return self.session.conf.get(key)

    # -- RDD creation ---------------------------------------------------------------------
    def parallelize(self, c: Iterable, numSlices: int | None = None) -> RDD:
        """Every rank holds ``c`` (SPMD driver); partition p keeps slice p of it."""
        data = list(c) if not isinstance(c, range) else c
        n = int(numSlices or self.defaultParallelism)
        size = len(data)
        bounds = [size * i // n for i in range(n + 1)]
        if isinstance(data, range):
            return RDD(self, n, lambda p: data[bounds[p]:bounds[p + 1]])
        return RDD(self, n, lambda p: data[bounds[p]:bounds[p + 1]])

    def range(self, start, end=None, step=1, numSlices=None) -> RDD:
        if end is None:
            start, end = 0, start
        return self.parallelize(range(start, end, step), numSlices)

    def emptyRDD(self) -> RDD:
        return RDD(self, 0, lambda p: ())

    def union(self, rdds) -> RDD:
        rdds = list(rdds)
        out = rdds[0]
        for r in rdds[1:]:
            out = out.union(r)
        return out

    def textFile(self, name: str, minPartitions: int | None = None, use_unicode=True) -> RDD:
        """Lines of a file / directory of files / glob; each partition reads its share of
        lines (files are visible to every rank on a node)."""
        files = _expand_paths(name)
        n = int(minPartitions or self.defaultMinPartitions)

        def lines():
            out = []
            for f in files:
                with open(f, "r", encoding="utf-8", errors="replace") as fh:
                    out.extend(line.rstrip("\n").rstrip("\r") for line in fh)
            return out
        cache = {}

        def compute(p):
            if "l" not in cache:
                cache["l"] = lines()
            data = cache["l"]
            return data[len(data) * p // n: len(data) * (p + 1) // n]
        return RDD(self, n, compute)

    def wholeTextFiles(self, path: str, minPartitions: int | None = None, use_unicode=True) -> RDD:
        files = _expand_paths(path)
        n = max(1, min(int(minPartitions or self.defaultMinPartitions), max(len(files), 1)))

        def compute(p):
            out = []
            for f in files[len(files) * p // n: len(files) * (p + 1) // n]:
                with open(f, "r", encoding="utf-8", errors="replace") as fh:
                    out.append((f, fh.read()))
            return out
        return RDD(self, n, compute)

    def pickleFile(self, name: str, minPartitions=None) -> RDD:
        files = sorted(f for f in _expand_paths(name) if f.endswith(".pkl"))
        n = max(1, len(files))

        def compute(p):
            if not files:
                return []
            with open(files[p], "rb") as fh:
                return pickle.load(fh)             # files this framework wrote (saveAsPickleFile)
        return RDD(self, n, compute)

    # -- shared variables --------------------------------------------------------------------
    def broadcast(self, value) -> Broadcast:
        return Broadcast(self, value)

    def accumulator(self, value, accum_param: AccumulatorParam | None = None) -> Accumulator:
        return Accumulator(self, value, accum_param)

    def stop(self):
        self.session.stop()

    def __repr__(self):
        return f"<SparkContext master={self.master} appName={self.appName} world={self.comm.world_size}>"


def _expand_paths(name: str) -> list[str]:
    import glob
    out = []
    for part in str(name).split(","):
        part = part.strip()
        if part.startswith("file://"):
            part = part[len("file://"):]
        if os.path.isdir(part):
            out.extend(sorted(os.path.join(part, f) for f in os.listdir(part)
                              if not f.startswith(("_", ".")) and os.path.isfile(os.path.join(part, f))))
        else:
            hits = sorted(glob.glob(part))
            out.extend(hits if hits else [part])
    return out
