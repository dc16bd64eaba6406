"""Frequent pattern mining (``pyspark.ml.fpm``): FPGrowth, PrefixSpan.

Transactions are gathered from all ranks and mined on the host (pattern mining is
branchy, pointer-chasing work with no dense kernel); item frequencies are counted with an
all-reduced dictionary first so infrequent items are pruned before the gather.
"""
from __future__ import annotations

from collections import Counter, OrderedDict, defaultdict
from itertools import combinations

import numpy as np
import torch

from ..frame import column as C
from ..frame.dataframe import DataFrame
from .base import Estimator, Model
from .param import HasPredictionCol, TypeConverters, keyword_only, shared
from .util import MLReadable, MLWritable, register


class _FPGrowthParams(HasPredictionCol):
    itemsCol = shared("itemsCol", "items column name", TypeConverters.toString)
    minSupport = shared("minSupport", "Minimal support level of the frequent pattern. [0.0, 1.0]. Any pattern that "
                                      "appears more than (minSupport * size-of-the-dataset) times will be output in "
                                      "the frequent itemsets.", TypeConverters.toFloat)
    numPartitions = shared("numPartitions", "Number of partitions (at least 1) used by parallel FP-growth. By "
                                            "default the param is not set, and partition number of the input "
                                            "dataset is used.", TypeConverters.toInt)
    minConfidence = shared("minConfidence", "Minimal confidence for generating Association Rule. [0.0, 1.0]. "
                                            "minConfidence will not affect the mining for frequent itemsets, but "
                                            "will affect the association rules generation.", TypeConverters.toFloat)

    def __init__(self):
        super().__init__()
        self._setDefault(itemsCol="items", minSupport=0.3, minConfidence=0.8)


def _fpgrowth(transactions: list, min_count: int) -> dict:
    """Classic FP-growth: returns {frozenset(itemset): count}."""
    counts = Counter(i for t in transactions for i in set(t))
    freq = {i: c for i, c in counts.items() if c >= min_count}
    order = {i: (-c, str(i)) for i, c in freq.items()}

    class Node:
        __slots__ = ("item", "count", "parent", "children")

        def __init__(self, item, parent):
            self.item, self.count, self.parent, self.children = item, 0, parent, {}

    def build(weighted):
        root = Node(None, None)
        header = defaultdict(list)
        for items, w in weighted:
            node = root
            for it in items:
                ch = node.children.get(it)
                if ch is None:
                    ch = Node(it, node)
                    node.children[it] = ch
                    header[it].append(ch)
                ch.count += w
                node = ch
        return header

    out = {}

    def mine(weighted, suffix):
        cnt = Counter()
        for items, w in weighted:
            for it in items:
                cnt[it] += w
        local = {i for i, c in cnt.items() if c >= min_count}
        trimmed = [(sorted([i for i in items if i in local], key=lambda x: order[x]), w) for items, w in weighted]
        header = build(trimmed)
        for it in sorted(local, key=lambda x: order[x], reverse=True):
            new = suffix | {it}
            out[frozenset(new)] = cnt[it]
            cond = []
            for node in header[it]:
                path, p = [], node.parent
                while p is not None and p.item is not None:
                    path.append(p.item)
                    p = p.parent
                if path:
                    cond.append((path[::-1], node.count))
            if cond:
                mine(cond, new)

    mine([([i for i in set(t) if i in freq], 1) for t in transactions], frozenset())
    return out


@register("org.apache.spark.ml.fpm.FPGrowth")
class FPGrowth(Estimator, _FPGrowthParams, MLWritable, MLReadable):
    """A parallel FP-growth algorithm to mine frequent itemsets."""

    @keyword_only
    def __init__(self, *, minSupport=0.3, minConfidence=0.8, itemsCol="items", predictionCol="prediction",
                 numPartitions=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        vals = df.column_data(self.getOrDefault(self.itemsCol)).values
        parts = df.comm.all_gather_object([list(v) if v is not None else [] for v in vals])
        trans = [t for p in parts for t in p]
        n = len(trans)
        min_count = int(np.ceil(self.getOrDefault(self.minSupport) * n))
        return FPGrowthModel._from(_fpgrowth(trans, max(min_count, 1)), n)._with_parent(self)


@register("org.apache.spark.ml.fpm.FPGrowthModel")
class FPGrowthModel(Model, _FPGrowthParams, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self._sets, self._n = {}, 0

    @classmethod
    def _from(cls, sets, n):
        m = cls()
        m._sets, m._n = sets, n
        return m

    def _session(self):
        from ..session import Session
        return Session.getOrCreate()

    @property
    def freqItemsets(self):
        items = sorted(self._sets.items(), key=lambda kv: (-kv[1], sorted(map(str, kv[0]))))
        arr = np.empty(len(items), dtype=object)
        arr[:] = [sorted(k, key=str) for k, _ in items]
        s = self._session()
        return DataFrame(s.local_view(), OrderedDict(items=C.ArrayColumn(arr), freq=C.NumericColumn(
            torch.tensor([v for _, v in items], dtype=torch.int64, device=s.device))))

    def _rules(self):
        mc = self.getOrDefault(self.minConfidence)
        rules = []
        for s, c in self._sets.items():
            if len(s) < 2:
                continue
            for k in range(1, len(s)):
                for ante in combinations(sorted(s, key=str), k):
                    a = frozenset(ante)
                    conf = c / self._sets[a]
                    if conf >= mc:
                        cons = s - a
                        if len(cons) != 1:
                            continue
                        lift = conf / (self._sets[cons] / self._n)
                        rules.append((sorted(a, key=str), sorted(cons, key=str), conf, lift, c / self._n))
        return rules

    @property
    def associationRules(self):
        rules = self._rules()
        s = self._session()
        ante = np.empty(len(rules), dtype=object)
        ante[:] = [r[0] for r in rules]
        cons = np.empty(len(rules), dtype=object)
        cons[:] = [r[1] for r in rules]
        cols = OrderedDict(antecedent=C.ArrayColumn(ante), consequent=C.ArrayColumn(cons),
                           confidence=C.NumericColumn(torch.tensor([r[2] for r in rules], dtype=torch.float64)),
                           lift=C.NumericColumn(torch.tensor([r[3] for r in rules], dtype=torch.float64)),
                           support=C.NumericColumn(torch.tensor([r[4] for r in rules], dtype=torch.float64)))
        return DataFrame(s.local_view(), cols)

    def _transform(self, df):
        rules = self._rules()
        vals = df.column_data(self.getOrDefault(self.itemsCol)).values
        preds = []
        for v in vals:
            have = set(v or [])
            p = []
            for a, c, *_ in rules:
                if set(a) <= have:
                    for x in c:
                        if x not in have and x not in p:
                            p.append(x)
            preds.append(p)
        arr = np.empty(len(preds), dtype=object)
        arr[:] = preds
        return df.withColumnData(self.getOrDefault(self.predictionCol), C.ArrayColumn(arr))


class PrefixSpan:
    """A parallel PrefixSpan algorithm to mine frequent sequential patterns."""

    @keyword_only
    def __init__(self, *, minSupport=0.1, maxPatternLength=10, maxLocalProjDBSize=32000000, sequenceCol="sequence"):
        self.minSupport, self.maxPatternLength = minSupport, maxPatternLength
        self.maxLocalProjDBSize, self.sequenceCol = maxLocalProjDBSize, sequenceCol

    def findFrequentSequentialPatterns(self, dataset):
        from ..runtime.executors import remote_pool_of
        pool = remote_pool_of(dataset)
        if pool is not None:                 # driver of an executor pool: run on the executors
            return pool.call(self, "findFrequentSequentialPatterns", (dataset,))
        return self._find_patterns(dataset)

    def _find_patterns(self, dataset):
        vals = dataset.column_data(self.sequenceCol).values
        parts = dataset.comm.all_gather_object([list(v) for v in vals])
        seqs = [[frozenset(e) for e in s] for p in parts for s in p]
        n = len(seqs)
        min_count = max(1, int(np.ceil(self.minSupport * n)))
        out = []

        def project(db, prefix, length):
            if length >= self.maxPatternLength:
                return
            cnt = Counter()
            for seq, start in db:
                seen = set()
                for e in seq[start:]:
                    for it in e:
                        if it not in seen:
                            seen.add(it)
                            cnt[it] += 1
            for it, c in sorted(cnt.items(), key=lambda kv: str(kv[0])):
                if c < min_count:
                    continue
                pat = prefix + [[it]]
                out.append((pat, c))
                newdb = []
                for seq, start in db:
                    for j in range(start, len(seq)):
                        if it in seq[j]:
                            newdb.append((seq, j + 1))
                            break
                project(newdb, pat, length + 1)
        project([(s, 0) for s in seqs], [], 0)
        s = dataset.session
        arr = np.empty(len(out), dtype=object)
        arr[:] = [p for p, _ in out]
        return DataFrame(s.local_view(), OrderedDict(sequence=C.ArrayColumn(arr), freq=C.NumericColumn(
            torch.tensor([c for _, c in out], dtype=torch.int64))))
