"""Recommendation (``pyspark.ml.recommendation`` surface): ALS / ALSModel.

Reached in the reference through the Recommendation widget
(orangecontrib/spark/widgets/ml/spark_ml_recommendation.py:15).
"""
from __future__ import annotations

import os
from collections import OrderedDict

import numpy as np
import torch

from ..frame import column as C
from ..frame.dataframe import DataFrame, Row
from ..models import als as ALSE
from . import common as U
from .base import Estimator, Model
from .param import (HasBlockSize, HasCheckpointInterval, HasMaxIter, HasPredictionCol, HasRegParam, HasSeed,
                    TypeConverters, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, register, save_metadata


class _ALSModelParams(HasPredictionCol, HasBlockSize):
    userCol = shared("userCol", "column name for user ids. Ids must be within the integer value range.",
                     TypeConverters.toString)
    itemCol = shared("itemCol", "column name for item ids. Ids must be within the integer value range.",
                     TypeConverters.toString)
    coldStartStrategy = shared("coldStartStrategy", "strategy for dealing with unknown or new users/items at "
                               "prediction time. This may be useful in cross-validation or production scenarios, "
                               "for handling user/item ids the model has not seen in the training data. Supported "
                               "values: 'nan', 'drop'.", TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(userCol="user", itemCol="item", coldStartStrategy="nan", blockSize=4096)


class _ALSParams(_ALSModelParams, HasMaxIter, HasRegParam, HasCheckpointInterval, HasSeed):
    rank = shared("rank", "rank of the factorization", TypeConverters.toInt)
    numUserBlocks = shared("numUserBlocks", "number of user blocks", TypeConverters.toInt)
    numItemBlocks = shared("numItemBlocks", "number of item blocks", TypeConverters.toInt)
    implicitPrefs = shared("implicitPrefs", "whether to use implicit preference", TypeConverters.toBoolean)
    alpha = shared("alpha", "alpha for implicit preference", TypeConverters.toFloat)
    ratingCol = shared("ratingCol", "column name for ratings", TypeConverters.toString)
    nonnegative = shared("nonnegative", "whether to use nonnegative constraint for least squares",
                         TypeConverters.toBoolean)
    intermediateStorageLevel = shared("intermediateStorageLevel", "StorageLevel for intermediate datasets. "
                                      "Cannot be 'NONE'.", TypeConverters.toString)
    finalStorageLevel = shared("finalStorageLevel", "StorageLevel for ALS model factors.", TypeConverters.toString)
    cgIters = shared("cgIters", "0 (default): every row's normal equations are solved exactly, as Spark does; "
                                "> 0: that many warm-started conjugate-gradient steps per half-iteration on large "
                                "problems (an approximation; small problems are always exact).", TypeConverters.toInt)

    def __init__(self):
        super().__init__()
        self._setDefault(rank=10, maxIter=10, regParam=0.1, numUserBlocks=10, numItemBlocks=10,
                         implicitPrefs=False, alpha=1.0, ratingCol="rating", nonnegative=False,
                         checkpointInterval=10, intermediateStorageLevel="MEMORY_AND_DISK",
                         finalStorageLevel="MEMORY_AND_DISK", cgIters=0, seed=0)


@register("org.apache.spark.ml.recommendation.ALS")
class ALS(Estimator, _ALSParams, MLWritable, MLReadable):
    """Alternating Least Squares matrix factorization (explicit or implicit feedback).
    Ratings are exchanged with all-to-all into user and item blocks; the other side's
    factors are all-gathered each half-iteration; every row's normal equations are solved
    exactly by the als_exact gfx950 kernels (cgIters > 0: opt-in conjugate gradient)."""
    _warm_family = "als"          # runtime/warmup.py lazy warm-up

    @keyword_only
    def __init__(self, *, rank=10, maxIter=10, regParam=0.1, numUserBlocks=10, numItemBlocks=10,
                 implicitPrefs=False, alpha=1.0, userCol="user", itemCol="item", seed=None, ratingCol="rating",
                 nonnegative=False, checkpointInterval=10, intermediateStorageLevel="MEMORY_AND_DISK",
                 finalStorageLevel="MEMORY_AND_DISK", coldStartStrategy="nan", blockSize=4096, cgIters=0):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        users = U.numeric_column(df, g(self.userCol), torch.int64)
        items = U.numeric_column(df, g(self.itemCol), torch.int64)
        r = U.numeric_column(df, g(self.ratingCol), torch.float32)
        from ..runtime.checkpoint import for_estimator
        res = ALSE.fit_als(df.comm, users, items, r, g(self.rank), g(self.maxIter), g(self.regParam),
                           g(self.implicitPrefs), g(self.alpha), g(self.seed), g(self.nonnegative), g(self.cgIters),
                           ckpt=for_estimator(self, df, sharded=True))
        m = ALSModel._from(res.user_ids, res.U, res.item_ids, res.V, g(self.rank))
        m.iterationSeconds = res.iter_seconds
        return m._with_parent(self)


@register("org.apache.spark.ml.recommendation.ALSModel")
class ALSModel(Model, _ALSModelParams, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self.rank = 0
        self._uid_t = self._U = self._iid_t = self._V = None

    @classmethod
    def _from(cls, uid, U_, iid, V, rank):
        m = cls()
        m._uid_t, m._U, m._iid_t, m._V, m.rank = uid, U_, iid, V, int(rank)
        return m

    def _factors_df(self, ids, F):
        from ..session import Session
        s = Session.active() or Session.getOrCreate()
        full = OrderedDict(id=C.NumericColumn(ids.to(torch.int32)), features=C.VectorColumn(F.float()))
        return DataFrame(s.local_view(), full)._from_full(full) if s.comm.world_size > 1 else \
            DataFrame(s, OrderedDict((k, _to(v, s.device)) for k, v in full.items()))

    @property
    def userFactors(self):
        return self._factors_df(self._uid_t, self._U)

    @property
    def itemFactors(self):
        return self._factors_df(self._iid_t, self._V)

    def _lookup(self, ids_t, table, q):
        q = q.to(ids_t.device, torch.int64)
        pos = torch.searchsorted(ids_t, q).clamp_max(max(ids_t.numel() - 1, 0))
        hit = ids_t[pos] == q if ids_t.numel() else torch.zeros_like(q, dtype=torch.bool)
        return pos, hit

    def _transform(self, df):
        g = self.getOrDefault
        u = U.numeric_column(df, g(self.userCol), torch.int64)
        i = U.numeric_column(df, g(self.itemCol), torch.int64)
        pu, hu = self._lookup(self._uid_t, self._U, u)
        pi, hi = self._lookup(self._iid_t, self._V, i)
        pred = torch.empty(pu.shape[0], dtype=torch.float64, device=pu.device)
        step = 1 << 21                        # bounded gathers: 2M rows x rank per chunk
        for a in range(0, pu.shape[0], step):
            pred[a:a + step] = (self._U[pu[a:a + step]].to(torch.float64)
                                * self._V[pi[a:a + step]].to(torch.float64)).sum(1)
        ok = hu & hi
        pred = torch.where(ok, pred, torch.full_like(pred, float("nan")))
        out = df.withColumnData(g(self.predictionCol), C.NumericColumn(pred.float()))
        if g(self.coldStartStrategy) == "drop":
            out = out._mask(ok.to(df.device))
        return out

    def _recommend(self, Q, ids_q, T, ids_t, k, qname, tname):
        """Top-``k`` rows of ``T`` per row of ``Q`` by dot product (Spark
        recommendForAll*): the score matrix is never materialised -- query x target
        blocks of bounded size, a running top-k merged per target block -- and the result
        stays on the device (``RecsColumn``: ids / scores [n, k]; Rows are built only when
        the column is read on the host).  Factors are replicated, so each rank recommends
        for its own block of query rows."""
        from ..session import Session
        s = Session.active() or Session.getOrCreate()
        if s.comm.world_size > 1:          # factors are replicated: each rank recommends its block
            lo, hi = s._shard_bounds(Q.shape[0])
            Q, ids_q = Q[lo:hi], ids_q[lo:hi]
        vals, idx = topk_scores(Q, T, k)
        ids_t = torch.as_tensor(ids_t).to(idx.device, torch.int64)
        cols = OrderedDict()
        cols[qname] = C.NumericColumn(ids_q.to(torch.int32).to(s.device))
        cols["recommendations"] = RecsColumn(ids_t[idx].to(torch.int32), vals.float(), tname)
        return DataFrame(s, cols, int(Q.shape[0]))

    def recommendForAllUsers(self, numItems):
        return self._recommend(self._U, self._uid_t, self._V, self._iid_t.cpu().numpy(), numItems,
                               self.getOrDefault(self.userCol), self.getOrDefault(self.itemCol))

    def recommendForAllItems(self, numUsers):
        return self._recommend(self._V, self._iid_t, self._U, self._uid_t.cpu().numpy(), numUsers,
                               self.getOrDefault(self.itemCol), self.getOrDefault(self.userCol))

    @staticmethod
    def _subset_ids(dataset, col):
        """Distinct ids of ``col`` over ALL ranks (each rank's rows hold an arbitrary part)."""
        q = U.numeric_column(dataset, col, torch.int64)
        return ALSE.global_ids(dataset.comm, q)

    def recommendForUserSubset(self, dataset, numItems):
        q = self._subset_ids(dataset, self.getOrDefault(self.userCol)).to(self._uid_t.device)
        pos, hit = self._lookup(self._uid_t, self._U, q)
        return self._recommend(self._U[pos[hit]], self._uid_t[pos[hit]], self._V, self._iid_t.cpu().numpy(),
                               numItems, self.getOrDefault(self.userCol), self.getOrDefault(self.itemCol))

    def recommendForItemSubset(self, dataset, numUsers):
        q = self._subset_ids(dataset, self.getOrDefault(self.itemCol)).to(self._iid_t.device)
        pos, hit = self._lookup(self._iid_t, self._V, q)
        return self._recommend(self._V[pos[hit]], self._iid_t[pos[hit]], self._U, self._uid_t.cpu().numpy(),
                               numUsers, self.getOrDefault(self.itemCol), self.getOrDefault(self.userCol))

    # Spark layout: metadata (+rank), userFactors/ and itemFactors/ parquet (id:int, features:array<float>)
    def _extra_metadata(self):
        return {"rank": self.rank}

    def write(self):
        from .util import MLWriter

        class _W(MLWriter):
            def saveImpl(w, path):
                save_metadata(self, path, self._extra_metadata())
                from .util import _is_rank0
                if _is_rank0():
                    import pyarrow as pa
                    from .util import write_data
                    # Spark ALSModel: userFactors/ and itemFactors/ = (id int NOT NULL,
                    # features array<float NOT NULL>), written as Spark's parquet parts
                    elem = pa.list_(pa.field("element", pa.float32(), False))
                    for name, ids, F in (("userFactors", self._uid_t, self._U), ("itemFactors", self._iid_t, self._V)):
                        Fh = F.float().cpu().numpy()
                        feats = pa.ListArray.from_arrays(pa.array(np.arange(0, Fh.size + 1, max(Fh.shape[1], 1),
                                                                            dtype=np.int32)[:Fh.shape[0] + 1]),
                                                         pa.array(Fh.reshape(-1)), type=elem)
                        t = pa.table({"id": pa.array(ids.cpu().numpy().astype(np.int32)), "features": feats})
                        write_data(path, t, subdir=name, non_null=("id",))
        return _W(self)

    @classmethod
    def _load_impl(cls, path, meta):
        import pyarrow.parquet as pq
        from ..session import Session
        dev = (Session.active() or Session.getOrCreate()).device
        parts = []
        for name in ("userFactors", "itemFactors"):
            t = pq.read_table(os.path.join(path, name)).to_pydict()
            ids = torch.tensor(t["id"], dtype=torch.int64)
            o = torch.argsort(ids)
            F = torch.tensor(t["features"], dtype=torch.float32)[o]
            parts += [ids[o].to(dev), F.to(dev)]
        m = cls._from(parts[0], parts[1], parts[2], parts[3], meta.get("rank", parts[1].shape[1]))
        apply_metadata(m, meta)
        return m


def topk_scores(Q: torch.Tensor, T: torch.Tensor, k: int, budget: int = 1 << 28):
    """(values, indices) [nQ, k] of the k largest Q @ T^T entries per row, computed over
    query x target blocks of at most ``budget`` scores (fp32 GEMM + top-k, merged per
    target block), so 50M x 5M never materialises."""
    nQ, nT = int(Q.shape[0]), int(T.shape[0])
    k = max(0, min(int(k), nT))
    dev = Q.device
    vals = torch.empty((nQ, k), dtype=torch.float32, device=dev)
    idx = torch.empty((nQ, k), dtype=torch.int64, device=dev)
    if nQ == 0 or k == 0:
        return vals, idx
    tc = min(nT, max(k, budget // max(1, min(nQ, 4096))))
    qc = max(1, min(nQ, budget // tc))
    Tf = T.float()
    for a in range(0, nQ, qc):
        Qa = Q[a:a + qc].float()
        bv = bi = None
        for t0 in range(0, nT, tc):
            sc = Qa @ Tf[t0:t0 + tc].T
            v, i = torch.topk(sc, min(k, sc.shape[1]), dim=1)
            i = i + t0
            if bv is None:
                bv, bi = v, i
            else:
                cv, ci = torch.cat([bv, v], 1), torch.cat([bi, i], 1)
                bv, pos = torch.topk(cv, k, dim=1)
                bi = ci.gather(1, pos)
            del sc
        vals[a:a + qc], idx[a:a + qc] = bv, bi
    return vals, idx


class RecsColumn(C.ArrayColumn):
    """array<struct<id, rating>> kept on the device as ids [n, k] (int32) and scores [n, k]
    (float32); the host ``values`` (lists of Rows, Spark's recommendation layout) are built
    on first access."""

    def __init__(self, ids: torch.Tensor, scores: torch.Tensor, id_name: str):
        from ..frame import types as T
        self.ids, self.scores, self.id_name = ids, scores, id_name
        self.dtype = T.ArrayType(T.StructType([T.StructField(id_name, T.IntegerType()),
                                               T.StructField("rating", T.FloatType())]))
        self._host = None

    def __len__(self):
        return int(self.ids.shape[0])

    @property
    def values(self):
        if self._host is None:
            ids, sc = self.ids.cpu().tolist(), self.scores.cpu().tolist()
            names = [self.id_name, "rating"]
            arr = np.empty(len(ids), dtype=object)
            arr[:] = [[Row._make(names, [i, float(v)]) for i, v in zip(ri, rv)] for ri, rv in zip(ids, sc)]
            self._host = arr
        return self._host

    @values.setter
    def values(self, v):
        self._host = v

    def _sub(self, sel):
        return RecsColumn(self.ids[sel], self.scores[sel], self.id_name)

    def take(self, idx):
        return self._sub(idx.to(self.ids.device).long())

    def mask_select(self, mask):
        return self._sub(mask.to(self.ids.device).bool())

    def slice(self, start, end):
        return RecsColumn(self.ids[start:end], self.scores[start:end], self.id_name)

    def null_mask(self):
        return torch.zeros(len(self), dtype=torch.bool)

    def nbytes(self):
        return self.ids.numel() * 4 + self.scores.numel() * 4

    @classmethod
    def concat(cls, cols):
        if all(isinstance(c, RecsColumn) and c.ids.shape[1:] == cols[0].ids.shape[1:] for c in cols):
            dev = cols[0].ids.device
            return RecsColumn(torch.cat([c.ids.to(dev) for c in cols]), torch.cat([c.scores.to(dev) for c in cols]),
                              cols[0].id_name)
        return C.ArrayColumn(np.concatenate([c.values for c in cols]), cols[0].dtype.elementType)


def _to(c, dev):
    if isinstance(c, C.NumericColumn):
        return C.NumericColumn(c.data.to(dev))
    return C.VectorColumn(c.data.to(dev))
