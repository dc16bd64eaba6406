"""Clustering estimators (``pyspark.ml.clustering`` surface).

Reached in the reference through the Clustering widget
(orangecontrib/spark/widgets/ml/spark_ml_clustering.py:14).
"""
from __future__ import annotations

import numpy as np
import torch

from ..models import kmeans as KM
from . import common as U
from .base import Estimator, Model
from .linalg import DenseVector
from .param import (HasDistanceMeasure, HasFeaturesCol, HasMaxIter, HasPredictionCol, HasSeed, HasTol,
                    HasWeightCol, TypeConverters, add_accessors, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, read_data, register, vec_col, write_data


class _KMeansParams(HasFeaturesCol, HasPredictionCol, HasMaxIter, HasTol, HasSeed, HasDistanceMeasure,
                    HasWeightCol):
    k = shared("k", "The number of clusters to create. Must be > 1.", TypeConverters.toInt)
    initMode = shared("initMode", 'The initialization algorithm. This can be either "random" to choose random '
                                  'points as initial cluster centers, or "k-means||" to use a parallel variant of '
                                  'k-means++', TypeConverters.toString)
    initSteps = shared("initSteps", "The number of steps for k-means|| initialization mode. Must be > 0.",
                       TypeConverters.toInt)
    solver = shared("solver", "The solver algorithm for optimization. Supported options: auto, row, block.",
                    TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(k=2, initMode="k-means||", initSteps=2, tol=1e-4, maxIter=20, distanceMeasure="euclidean",
                         solver="auto", seed=0)


class _ClusteringSummary:
    def __init__(self, k, sizes, cost, iters, predictions=None):
        self.k = k
        self.clusterSizes = sizes
        self.trainingCost = cost
        self.numIter = iters
        self.predictions = predictions


@add_accessors
@register("org.apache.spark.ml.clustering.KMeans")
class KMeans(Estimator, _KMeansParams, MLWritable, MLReadable):
    """K-means clustering with a k-means++ like initialization mode (the k-means|| algorithm
    by Bahmani et al).  Assignment is a split-bf16 MFMA GEMM with a fused argmin on gfx950;
    per-cluster sums use deterministic slab reductions and one RCCL all-reduce/iteration."""
    _warm_family = "kmeans"          # runtime/warmup.py lazy warm-up

    @keyword_only
    def __init__(self, *, featuresCol="features", predictionCol="prediction", k=2, initMode="k-means||",
                 initSteps=2, tol=1e-4, maxIter=20, seed=None, distanceMeasure="euclidean", weightCol=None,
                 solver="auto"):
        super().__init__()
        self._set(**self._input_kwargs)

    @keyword_only
    def setParams(self, *, featuresCol="features", predictionCol="prediction", k=2, initMode="k-means||",
                  initSteps=2, tol=1e-4, maxIter=20, seed=None, distanceMeasure="euclidean", weightCol=None,
                  solver="auto"):
        return self._set(**self._input_kwargs)

    def _fit(self, df):
        from ..frame.spill import RowBlocks, SpilledVectorColumn
        g = self.getOrDefault
        w = U.weights_or_none(df, self)
        col = U.features_column(df, g(self.featuresCol))
        cosine = g(self.distanceMeasure) == "cosine"
        if isinstance(col, SpilledVectorColumn) and col.spilled_rows and w is None:
            def prep(X):          # the assign/update kernels' operand (+ cosine normalisation)
                X = X.float().contiguous() if X.is_cuda else X.to(torch.float64)
                return X / X.norm(dim=1, keepdim=True).clamp_min(1e-300) if cosine else X
            X = RowBlocks(col, prep)
        else:
            X = U.dense_features(df, g(self.featuresCol))
            X = X.float().contiguous() if X.is_cuda else X.to(torch.float64)
        from ..runtime.checkpoint import for_estimator
        res = KM.fit_kmeans(df.comm, X, g(self.k), g(self.maxIter), g(self.tol), g(self.seed), g(self.initMode),
                            g(self.initSteps), weights=w, cosine=g(self.distanceMeasure) == "cosine",
                            ckpt=for_estimator(self, df))
        m = KMeansModel._from(res.centers.numpy())
        m.summary = _ClusteringSummary(g(self.k), res.sizes, res.cost, res.iterations)
        m.trainingSeconds = res.seconds
        return m._with_parent(self)


@register("org.apache.spark.ml.clustering.KMeansModel")
class KMeansModel(Model, _KMeansParams, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self._C = np.zeros((0, 0))
        self.summary = None

    @classmethod
    def _from(cls, C):
        m = cls()
        m._C = np.asarray(C, dtype=np.float64)
        return m

    @property
    def hasSummary(self):
        return self.summary is not None

    def clusterCenters(self):
        return [c.copy() for c in self._C]

    def _predict_tensor(self, X):
        return KM.predict(X, torch.from_numpy(self._C), self.getOrDefault(self.distanceMeasure) == "cosine")

    def _transform(self, df):
        X = U.dense_features(df, self.getOrDefault(self.featuresCol))
        X = X.float().contiguous() if X.is_cuda else X.to(torch.float64)
        return df.withColumnData(self.getOrDefault(self.predictionCol),
                                 U.C.NumericColumn(self._predict_tensor(X).to(torch.int32)))

    def predict(self, value):
        x = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value), dtype=torch.float64)
        return int(self._predict_tensor(x[None, :])[0])

    def computeCost(self, df):
        X = U.dense_features(df, self.getOrDefault(self.featuresCol)).to(torch.float64)
        C = torch.from_numpy(self._C).to(X.device)
        d = ((X[:, None, :] - C[None]) ** 2).sum(-1).min(1).values.sum()
        df.comm.all_reduce(d)
        return float(d)

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"clusterIdx": pa.array(list(range(len(self._C))), pa.int32()),
                          "clusterCenter": vec_col([DenseVector(c) for c in self._C])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        rows = sorted(read_data(path).to_pylist(), key=lambda r: r["clusterIdx"])
        m = cls._from(np.array([vector_from_struct(r["clusterCenter"]).toArray() for r in rows]))
        apply_metadata(m, meta)
        return m


from ._clustering_extra import (LDA, BisectingKMeans, BisectingKMeansModel, GaussianMixture,  # noqa: E402,F401
                                GaussianMixtureModel, LDAModel, LocalLDAModel, DistributedLDAModel,
                                PowerIterationClustering)
