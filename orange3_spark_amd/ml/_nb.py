"""NaiveBayes (``pyspark.ml.classification.NaiveBayes``; multinomial / bernoulli /
complement / gaussian).

Reached through the Classification widget's reflection over ``classification``
(orangecontrib/spark/widgets/ml/spark_ml_classification.py:15).

Training is ONE pass: the per-class feature sums are the GEMM ``onehot(y)^T (w * X)``
([K, n] x [n, D], hipBLASLt on the rank's GPU, chunked), plus ``onehot^T (w * X^2)`` for
the gaussian model, then one all-reduce of the [K, 2D + 1] statistics.  Prediction is
another GEMM, ``X theta^T`` (+ the gaussian quadratic terms).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops.gram import rows_t_matmul

from ..frame import column as C
from . import common as U
from .base import Estimator, Model
from .linalg import DenseMatrix, DenseVector
from .param import (HasFeaturesCol, HasLabelCol, HasPredictionCol, HasProbabilityCol, HasRawPredictionCol,
                    HasThresholds, HasWeightCol, TypeConverters, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, mat_col, read_data, register, vec_col, write_data

_TYPES = ("multinomial", "bernoulli", "complement", "gaussian")


class _NaiveBayesParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasProbabilityCol, HasRawPredictionCol,
                        HasThresholds, HasWeightCol):
    smoothing = shared("smoothing", "The smoothing parameter, should be >= 0, default is 1.0",
                       TypeConverters.toFloat)
    modelType = shared("modelType", "The model type which is a string (case-sensitive). Supported options: "
                                    "multinomial (default), bernoulli, complement and gaussian.",
                       TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(smoothing=1.0, modelType="multinomial")


def class_sums(comm, X: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None, K: int, squares: bool,
               chunk: int = 1 << 20):
    """All-reduced (S [K,D], S2 [K,D] or None, weight per class [K]) in fp64."""
    dev = X.device
    dt = torch.float32 if X.is_cuda else torch.float64
    n, D = X.shape
    S = torch.zeros((K, D), dtype=torch.float64, device=dev)
    S2 = torch.zeros((K, D), dtype=torch.float64, device=dev) if squares else None
    cnt = torch.zeros(K, dtype=torch.float64, device=dev)
    yl = y.to(dev).long()
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        Xc = X[a:b].to(dt)
        wc = torch.ones(b - a, dtype=dt, device=dev) if w is None else w[a:b].to(dev, dt)
        oh = torch.zeros((b - a, K), dtype=dt, device=dev)
        oh.scatter_(1, yl[a:b, None], wc[:, None])
        S += rows_t_matmul(oh, Xc).double()
        if squares:
            S2 += rows_t_matmul(oh, Xc * Xc).double()
        cnt += oh.sum(0).double()
    buf = torch.cat([S.reshape(-1), S2.reshape(-1) if squares else S.new_zeros(0), cnt])
    comm.all_reduce(buf)
    S = buf[: K * D].reshape(K, D)
    S2 = buf[K * D: 2 * K * D].reshape(K, D) if squares else None
    return S, S2, buf[-K:]


def sparse_class_sums(comm, rows, y: torch.Tensor, w: torch.Tensor | None, K: int):
    """All-reduced (S [K,D], None, weight per class [K]) fp64 for CSR rows (ops.sparse):
    one CSC column-sum pass per class with r = w * [y == k]."""
    dev = rows.device
    yd = y.to(dev)
    wd = torch.ones_like(yd, dtype=torch.float32) if w is None else w.to(dev, torch.float32)
    S = torch.stack([rows.colsum(torch.where(yd == k, wd, torch.zeros_like(wd))) for k in range(K)])
    cnt = torch.zeros(K, dtype=torch.float64, device=dev).index_add_(0, yd.long(), wd.to(torch.float64))
    buf = torch.cat([S.reshape(-1), cnt])
    comm.all_reduce(buf)
    return buf[: K * rows.d].reshape(K, rows.d), None, buf[-K:]


@register("org.apache.spark.ml.classification.NaiveBayes")
class NaiveBayes(Estimator, _NaiveBayesParams, MLWritable, MLReadable):
    """Naive Bayes Classifiers. It supports both Multinomial and Bernoulli NB. Multinomial
    NB can handle finitely supported discrete data (e.g. TF vectors); Bernoulli NB needs
    0-1 feature vectors.  Complement NB and Gaussian NB are also supported.
    """

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction",
                 probabilityCol="probability", rawPredictionCol="rawPrediction", smoothing=1.0,
                 modelType="multinomial", thresholds=None, weightCol=None):
        super().__init__()
        self._set(**self._input_kwargs)

    @keyword_only
    def setParams(self, *, featuresCol="features", labelCol="label", predictionCol="prediction",
                  probabilityCol="probability", rawPredictionCol="rawPrediction", smoothing=1.0,
                  modelType="multinomial", thresholds=None, weightCol=None):
        return self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        mt = g(self.modelType)
        if mt not in _TYPES:
            raise ValueError(f"Invalid modelType: {mt}. Supported: {', '.join(_TYPES)}")
        lam = float(g(self.smoothing))
        comm = df.comm
        y = U.numeric_column(df, g(self.labelCol))
        w = U.weights_or_none(df, self)
        K = U.num_classes(comm, y)
        col = U.features_column(df, g(self.featuresCol))
        if isinstance(col, C.SparseVectorColumn) and mt != "gaussian":
            # term counts stay CSR: per-class column sums by the CSC piece kernels
            X = U.linear_features(df, g(self.featuresCol))
            vals = X.val
        else:
            X = U.dense_features(df, g(self.featuresCol))
            vals = X
        if mt in ("multinomial", "complement") and vals.numel():
            lo = -comm.max_scalar(float(-vals.float().min()))
            if lo < 0:
                raise ValueError(f"Naive Bayes requires nonnegative feature values but found {lo}.")
        if mt == "bernoulli" and vals.numel():
            Xf = vals.float()
            if not bool(((Xf == 0) | (Xf == 1)).all()):
                raise ValueError("Bernoulli naive Bayes requires 0 or 1 feature values.")
        if isinstance(X, torch.Tensor):
            S, S2, cnt = class_sums(comm, X, y, w, K, squares=mt == "gaussian")
        else:
            S, S2, cnt = sparse_class_sums(comm, X, y, w, K)
        S, cnt = S.cpu().numpy(), cnt.cpu().numpy()
        D = S.shape[1]
        N = cnt.sum()
        sigma = np.zeros((0, 0))
        if mt == "gaussian":
            pi = np.log(np.maximum(cnt, 1e-300)) - math.log(N)
            mean = S / np.maximum(cnt, 1e-300)[:, None]
            var = S2.cpu().numpy() / np.maximum(cnt, 1e-300)[:, None] - mean ** 2
            tot1, tot2 = S.sum(0), S2.cpu().numpy().sum(0)
            gvar = np.maximum(tot2 / N - (tot1 / N) ** 2, 0.0)
            eps = 1e-9 * float(gvar.max()) if gvar.size else 0.0
            theta, sigma = mean, np.maximum(var, 0.0) + eps
        else:
            pi = np.log(cnt + lam) - math.log(N + K * lam)
            if mt == "multinomial":
                theta = np.log(S + lam) - np.log(S.sum(1, keepdims=True) + D * lam)
            elif mt == "bernoulli":
                theta = np.log(S + lam) - np.log(cnt[:, None] + 2 * lam)
            else:  # complement: weights from the statistics of all OTHER classes
                fs = S.sum(0, keepdims=True)
                comp = fs - S
                theta = -(np.log(comp + lam) - np.log(comp.sum(1, keepdims=True) + D * lam))
        return NaiveBayesModel._from(pi, theta, sigma, mt)._with_parent(self)


@register("org.apache.spark.ml.classification.NaiveBayesModel")
class NaiveBayesModel(U.ProbabilisticClassifierMixin, Model, _NaiveBayesParams, MLWritable, MLReadable):
    """Model fitted by NaiveBayes."""

    def __init__(self):
        super().__init__()
        self._pi = np.zeros(0)
        self._theta = np.zeros((0, 0))
        self._sigma = np.zeros((0, 0))
        self._type = "multinomial"

    @classmethod
    def _from(cls, pi, theta, sigma, model_type):
        m = cls()
        m._pi, m._theta, m._sigma = np.asarray(pi, float), np.asarray(theta, float), np.asarray(sigma, float)
        m._type = model_type
        return m

    @property
    def pi(self) -> DenseVector:
        return DenseVector(self._pi)

    @property
    def theta(self) -> DenseMatrix:
        return DenseMatrix.from_array(self._theta)

    @property
    def sigma(self) -> DenseMatrix:
        return DenseMatrix.from_array(self._sigma)

    @property
    def numClasses(self) -> int:
        return int(self._pi.shape[0])

    @property
    def numFeatures(self) -> int:
        return int(self._theta.shape[1])

    def _features_for_predict(self, df, name):
        mt = self.getOrDefault(self.modelType) if self.isDefined(self.modelType) else self._type
        if mt != "gaussian":
            return U.linear_features(df, name)      # CSR rows for sparse counts
        return U.dense_features(df, name)

    def _raw(self, X):
        if not isinstance(X, torch.Tensor):         # CSR rows: one sparse margin pass per class
            return self._raw_sparse(X)
        dt = torch.float32 if X.is_cuda else torch.float64
        Xf = X.to(dt)[:, : self.numFeatures]
        th = torch.from_numpy(self._theta).to(X.device, dt)
        pi = torch.from_numpy(self._pi).to(X.device, dt)
        mt = self.getOrDefault(self.modelType) if self.isDefined(self.modelType) else self._type
        if mt == "multinomial":
            raw = Xf @ th.T + pi
        elif mt == "bernoulli":
            neg = torch.log1p(-torch.exp(th))
            raw = Xf @ (th - neg).T + pi + neg.sum(1)
        elif mt == "complement":
            s = Xf @ th.T
            raw = s - torch.logsumexp(s, dim=1, keepdim=True)
        else:
            var = torch.from_numpy(self._sigma).to(X.device, dt)
            iv = 1.0 / var
            quad = (Xf * Xf) @ iv.T - 2.0 * Xf @ (th * iv).T + (th * th * iv).sum(1)
            raw = pi - 0.5 * torch.log(2 * math.pi * var).sum(1) - 0.5 * quad
        return raw.to(torch.float64)

    def _raw_sparse(self, X):
        mt = self.getOrDefault(self.modelType) if self.isDefined(self.modelType) else self._type
        th, pi = self._theta, self._pi
        K = th.shape[0]
        if mt == "multinomial":
            cols = [U.linear_margin(X, th[k], pi[k]) for k in range(K)]
        elif mt == "bernoulli":
            neg = np.log1p(-np.exp(th))
            cols = [U.linear_margin(X, th[k] - neg[k], pi[k] + neg[k].sum()) for k in range(K)]
        else:  # complement
            s = torch.stack([U.linear_margin(X, th[k], 0.0) for k in range(K)], 1)
            return s - torch.logsumexp(s, dim=1, keepdim=True)
        return torch.stack(cols, 1)

    def _raw2prob(self, raw):
        return torch.softmax(raw, dim=1)

    def _save_data(self, path):
        write_data(path, {"pi": vec_col([self.pi]), "theta": mat_col([self.theta]), "sigma": mat_col([self.sigma])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import matrix_from_struct, vector_from_struct
        t = read_data(path).to_pylist()[0]
        mt = meta.get("paramMap", {}).get("modelType") or meta.get("defaultParamMap", {}).get("modelType",
                                                                                             "multinomial")
        sig = matrix_from_struct(t["sigma"]).toArray() if t.get("sigma") else np.zeros((0, 0))
        m = cls._from(vector_from_struct(t["pi"]).toArray(), matrix_from_struct(t["theta"]).toArray(), sig, mt)
        apply_metadata(m, meta)
        return m
