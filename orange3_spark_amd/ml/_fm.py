"""Factorization machines: FMClassifier / FMRegressor (``pyspark.ml`` >= 3.0).

    y(x) = w0 + sum_i w_i x_i + 1/2 sum_f [ (sum_i v_if x_i)^2 - sum_i v_if^2 x_i^2 ]

The pairwise term is two GEMMs per chunk, ``X V`` and ``X^2 V^2`` ([n, D] x [D, F]),
so a forward/backward pass is GEMM-shaped work for hipBLASLt; the flat gradient
[V | w | w0] (Spark's parameter layout) is all-reduced once per step
(models/dist_opt.py).  Solvers: ``adamW`` (Spark's default) and ``gd``, with
``miniBatchFraction`` sampling.
"""
from __future__ import annotations

import numpy as np
import torch

from ..models import dist_opt
from . import common as U
from .base import Estimator, Model
from .linalg import DenseMatrix, DenseVector
from .param import (HasFeaturesCol, HasFitIntercept, HasLabelCol, HasMaxIter, HasPredictionCol,
                    HasProbabilityCol, HasRawPredictionCol, HasRegParam, HasSeed, HasSolver, HasStepSize,
                    HasThresholds, HasTol, HasWeightCol, TypeConverters, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, mat_col, read_data, register, vec_col, write_data
from . import _summary as S


class _FMParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasMaxIter, HasStepSize, HasTol, HasSolver,
                HasSeed, HasFitIntercept, HasRegParam, HasWeightCol):
    factorSize = shared("factorSize", "Dimensionality of the factor vectors, which are used to get pairwise "
                                      "interactions between variables", TypeConverters.toInt)
    fitLinear = shared("fitLinear", "whether to fit linear term (aka 1-way term)", TypeConverters.toBoolean)
    miniBatchFraction = shared("miniBatchFraction", "fraction of the input data set that should be used for one "
                                                    "iteration of gradient descent", TypeConverters.toFloat)
    initStd = shared("initStd", "standard deviation of initial coefficients", TypeConverters.toFloat)

    def __init__(self):
        super().__init__()
        self._setDefault(factorSize=8, fitIntercept=True, fitLinear=True, regParam=0.0, miniBatchFraction=1.0,
                         initStd=0.01, maxIter=100, stepSize=1.0, tol=1e-6, solver="adamW", seed=0)


def fm_forward(theta: torch.Tensor, X: torch.Tensor, D: int, F: int) -> torch.Tensor:
    V = theta[: D * F].reshape(D, F)
    w = theta[D * F: D * F + D]
    w0 = theta[-1]
    XV = X @ V
    X2V2 = (X * X) @ (V * V)
    return w0 + X @ w + 0.5 * (XV * XV - X2V2).sum(1)


def _fit_fm(est, df, classification: bool):
    g = est.getOrDefault
    comm = df.comm
    X = U.dense_features(df, g(est.featuresCol))
    y = U.numeric_column(df, g(est.labelCol))
    sw = U.weights_or_none(df, est)
    if classification and U.num_classes(comm, y) > 2:
        raise ValueError("FMClassifier only supports binary classification.")
    dev = X.device
    dt = dist_opt.compute_dtype(dev)
    n, D = X.shape
    D = int(comm.max_scalar(float(D)))
    F = int(g(est.factorSize))
    yt = y.to(dev, dt)
    swt = None if sw is None else sw.to(dev, dt)
    W = float(comm.sum_scalar(float(n if sw is None else sw.sum())))
    fit_lin, fit_b = g(est.fitLinear), g(est.fitIntercept)
    lin_mask = torch.zeros(D * F + D + 1, dtype=dt, device=dev)
    lin_mask[: D * F] = 1
    if fit_lin:
        lin_mask[D * F: D * F + D] = 1
    if fit_b:
        lin_mask[-1] = 1

    def local_loss(theta, a, b):
        th = theta * lin_mask
        m = fm_forward(th, X[a:b].to(dt), D, F)
        if classification:
            l = torch.nn.functional.softplus(m) - yt[a:b] * m      # log(1 + e^m) - y m
        else:
            l = 0.5 * (m - yt[a:b]) ** 2
        return (l if swt is None else l * swt[a:b]).sum()

    l2_mask = np.concatenate([np.ones(D * F), np.ones(D), np.zeros(1)])
    chunk = 1 << 18
    frac = float(g(est.miniBatchFraction))
    if frac < 1.0:
        chunk = max(1024, min(chunk, int(max(n, 1) * frac) // 4 or 1024))
    obj = dist_opt.Objective(comm, dev, n, local_loss, W, l2=g(est.regParam), l2_mask=l2_mask, chunk=chunk, sw=swt)
    rng = np.random.default_rng(int(g(est.seed)) & 0xFFFFFFFF)
    x0 = np.zeros(D * F + D + 1)
    x0[: D * F] = rng.normal(0.0, g(est.initStd), D * F)
    solver = g(est.solver).lower()
    res = dist_opt.gradient_descent(obj, x0, g(est.maxIter), g(est.stepSize), g(est.tol), fraction=frac,
                                    seed=int(g(est.seed)) & 0xFFFFFFFF, adam=solver == "adamw")
    x = res.x * lin_mask.double().cpu().numpy()
    return x[: D * F].reshape(D, F), x[D * F: D * F + D], float(x[-1]), res


class _FMModelBase(Model, _FMParams, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self._V = np.zeros((0, 0))
        self._w = np.zeros(0)
        self._b = 0.0
        self.summary = None

    @classmethod
    def _from(cls, V, w, b):
        m = cls()
        m._V, m._w, m._b = np.asarray(V, float), np.asarray(w, float), float(b)
        return m

    @property
    def factors(self) -> DenseMatrix:
        return DenseMatrix.from_array(self._V)

    @property
    def linear(self) -> DenseVector:
        return DenseVector(self._w)

    @property
    def intercept(self) -> float:
        return self._b

    @property
    def numFeatures(self) -> int:
        return int(self._w.shape[0])

    def _margin(self, X):
        dt = dist_opt.compute_dtype(X.device)
        D, F = self._V.shape
        theta = torch.from_numpy(np.concatenate([self._V.reshape(-1), self._w, [self._b]])).to(X.device, dt)
        return fm_forward(theta, X.to(dt)[:, :D], D, F).to(torch.float64)

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"intercept": pa.array([self._b]), "linear": vec_col([self.linear]),
                          "factors": mat_col([self.factors])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import matrix_from_struct, vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls._from(matrix_from_struct(t["factors"]).toArray(), vector_from_struct(t["linear"]).toArray(),
                      t["intercept"])
        apply_metadata(m, meta)
        return m


class FMClassificationTrainingSummary(S.BinaryClassificationSummary, S.TrainingSummaryMixin):
    """Spark FMClassificationTrainingSummary: binary metrics over the training predictions."""

    def __init__(self, model, df, res):
        g = model.getOrDefault
        super().__init__(lambda: model.transform(df), scoreCol=g(model.probabilityCol), labelCol=g(model.labelCol),
                         predictionCol=g(model.predictionCol))
        self._init_training(res.history, res.iterations)


class FMRegressionTrainingSummary(S.LinearRegressionSummary, S.TrainingSummaryMixin):
    def __init__(self, model, df, res):
        g = model.getOrDefault
        super().__init__(lambda: model.transform(df), labelCol=g(model.labelCol), predictionCol=g(model.predictionCol),
                         featuresCol=g(model.featuresCol), fitIntercept=g(model.fitIntercept))
        self._init_training(res.history, res.iterations)


class _FMClassifierParams(_FMParams, HasProbabilityCol, HasRawPredictionCol, HasThresholds):
    pass


@register("org.apache.spark.ml.classification.FMClassifier")
class FMClassifier(Estimator, _FMClassifierParams, MLWritable, MLReadable):
    """Factorization Machines learning algorithm for classification (logistic loss)."""

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction",
                 probabilityCol="probability", rawPredictionCol="rawPrediction", factorSize=8, fitIntercept=True,
                 fitLinear=True, regParam=0.0, miniBatchFraction=1.0, initStd=0.01, maxIter=100, stepSize=1.0,
                 tol=1e-6, solver="adamW", thresholds=None, seed=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        V, w, b, res = _fit_fm(self, df, True)
        m = FMClassificationModel._from(V, w, b)._with_parent(self)
        m.summary = FMClassificationTrainingSummary(m, df, res)
        return m


@register("org.apache.spark.ml.classification.FMClassificationModel")
class FMClassificationModel(U.ProbabilisticClassifierMixin, _FMModelBase, _FMClassifierParams):
    """Model fitted by FMClassifier."""

    numClasses = 2

    def _raw(self, X):
        m = self._margin(X)
        return torch.stack([-m, m], dim=1)

    def _raw2prob(self, raw):
        p = torch.sigmoid(raw[:, 1])
        return torch.stack([1 - p, p], dim=1)


@register("org.apache.spark.ml.regression.FMRegressor")
class FMRegressor(Estimator, _FMParams, MLWritable, MLReadable):
    """Factorization Machines learning algorithm for regression (squared loss)."""

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", factorSize=8,
                 fitIntercept=True, fitLinear=True, regParam=0.0, miniBatchFraction=1.0, initStd=0.01,
                 maxIter=100, stepSize=1.0, tol=1e-6, solver="adamW", seed=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        V, w, b, res = _fit_fm(self, df, False)
        m = FMRegressionModel._from(V, w, b)._with_parent(self)
        m.summary = FMRegressionTrainingSummary(m, df, res)
        return m


@register("org.apache.spark.ml.regression.FMRegressionModel")
class FMRegressionModel(U.PredictionModelMixin, _FMModelBase):
    """Model fitted by FMRegressor."""

    def _predict_tensor(self, X):
        return self._margin(X)
