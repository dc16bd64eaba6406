"""Regression estimators (``pyspark.ml.regression`` surface).

Reached in the reference through the Regression widget
(orangecontrib/spark/widgets/ml/spark_ml_regression.py:15).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..models import glm as GLM
from . import common as U
from ._tree import (DecisionTreeRegressionModel, DecisionTreeRegressor, GBTRegressionModel,  # noqa: F401
                    GBTRegressor, RandomForestRegressionModel, RandomForestRegressor)
from .base import Estimator, Model
from .linalg import DenseVector
from .param import (HasAggregationDepth, HasElasticNetParam, HasFeaturesCol, HasFitIntercept, HasLabelCol,
                    HasMaxBlockSizeInMB, HasMaxIter, HasPredictionCol, HasRegParam, HasStandardization, HasTol,
                    HasWeightCol, TypeConverters, keyword_only, shared)
from ..runtime.checkpoint import for_estimator
from .util import MLReadable, MLWritable, apply_metadata, read_data, register, vec_col, write_data


from . import _summary as S  # noqa: E402


def _linreg_summary(model, df, res_history=None, iterations=0):
    g = model.getOrDefault
    kw = dict(labelCol=g(model.labelCol), predictionCol=g(model.predictionCol), featuresCol=g(model.featuresCol),
              weightCol=g(model.weightCol) if model.isDefined(model.weightCol) and g(model.weightCol) else None,
              coefficients=model._w, intercept=model._b, fitIntercept=g(model.fitIntercept),
              regParam=g(model.regParam))
    pred = (lambda: model.transform(df))
    if res_history is None:
        return S.LinearRegressionSummary(pred, **kw)
    return S.LinearRegressionTrainingSummary(pred, res_history, iterations, **kw)


class _LinearRegressionParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasMaxIter, HasRegParam,
                              HasElasticNetParam, HasTol, HasFitIntercept, HasStandardization, HasWeightCol,
                              HasAggregationDepth, HasMaxBlockSizeInMB):
    solver = shared("solver", "The solver algorithm for optimization. Supported options: auto, normal, l-bfgs.",
                    TypeConverters.toString)
    loss = shared("loss", "The loss function to be optimized. Supported options: squared, huber.",
                  TypeConverters.toString)
    epsilon = shared("epsilon", "The shape parameter to control the amount of robustness. Must be > 1.0. Only "
                                "valid when loss is huber", TypeConverters.toFloat)

    def __init__(self):
        super().__init__()
        self._setDefault(maxIter=100, regParam=0.0, tol=1e-6, solver="auto", loss="squared", epsilon=1.35,
                         elasticNetParam=0.0, fitIntercept=True, standardization=True)


@register("org.apache.spark.ml.regression.LinearRegression")
class LinearRegression(Estimator, _LinearRegressionParams, MLWritable, MLReadable):
    """Linear regression (squared loss; L2 / L1 / elastic net).  ``normal`` solves the
    all-reduced weighted Gram system (X^T W X is one GEMM per rank); ``l-bfgs`` streams
    the fused GLM kernel."""
    _warm_family = "glm"          # runtime/warmup.py lazy warm-up

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxIter=100,
                 regParam=0.0, elasticNetParam=0.0, tol=1e-6, fitIntercept=True, standardization=True,
                 solver="auto", weightCol=None, aggregationDepth=2, loss="squared", epsilon=1.35,
                 maxBlockSizeInMB=0.0):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        comm = df.comm
        feat = U.features_column(df, g(self.featuresCol))
        y = U.numeric_column(df, g(self.labelCol))
        w = U.weights_or_none(df, self)
        solver = g(self.solver)
        alpha = g(self.elasticNetParam)
        if solver == "normal" or (solver == "auto" and alpha == 0.0 and feat.size <= 4096):
            coef, b, hist = _normal_equations(comm, U.dense_features(df, g(self.featuresCol)), y, w, g(self.regParam),
                                              g(self.fitIntercept), g(self.standardization))
            m = LinearRegressionModel._from(coef, b)._with_parent(self)
            m.summary = _linreg_summary(m, df, hist, 0)
            return m
        data = GLM.make_glm_data(comm, feat, y, w)
        res = GLM.fit_glm(data, "squared", g(self.regParam), alpha, g(self.fitIntercept), g(self.standardization),
                          g(self.maxIter), g(self.tol), ckpt=for_estimator(self, df))
        m = LinearRegressionModel._from(res.coef, res.intercept)._with_parent(self)
        m.summary = _linreg_summary(m, df, res.history, res.iterations)
        return m


def _normal_equations(comm, X, y, w, reg, fit_intercept, standardization):
    """Weighted ridge via all-reduced sufficient statistics (Spark WeightedLeastSquares)."""
    Xd = X.to(torch.float64)
    yd = y.to(torch.float64).to(Xd.device)
    wd = torch.ones_like(yd) if w is None else w.to(torch.float64).to(Xd.device)
    D = Xd.shape[1]
    Xw = Xd * wd[:, None]
    from ..ops.gram import rows_t_matmul
    st = torch.cat([rows_t_matmul(Xw, Xd).reshape(-1), rows_t_matmul(Xw, yd), Xw.sum(0), (wd * yd).sum().reshape(1),
                    wd.sum().reshape(1), (wd * yd * yd).sum().reshape(1)])
    comm.all_reduce(st)
    st = st.cpu().numpy()
    XtX = st[: D * D].reshape(D, D)
    Xty = st[D * D: D * D + D]
    sx = st[D * D + D: D * D + 2 * D]
    sy, W = st[-3], st[-2]
    if fit_intercept:
        mx, my = sx / W, sy / W
        A = XtX / W - np.outer(mx, mx)
        bvec = Xty / W - mx * my
    else:
        A, bvec = XtX / W, Xty / W
        mx, my = np.zeros(D), 0.0
    var = np.clip(np.diag(XtX) / W - mx * mx, 0, None) * (W / max(W - 1, 1e-300))
    std = np.sqrt(var)
    # Spark: L2 penalty regParam*||beta||^2/2 on the (label-std-scaled) objective
    ystd = math.sqrt(max((st[-1] / W - (sy / W) ** 2) * (W / max(W - 1, 1e-300)), 0.0))
    lam = reg * (ystd if ystd > 0 else 1.0)
    pen = lam * (std ** 2 if standardization else np.ones(D))
    coef = np.linalg.solve(A + np.diag(pen) + 1e-12 * np.eye(D), bvec)
    b = (my - mx @ coef) if fit_intercept else 0.0
    return coef, float(b), [0.0]


@register("org.apache.spark.ml.regression.LinearRegressionModel")
class LinearRegressionModel(U.PredictionModelMixin, Model, _LinearRegressionParams, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self._w = np.zeros(0)
        self._b = 0.0
        self.summary = None

    @classmethod
    def _from(cls, w, b):
        m = cls()
        m._w, m._b = np.asarray(w, dtype=np.float64), float(b)
        return m

    @property
    def coefficients(self):
        return DenseVector(self._w)

    @property
    def intercept(self):
        return self._b

    @property
    def numFeatures(self):
        return len(self._w)

    @property
    def scale(self):
        return 1.0

    def _features_for_predict(self, df, name):
        return U.linear_features(df, name)        # sparse rows stay CSR

    def _predict_tensor(self, X):
        return U.linear_margin(X, self._w, self._b)

    def evaluate(self, df):
        """Evaluate on ``df``: a LinearRegressionSummary (metrics computed lazily)."""
        return _linreg_summary(self, df)

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"intercept": pa.array([self._b]), "coefficients": vec_col([self.coefficients]),
                          "scale": pa.array([1.0])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls._from(vector_from_struct(t["coefficients"]).toArray(), t["intercept"])
        apply_metadata(m, meta)
        return m
from ._fm import FMRegressionModel, FMRegressor  # noqa: E402,F401
from ._regression_extra import (AFTSurvivalRegression, AFTSurvivalRegressionModel,  # noqa: E402,F401
                                GeneralizedLinearRegression, GeneralizedLinearRegressionModel,
                                GeneralizedLinearRegressionTrainingSummary, IsotonicRegression,
                                IsotonicRegressionModel)
