"""IsotonicRegression, AFTSurvivalRegression and GeneralizedLinearRegression
(``pyspark.ml.regression``), reached through the Regression widget's reflection
(orangecontrib/spark/widgets/ml/spark_ml_regression.py:15).

* Isotonic: Spark's parallel PAV -- range partition by feature (all_to_all), per-rank
  PAV in C++, final PAV over the gathered blocks (models/isotonic.py).
* AFT: Weibull accelerated-failure-time model; the negative log-likelihood gradient of
  [coefficients | intercept | log sigma] is one GEMV-shaped pass per evaluation plus one
  all-reduce, minimised by L-BFGS (models/dist_opt.py).  Features are scaled by their
  standard deviation during optimisation, as in Spark.
* GLR: IRLS with one all-reduced weighted Gram matrix per iteration (models/irls.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame import column as C
from ..models import dist_opt, irls
from ..models import isotonic as ISO
from . import common as U
from .base import Estimator, Model
from .linalg import DenseVector
from .param import (HasAggregationDepth, HasFeaturesCol, HasFitIntercept, HasLabelCol, HasMaxBlockSizeInMB,
                    HasMaxIter, HasPredictionCol, HasRegParam, HasSolver, HasTol, HasWeightCol, TypeConverters,
                    keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, prim_list, read_data, register, vec_col, write_data


# ===================================================================== Isotonic
class _IsotonicRegressionParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasWeightCol):
    isotonic = shared("isotonic", "whether the output sequence should be isotonic/increasing (true) or"
                                  "antitonic/decreasing (false).", TypeConverters.toBoolean)
    featureIndex = shared("featureIndex", "The index of the feature if featuresCol is a vector column, no effect "
                                          "otherwise.", TypeConverters.toInt)

    def __init__(self):
        super().__init__()
        self._setDefault(isotonic=True, featureIndex=0)


def _feature_values(df, name: str, index: int) -> torch.Tensor:
    c = df.column_data(name)
    if isinstance(c, C.NumericColumn):
        return c.data.to(torch.float64)
    X = U.dense_features(df, name)
    return X[:, index].to(torch.float64)


@register("org.apache.spark.ml.regression.IsotonicRegression")
class IsotonicRegression(Estimator, _IsotonicRegressionParams, MLWritable, MLReadable):
    """Currently implemented using parallelized pool adjacent violators algorithm. Only
    univariate (single feature) algorithm supported."""

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", weightCol=None,
                 isotonic=True, featureIndex=0):
        super().__init__()
        self._set(**self._input_kwargs)

    @keyword_only
    def setParams(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", weightCol=None,
                  isotonic=True, featureIndex=0):
        return self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        x = _feature_values(df, g(self.featuresCol), g(self.featureIndex))
        y = U.numeric_column(df, g(self.labelCol))
        w = U.weights_or_none(df, self)
        b, p = ISO.fit_isotonic(df.comm, x, y.to(x.device), w, g(self.isotonic))
        return IsotonicRegressionModel._from(b, p)._with_parent(self)


@register("org.apache.spark.ml.regression.IsotonicRegressionModel")
class IsotonicRegressionModel(Model, _IsotonicRegressionParams, MLWritable, MLReadable):
    """Model fitted by IsotonicRegression: piecewise-linear through (boundaries, predictions)."""

    def __init__(self):
        super().__init__()
        self._bounds = np.zeros(0)
        self._preds = np.zeros(0)

    @classmethod
    def _from(cls, bounds, preds):
        m = cls()
        m._bounds, m._preds = np.asarray(bounds, float), np.asarray(preds, float)
        return m

    @property
    def boundaries(self) -> DenseVector:
        return DenseVector(self._bounds)

    @property
    def predictions(self) -> DenseVector:
        return DenseVector(self._preds)

    @property
    def numFeatures(self) -> int:
        return 1

    def _predict_x(self, x: torch.Tensor) -> torch.Tensor:
        b = torch.from_numpy(self._bounds).to(x.device)
        p = torch.from_numpy(self._preds).to(x.device)
        return ISO.predict(b, p, x.to(torch.float64))

    def predict(self, value: float) -> float:
        return float(self._predict_x(torch.tensor([float(value)], dtype=torch.float64))[0])

    def _transform(self, df):
        x = _feature_values(df, self.getOrDefault(self.featuresCol), self.getOrDefault(self.featureIndex))
        return df.withColumnData(self.getOrDefault(self.predictionCol), U.num_out(self._predict_x(x)))

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"boundaries": pa.array([self._bounds.tolist()], prim_list(pa.float64())),
                          "predictions": pa.array([self._preds.tolist()], prim_list(pa.float64())),
                          "isotonic": pa.array([bool(self.getOrDefault(self.isotonic))])})

    @classmethod
    def _load_impl(cls, path, meta):
        t = read_data(path).to_pylist()[0]
        m = cls._from(t["boundaries"], t["predictions"])
        apply_metadata(m, meta)
        return m


# ========================================================================== AFT
class _AFTSurvivalRegressionParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasMaxIter, HasTol,
                                   HasFitIntercept, HasAggregationDepth, HasMaxBlockSizeInMB):
    censorCol = shared("censorCol", "censor column name. The value of this column could be 0 or 1. If the value "
                                    "is 1, it means the event has occurred i.e. uncensored; otherwise censored.",
                       TypeConverters.toString)
    quantileProbabilities = shared("quantileProbabilities", "quantile probabilities array. Values of the quantile "
                                                            "probabilities array should be in the range (0, 1) and "
                                                            "the array should be non-empty.",
                                   TypeConverters.toListFloat)
    quantilesCol = shared("quantilesCol", "quantiles column name. This column will output quantiles of "
                                          "corresponding quantileProbabilities if it is set.",
                          TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(censorCol="censor", quantileProbabilities=[0.01, 0.05, 0.1, 0.25, 0.5, 0.75, 0.9, 0.95,
                                                                    0.99],
                         maxIter=100, tol=1e-6, fitIntercept=True, aggregationDepth=2, maxBlockSizeInMB=0.0)


def aft_nll_sum(theta: torch.Tensor, X: torch.Tensor, logt: torch.Tensor, delta: torch.Tensor,
                fit_intercept: bool) -> torch.Tensor:
    """Sum over rows of -(delta * (eps - log sigma) - exp(eps)), eps = (log t - x.b - b0)/sigma."""
    D = X.shape[1]
    beta = theta[:D]
    b0 = theta[D] if fit_intercept else theta.new_zeros(())
    log_sigma = theta[D + 1]
    eps = (logt - X @ beta - b0) * torch.exp(-log_sigma)
    return (delta * (log_sigma - eps) + torch.exp(eps)).sum()


@register("org.apache.spark.ml.regression.AFTSurvivalRegression")
class AFTSurvivalRegression(Estimator, _AFTSurvivalRegressionParams, MLWritable, MLReadable):
    """Accelerated Failure Time (AFT) Model Survival Regression. Fit a parametric AFT
    survival regression model based on the Weibull distribution of the survival time."""

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", fitIntercept=True,
                 maxIter=100, tol=1e-6, censorCol="censor",
                 quantileProbabilities=[0.01, 0.05, 0.1, 0.25, 0.5, 0.75, 0.9, 0.95, 0.99],  # noqa: B006
                 quantilesCol=None, aggregationDepth=2, maxBlockSizeInMB=0.0):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        comm = df.comm
        X = U.dense_features(df, g(self.featuresCol))
        t = U.numeric_column(df, g(self.labelCol))
        delta = U.numeric_column(df, g(self.censorCol))
        if t.numel() and float(t.min()) <= 0:
            raise ValueError("The lifetime or label should be  greater than 0.")
        dev = X.device
        dt = dist_opt.compute_dtype(dev)
        n, D = X.shape
        # feature scaling by std (no centring), like Spark's AFT aggregator
        Xf = X.to(torch.float64)
        st = torch.cat([Xf.sum(0), (Xf * Xf).sum(0), torch.tensor([float(n)], dtype=torch.float64, device=dev)])
        comm.all_reduce(st)
        N = float(st[-1])
        mean = st[:D] / max(N, 1.0)
        var = (st[D:2 * D] - N * mean * mean) / max(N - 1.0, 1.0)
        std = torch.sqrt(var.clamp_min(0)).cpu().numpy()
        inv = np.where(std > 0, 1.0 / np.where(std > 0, std, 1.0), 0.0)
        inv_t = torch.from_numpy(inv).to(dev, dt)
        logt = torch.log(t.to(dev, dt))
        dl = delta.to(dev, dt)
        fi = g(self.fitIntercept)

        def local_loss(theta, a, b):
            return aft_nll_sum(theta, X[a:b].to(dt) * inv_t, logt[a:b], dl[a:b], fi)

        obj = dist_opt.Objective(comm, dev, n, local_loss, N)
        res = dist_opt.lbfgs(obj, np.zeros(D + 2), g(self.maxIter), g(self.tol))
        coef = res.x[:D] * inv
        m = AFTSurvivalRegressionModel._from(coef, float(res.x[D]) if fi else 0.0, math.exp(res.x[D + 1]))
        return m._with_parent(self)


@register("org.apache.spark.ml.regression.AFTSurvivalRegressionModel")
class AFTSurvivalRegressionModel(Model, _AFTSurvivalRegressionParams, MLWritable, MLReadable):
    """Model fitted by AFTSurvivalRegression."""

    def __init__(self):
        super().__init__()
        self._w = np.zeros(0)
        self._b = 0.0
        self._scale = 1.0

    @classmethod
    def _from(cls, w, b, scale):
        m = cls()
        m._w, m._b, m._scale = np.asarray(w, float), float(b), float(scale)
        return m

    @property
    def coefficients(self) -> DenseVector:
        return DenseVector(self._w)

    @property
    def intercept(self) -> float:
        return self._b

    @property
    def scale(self) -> float:
        return self._scale

    @property
    def numFeatures(self) -> int:
        return int(self._w.shape[0])

    def _mu(self, X):
        w = torch.from_numpy(self._w).to(X.device)
        return torch.exp(X.to(torch.float64)[:, : w.shape[0]] @ w + self._b)

    def predict(self, features) -> float:
        x = torch.as_tensor(np.asarray(features.toArray() if hasattr(features, "toArray") else features),
                            dtype=torch.float64)
        return float(self._mu(x[None, :])[0])

    def _quantiles_of(self, mu):
        p = torch.tensor(self.getOrDefault(self.quantileProbabilities), dtype=torch.float64, device=mu.device)
        return mu[:, None] * torch.pow(-torch.log1p(-p), self._scale)[None, :]

    def predictQuantiles(self, features) -> DenseVector:
        x = torch.as_tensor(np.asarray(features.toArray() if hasattr(features, "toArray") else features),
                            dtype=torch.float64)
        return DenseVector(self._quantiles_of(self._mu(x[None, :]))[0].cpu().numpy())

    def _transform(self, df):
        X = U.dense_features(df, self.getOrDefault(self.featuresCol))
        mu = self._mu(X)
        out = df
        if self.getOrDefault(self.predictionCol):
            out = out.withColumnData(self.getOrDefault(self.predictionCol), U.num_out(mu))
        if self.isDefined(self.quantilesCol) and self.getOrDefault(self.quantilesCol):
            out = out.withColumnData(self.getOrDefault(self.quantilesCol), U.vec_out(self._quantiles_of(mu)))
        return out

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"coefficients": vec_col([self.coefficients]), "intercept": pa.array([self._b]),
                          "scale": pa.array([self._scale])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls._from(vector_from_struct(t["coefficients"]).toArray(), t["intercept"], t["scale"])
        apply_metadata(m, meta)
        return m


# ========================================================================== GLR
class _GLRParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasFitIntercept, HasMaxIter, HasTol, HasRegParam,
                 HasWeightCol, HasSolver, HasAggregationDepth):
    family = shared("family", "The name of family which is a description of the error distribution to be used "
                              "in the model. Supported options: gaussian (default), binomial, poisson, gamma and "
                              "tweedie.", TypeConverters.toString)
    link = shared("link", "The name of link function which provides the relationship between the linear "
                          "predictor and the mean of the distribution function. Supported options: identity, log, "
                          "inverse, logit, probit, cloglog and sqrt.", TypeConverters.toString)
    linkPredictionCol = shared("linkPredictionCol", "link prediction (linear predictor) column name",
                               TypeConverters.toString)
    variancePower = shared("variancePower", "The power in the variance function of the Tweedie distribution "
                                            "which characterizes the relationship between the variance and mean of "
                                            "the distribution. Only applicable for the Tweedie family. Supported "
                                            "values: 0 and [1, Inf).", TypeConverters.toFloat)
    linkPower = shared("linkPower", "The index in the power link function. Only applicable to the Tweedie "
                                    "family.", TypeConverters.toFloat)
    offsetCol = shared("offsetCol", "The offset column name. If this is not set or empty, we treat all instance "
                                    "offsets as 0.0", TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(family="gaussian", maxIter=25, tol=1e-6, regParam=0.0, solver="irls", variancePower=0.0,
                         aggregationDepth=2, fitIntercept=True)

    def _family_link(self):
        g = self.getOrDefault
        fam = g(self.family).lower()
        vp = float(g(self.variancePower))
        lk = g(self.link) if self.isDefined(self.link) else None
        lp = g(self.linkPower) if self.isDefined(self.linkPower) else None
        return irls.Family(fam, vp), irls.make_link(fam, lk, vp, lp)


class GeneralizedLinearRegressionTrainingSummary:
    def __init__(self, r: irls.IrlsResult, family: str, D: int, fit_intercept: bool):
        from scipy import stats
        self.numIterations = r.iterations
        self.solver = "irls"
        self.deviance = r.deviance
        self.nullDeviance = r.null_deviance
        self.dispersion = r.dispersion
        self.rank = r.rank
        self.numInstances = int(r.n_obs)
        self.degreesOfFreedom = r.rank
        self.residualDegreeOfFreedom = int(r.n_obs - r.rank)
        self.residualDegreeOfFreedomNull = int(r.n_obs - (1 if fit_intercept else 0))
        if r.cov_unscaled is not None:
            se = np.sqrt(np.maximum(np.diag(r.cov_unscaled) * r.dispersion, 0))
            est = np.concatenate([r.coef, [r.intercept]]) if fit_intercept else r.coef
            self.coefficientStandardErrors = se.tolist()
            self.tValues = (est / np.where(se > 0, se, np.nan)).tolist()
            if family in ("binomial", "poisson"):
                self.pValues = (2 * stats.norm.sf(np.abs(self.tValues))).tolist()
            else:
                self.pValues = (2 * stats.t.sf(np.abs(self.tValues), max(self.residualDegreeOfFreedom, 1))).tolist()
        self.aic = None


@register("org.apache.spark.ml.regression.GeneralizedLinearRegression")
class GeneralizedLinearRegression(Estimator, _GLRParams, MLWritable, MLReadable):
    """Generalized Linear Regression. Fit a Generalized Linear Model specified by giving a
    symbolic description of the linear predictor (link function) and a description of the
    error distribution (family). It supports "gaussian", "binomial", "poisson", "gamma" and
    "tweedie" as family."""

    @keyword_only
    def __init__(self, *, labelCol="label", featuresCol="features", predictionCol="prediction", family="gaussian",
                 link=None, fitIntercept=True, maxIter=25, tol=1e-6, regParam=0.0, weightCol=None, solver="irls",
                 linkPredictionCol=None, variancePower=0.0, linkPower=None, offsetCol=None, aggregationDepth=2):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        fam, lk = self._family_link()
        X = U.dense_features(df, g(self.featuresCol))
        y = U.numeric_column(df, g(self.labelCol))
        w = U.weights_or_none(df, self)
        off = None
        if self.isDefined(self.offsetCol) and g(self.offsetCol):
            off = U.numeric_column(df, g(self.offsetCol))
        r = irls.fit_irls(df.comm, X, y, w, off, fam, lk, g(self.fitIntercept), g(self.regParam), g(self.maxIter),
                          g(self.tol))
        m = GeneralizedLinearRegressionModel._from(r.coef, r.intercept)
        m.summary = GeneralizedLinearRegressionTrainingSummary(r, fam.name, X.shape[1], g(self.fitIntercept))
        return m._with_parent(self)


@register("org.apache.spark.ml.regression.GeneralizedLinearRegressionModel")
class GeneralizedLinearRegressionModel(Model, _GLRParams, MLWritable, MLReadable):
    """Model fitted by GeneralizedLinearRegression."""

    def __init__(self):
        super().__init__()
        self._w = np.zeros(0)
        self._b = 0.0
        self.summary = None

    @classmethod
    def _from(cls, w, b):
        m = cls()
        m._w, m._b = np.asarray(w, float), float(b)
        return m

    @property
    def coefficients(self) -> DenseVector:
        return DenseVector(self._w)

    @property
    def intercept(self) -> float:
        return self._b

    @property
    def numFeatures(self) -> int:
        return int(self._w.shape[0])

    @property
    def hasSummary(self) -> bool:
        return self.summary is not None

    def _eta(self, X, df=None):
        w = torch.from_numpy(self._w).to(X.device)
        eta = X.to(torch.float64)[:, : w.shape[0]] @ w + self._b
        if df is not None and self.isDefined(self.offsetCol) and self.getOrDefault(self.offsetCol):
            eta = eta + U.numeric_column(df, self.getOrDefault(self.offsetCol)).to(X.device)
        return eta

    def predict(self, features) -> float:
        x = torch.as_tensor(np.asarray(features.toArray() if hasattr(features, "toArray") else features),
                            dtype=torch.float64)
        _, lk = self._family_link()
        return float(lk.unlink(self._eta(x[None, :]))[0])

    def _transform(self, df):
        X = U.dense_features(df, self.getOrDefault(self.featuresCol))
        _, lk = self._family_link()
        eta = self._eta(X, df)
        out = df
        if self.getOrDefault(self.predictionCol):
            out = out.withColumnData(self.getOrDefault(self.predictionCol), U.num_out(lk.unlink(eta)))
        if self.isDefined(self.linkPredictionCol) and self.getOrDefault(self.linkPredictionCol):
            out = out.withColumnData(self.getOrDefault(self.linkPredictionCol), U.num_out(eta))
        return out

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"intercept": pa.array([self._b]), "coefficients": vec_col([self.coefficients])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls._from(vector_from_struct(t["coefficients"]).toArray(), t["intercept"])
        apply_metadata(m, meta)
        return m
