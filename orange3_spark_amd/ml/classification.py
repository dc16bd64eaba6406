"""Classification estimators (``pyspark.ml.classification`` surface).

Reached in the reference by the Classification widget, which reflects over this module
(orangecontrib/spark/widgets/ml/spark_ml_classification.py:15) and calls
``fit(df, params=...)`` (base/spark_ml_estimator.py:19-25).
"""
from __future__ import annotations

import numpy as np
import torch

from ..frame import column as C
from ..models import glm as GLM
from ..ops import glm as G
from ..synthetic import LineageVectorColumn
from . import common as U
from .base import Estimator, Model
from .linalg import DenseMatrix, DenseVector, Vectors
from .param import (HasAggregationDepth, HasElasticNetParam, HasFeaturesCol, HasFitIntercept, HasLabelCol,
                    HasMaxBlockSizeInMB, HasMaxIter, HasPredictionCol, HasProbabilityCol, HasRawPredictionCol,
                    HasRegParam, HasSeed, HasStandardization, HasStepSize, HasThreshold, HasThresholds, HasTol,
                    HasWeightCol, TypeConverters, add_accessors, keyword_only, shared)
from ..runtime.checkpoint import for_estimator
from .util import MLReadable, MLWritable, apply_metadata, mat_col, read_data, register, vec_col, write_data


from . import _summary as S  # noqa: E402


def _lr_summary(model, df, training, res=None):
    """Spark (Binary)LogisticRegression(Training)Summary over ``model.transform(df)``."""
    g = model.getOrDefault
    kw = dict(labelCol=g(model.labelCol), predictionCol=g(model.predictionCol),
              probabilityCol=g(model.probabilityCol), featuresCol=g(model.featuresCol),
              weightCol=g(model.weightCol) if model.isDefined(model.weightCol) and g(model.weightCol) else None)
    pred = (lambda: model.transform(df))
    binary = not model._multinomial
    if training:
        cls = S.BinaryLogisticRegressionTrainingSummary if binary else S.LogisticRegressionTrainingSummary
        return cls(pred, res.history, res.iterations, getattr(res, "seconds", 0.0), getattr(res, "passes", 0), **kw)
    return (S.BinaryLogisticRegressionSummary if binary else S.LogisticRegressionSummary)(pred, **kw)


def _svc_summary(model, df, res=None):
    g = model.getOrDefault
    kw = dict(labelCol=g(model.labelCol), predictionCol=g(model.predictionCol),
              weightCol=g(model.weightCol) if model.isDefined(model.weightCol) and g(model.weightCol) else None)
    pred = (lambda: model.transform(df))
    if res is None:
        return S.LinearSVCSummary(pred, **kw)
    return S.LinearSVCTrainingSummary(pred, res.history, res.iterations, res.seconds, res.passes, **kw)


# ====================================================================== Logistic
class _LogisticRegressionParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasProbabilityCol,
                                HasRawPredictionCol, HasMaxIter, HasRegParam, HasElasticNetParam, HasTol,
                                HasFitIntercept, HasThreshold, HasThresholds, HasStandardization, HasWeightCol,
                                HasAggregationDepth, HasStepSize, HasMaxBlockSizeInMB, HasSeed):
    family = shared("family", "The name of family which is a description of the label distribution to be used in "
                              "the model. Supported options: auto, binomial, multinomial", TypeConverters.toString)
    solver = shared("solver", "The solver algorithm for optimization. Supported options: auto, l-bfgs, sgd "
                              "(sgd = mini-batch gradient descent with stepSize/sqrt(t) steps, mllib "
                              "GradientDescent semantics).",
                    TypeConverters.toString)
    miniBatchFraction = shared("miniBatchFraction", "Fraction of rows used per SGD iteration, in (0, 1]; each "
                                                    "iteration draws its own Bernoulli sample keyed on (seed, "
                                                    "iteration, row).", TypeConverters.toFloat)

    def __init__(self):
        super().__init__()
        self._setDefault(maxIter=100, regParam=0.0, tol=1e-6, threshold=0.5, family="auto", solver="auto",
                         stepSize=1.0, miniBatchFraction=1.0, elasticNetParam=0.0, fitIntercept=True,
                         standardization=True, seed=42)


@add_accessors
@register("org.apache.spark.ml.classification.LogisticRegression")
class LogisticRegression(Estimator, _LogisticRegressionParams, MLWritable, MLReadable):
    """Logistic regression. Supports multinomial logistic (softmax) and binomial logistic
    regression, L2 / L1 / elastic-net regularisation.  Binomial training streams bf16
    features through the fused gfx950 gradient kernel with one RCCL all-reduce per pass.
    """
    _warm_family = "glm"          # runtime/warmup.py lazy warm-up

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxIter=100,
                 regParam=0.0, elasticNetParam=0.0, tol=1e-6, fitIntercept=True, threshold=0.5, thresholds=None,
                 probabilityCol="probability", rawPredictionCol="rawPrediction", standardization=True,
                 weightCol=None, aggregationDepth=2, family="auto", solver="auto", stepSize=1.0,
                 miniBatchFraction=1.0, maxBlockSizeInMB=0.0, seed=42):
        super().__init__()
        self._set(**self._input_kwargs)

    @keyword_only
    def setParams(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxIter=100,
                  regParam=0.0, elasticNetParam=0.0, tol=1e-6, fitIntercept=True, threshold=0.5, thresholds=None,
                  probabilityCol="probability", rawPredictionCol="rawPrediction", standardization=True,
                  weightCol=None, aggregationDepth=2, family="auto", solver="auto", stepSize=1.0,
                  miniBatchFraction=1.0, maxBlockSizeInMB=0.0, seed=42):
        return self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        comm = df.comm
        feat = U.features_column(df, g(self.featuresCol))
        y = U.numeric_column(df, g(self.labelCol), None)      # storage dtype: no 1B-row copy
        sw = U.weights_or_none(df, self)
        k = U.num_classes(comm, y)
        fam = g(self.family).lower()
        if fam == "binomial" and k > 2:
            raise ValueError(f"Binomial family only supports 1 or 2 outcome classes but found {k}.")
        multinomial = fam == "multinomial" or (fam == "auto" and k > 2)
        if multinomial:
            X = U.dense_features(df, g(self.featuresCol))
            B, b, r = GLM.fit_multinomial(comm, X, y, sw, max(k, 2), g(self.regParam), g(self.elasticNetParam),
                                          g(self.fitIntercept), g(self.standardization), g(self.maxIter), g(self.tol))
            m = LogisticRegressionModel._from(B, b, True, max(k, 2))._with_parent(self)
            m.summary = _lr_summary(m, df, True, r)
            return m
        data = GLM.make_glm_data(comm, feat, y, sw)
        solver = g(self.solver).lower()
        res = GLM.fit_glm(data, "logistic", g(self.regParam), g(self.elasticNetParam), g(self.fitIntercept),
                          g(self.standardization), g(self.maxIter), g(self.tol),
                          "sgd" if solver == "sgd" else "auto", g(self.stepSize), g(self.miniBatchFraction),
                          g(self.seed), ckpt=for_estimator(self, df))
        m = LogisticRegressionModel._from(res.coef[None, :], np.array([res.intercept]), False, 2)._with_parent(self)
        m.summary = _lr_summary(m, df, True, res)
        m._fit_setup_seconds = getattr(res, "setup_seconds", 0.0)
        return m

    def trainer(self, df):
        """Device-resident SGD stepper for this estimator's params (the engine of
        ``fit(solver='sgd')``, exposed for step-level tests and tools)."""
        g = self.getOrDefault
        feat = U.features_column(df, g(self.featuresCol))
        y = U.numeric_column(df, g(self.labelCol), torch.float32)
        data = GLM.GlmData(df.comm, feat, y, U.weights_or_none(df, self))
        std = None
        if g(self.standardization):
            _, var, *_ = data.moments()
            std = np.sqrt(var)
        return GLM.DeviceSGD(data, "logistic", g(self.regParam), g(self.fitIntercept), g(self.stepSize),
                             g(self.standardization), std, elastic_net=g(self.elasticNetParam),
                             mini_batch_fraction=g(self.miniBatchFraction), seed=g(self.seed))


@register("org.apache.spark.ml.classification.LogisticRegressionModel")
class LogisticRegressionModel(U.ProbabilisticClassifierMixin, Model, _LogisticRegressionParams, MLWritable,
                              MLReadable):
    """Model fitted by LogisticRegression."""

    def __init__(self):
        super().__init__()
        self._B = np.zeros((1, 0))
        self._b = np.zeros(1)
        self._multinomial = False
        self.numClasses = 2
        self.summary = None

    @classmethod
    def _from(cls, B, b, multinomial, num_classes):
        m = cls()
        m._B = np.asarray(B, dtype=np.float64)
        m._b = np.asarray(b, dtype=np.float64)
        m._multinomial = bool(multinomial)
        m.numClasses = int(num_classes)
        return m

    @property
    def numFeatures(self) -> int:
        return int(self._B.shape[1])

    @property
    def coefficients(self) -> DenseVector:
        if self._multinomial:
            raise ValueError("Multinomial models contain a matrix of coefficients, use coefficientMatrix instead.")
        return DenseVector(self._B[0])

    @property
    def intercept(self) -> float:
        if self._multinomial:
            raise ValueError("Multinomial models contain a vector of intercepts, use interceptVector instead.")
        return float(self._b[0])

    @property
    def coefficientMatrix(self) -> DenseMatrix:
        return DenseMatrix.from_array(self._B)

    @property
    def interceptVector(self) -> DenseVector:
        return DenseVector(self._b)

    @property
    def hasSummary(self) -> bool:
        return self.summary is not None

    def _features_for_predict(self, df, name):
        from ..frame.spill import SpilledVectorColumn
        c = U.features_column(df, name)
        if isinstance(c, SpilledVectorColumn) and c.data.is_cuda and c.data.dtype == torch.bfloat16 \
                and not self._multinomial:
            return c                 # resident + host-streamed rows -> margin kernel per chunk
        if isinstance(c, C.VectorColumn) and c.data.is_cuda and c.data.dtype == torch.bfloat16 \
                and not self._multinomial and not isinstance(c, (LineageVectorColumn, SpilledVectorColumn)):
            return c.data            # padded bf16 -> margin kernel
        if isinstance(c, C.SparseVectorColumn) and not self._multinomial:
            return U.linear_features(df, name)     # CSR rows -> sparse margin kernel
        return U.dense_features(df, name)

    def _raw(self, X):
        from ..frame.spill import SpilledVectorColumn, map_rows
        if isinstance(X, SpilledVectorColumn):
            w = torch.from_numpy(self._B[0]).float().to(X.data.device)
            m = map_rows(X, lambda Xc: G.glm_margin(Xc, w, float(self._b[0])).double())
            return torch.stack([-m, m], dim=1)
        if not self._multinomial:
            if isinstance(X, torch.Tensor) and X.is_cuda and X.dtype == torch.bfloat16:
                m = G.glm_margin(X, torch.from_numpy(self._B[0]).float().to(X.device), float(self._b[0])).double()
            else:
                m = U.linear_margin(X, self._B[0], float(self._b[0]))
            return torch.stack([-m, m], dim=1)
        W = torch.from_numpy(self._B.T).to(X.device, torch.float32 if X.is_cuda else torch.float64)
        b = torch.from_numpy(self._b).to(X.device, W.dtype)
        return (X.to(W.dtype) @ W + b).to(torch.float64)

    def _raw2prob(self, raw):
        if not self._multinomial:
            p = torch.sigmoid(raw[:, 1])
            return torch.stack([1 - p, p], dim=1)
        return torch.softmax(raw, dim=1)

    def evaluate(self, df):
        """Evaluate on ``df``: a (Binary)LogisticRegressionSummary (metrics computed lazily)."""
        return _lr_summary(self, df, False)

    # persistence (Spark >= 2.1 LogisticRegressionModel data schema)
    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {
            "numClasses": pa.array([self.numClasses], pa.int32()),
            "numFeatures": pa.array([self.numFeatures], pa.int32()),
            "interceptVector": vec_col([self.interceptVector]),
            "coefficientMatrix": mat_col([self.coefficientMatrix]),
            "isMultinomial": pa.array([self._multinomial], pa.bool_()),
        })

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import matrix_from_struct, vector_from_struct
        t = read_data(path).to_pylist()[0]
        B = matrix_from_struct(t["coefficientMatrix"]).toArray()
        b = vector_from_struct(t["interceptVector"]).toArray()
        m = cls._from(B, b, t["isMultinomial"], t["numClasses"])
        apply_metadata(m, meta)
        return m


# ====================================================================== LinearSVC
class _LinearSVCParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasRawPredictionCol, HasMaxIter,
                       HasRegParam, HasTol, HasFitIntercept, HasStandardization, HasThreshold, HasWeightCol,
                       HasAggregationDepth, HasMaxBlockSizeInMB, HasStepSize):
    solver = shared("solver", "The solver algorithm for optimization. Supported options: auto, l-bfgs, sgd.",
                    TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(maxIter=100, regParam=0.0, tol=1e-6, fitIntercept=True, standardization=True,
                         threshold=0.0, solver="auto", stepSize=1.0)


@add_accessors
@register("org.apache.spark.ml.classification.LinearSVC")
class LinearSVC(Estimator, _LinearSVCParams, MLWritable, MLReadable):
    """Linear SVM classifier (hinge loss, L2 regularisation); same fused kernel as
    LogisticRegression with a hinge epilogue (beyond-ref: Spark >= 2.2)."""
    _warm_family = "glm"          # runtime/warmup.py lazy warm-up

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxIter=100,
                 regParam=0.0, tol=1e-6, rawPredictionCol="rawPrediction", fitIntercept=True, standardization=True,
                 threshold=0.0, weightCol=None, aggregationDepth=2, maxBlockSizeInMB=0.0, solver="auto",
                 stepSize=1.0):
        super().__init__()
        self._set(**self._input_kwargs)

    @keyword_only
    def setParams(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxIter=100,
                  regParam=0.0, tol=1e-6, rawPredictionCol="rawPrediction", fitIntercept=True, standardization=True,
                  threshold=0.0, weightCol=None, aggregationDepth=2, maxBlockSizeInMB=0.0, solver="auto",
                  stepSize=1.0):
        return self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        comm = df.comm
        y = U.numeric_column(df, g(self.labelCol), None)
        k = U.num_classes(comm, y)
        if k > 2:
            raise ValueError(f"LinearSVC only supports binary classification. {k} classes detected in labelCol")
        data = GLM.make_glm_data(comm, U.features_column(df, g(self.featuresCol)), y, U.weights_or_none(df, self))
        res = GLM.fit_glm(data, "hinge", g(self.regParam), 0.0, g(self.fitIntercept), g(self.standardization),
                          g(self.maxIter), g(self.tol), "sgd" if g(self.solver) == "sgd" else "auto",
                          g(self.stepSize), init_intercept=0.0, ckpt=for_estimator(self, df))
        m = LinearSVCModel._from(res.coef, res.intercept)._with_parent(self)
        m.summary = _svc_summary(m, df, res)
        return m


@register("org.apache.spark.ml.classification.LinearSVCModel")
class LinearSVCModel(U.ProbabilisticClassifierMixin, Model, _LinearSVCParams, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self._w = np.zeros(0)
        self._b = 0.0
        self.numClasses = 2
        self.summary = None

    @classmethod
    def _from(cls, w, b):
        m = cls()
        m._w, m._b = np.asarray(w, dtype=np.float64), float(b)
        return m

    def evaluate(self, df):
        """Evaluate on ``df``: a LinearSVCSummary (binary metrics on rawPrediction)."""
        return _svc_summary(self, df)

    @property
    def coefficients(self):
        return DenseVector(self._w)

    @property
    def intercept(self):
        return self._b

    @property
    def numFeatures(self):
        return int(self._w.shape[0])

    def _features_for_predict(self, df, name):
        return U.linear_features(df, name)        # sparse rows stay CSR

    def _raw(self, X):
        if isinstance(X, torch.Tensor) and X.is_cuda and X.dtype == torch.bfloat16:
            m = G.glm_margin(X, torch.from_numpy(self._w).float().to(X.device), self._b).double()
        else:
            m = U.linear_margin(X, self._w, self._b)
        return torch.stack([-m, m], dim=1)

    def _raw2prob(self, raw):
        return raw

    def _prob2pred(self, raw):
        return (raw[:, 1] > self.getOrDefault(self.threshold)).to(torch.float64)

    def _transform(self, df):
        X = U.dense_features(df, self.getOrDefault(self.featuresCol))
        raw = self._raw(X)
        out = df
        if self.getOrDefault(self.rawPredictionCol):
            out = out.withColumnData(self.getOrDefault(self.rawPredictionCol), U.vec_out(raw))
        if self.getOrDefault(self.predictionCol):
            out = out.withColumnData(self.getOrDefault(self.predictionCol), U.num_out(self._prob2pred(raw)))
        return out

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"coefficients": vec_col([self.coefficients]), "intercept": pa.array([self._b])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls._from(vector_from_struct(t["coefficients"]).toArray(), t["intercept"])
        apply_metadata(m, meta)
        return m


_ = Vectors


from ._tree import (DecisionTreeClassificationModel, DecisionTreeClassifier, GBTClassificationModel,  # noqa: E402,F401
                    GBTClassifier, RandomForestClassificationModel, RandomForestClassifier)
from ._fm import FMClassificationModel, FMClassifier  # noqa: E402,F401
from ._mlp import MultilayerPerceptronClassificationModel, MultilayerPerceptronClassifier  # noqa: E402,F401
from ._nb import NaiveBayes, NaiveBayesModel  # noqa: E402,F401
from ._ovr import OneVsRest, OneVsRestModel  # noqa: E402,F401
