"""Model selection (``pyspark.ml.tuning``): ParamGridBuilder, CrossValidator, TrainValidationSplit.

Listed by the reference's ``get_ml_modules`` (orangecontrib/spark/utils/ml_api_utils.py:76-78)
but never exposed by a widget there; the add-on's Tuning widget uses it.  Folds are
assigned by the counter-hash of (seed, global row), so they are identical on any number
of GPUs.
"""
from __future__ import annotations

import numpy as np

from ..ops import sampling
from .base import Estimator, Evaluator, Model
from .param import HasSeed, Param, ParamGridBuilder, TypeConverters, keyword_only, shared  # noqa: F401
from .util import MLReadable, MLWritable, register


class _ValidatorParams(HasSeed):
    estimator = shared("estimator", "estimator to be cross-validated")
    estimatorParamMaps = shared("estimatorParamMaps", "estimator param maps")
    evaluator = shared("evaluator", "evaluator used to select hyper-parameters that maximize the validator metric")
    parallelism = shared("parallelism", "the number of threads to use when running parallel algorithms (>= 1).",
                         TypeConverters.toInt)
    collectSubModels = shared("collectSubModels", "Param for whether to collect a list of sub-models trained "
                              "during tuning. If set to false, then only the single best sub-model will be "
                              "available after fitting.", TypeConverters.toBoolean)

    def __init__(self):
        super().__init__()
        self._setDefault(parallelism=1, collectSubModels=False, seed=0)

    def _maps(self):
        maps = self.getOrDefault(self.estimatorParamMaps) if self.isDefined(self.estimatorParamMaps) else None
        return maps or [{}]


def _rebind(est, pm):
    """Param maps may carry Params of another instance (same name): rebind by name."""
    return {est.getParam(p.name if isinstance(p, Param) else p): v for p, v in pm.items()}


@register("org.apache.spark.ml.tuning.CrossValidator")
class CrossValidator(Estimator, _ValidatorParams, MLWritable, MLReadable):
    """K-fold cross validation performs model selection by splitting the dataset into a set of
    non-overlapping randomly partitioned folds which are used as separate training and test datasets."""

    numFolds = shared("numFolds", "number of folds for cross validation", TypeConverters.toInt)
    foldCol = shared("foldCol", "Param for the column name of user specified fold number. Once this is specified, "
                                ":py:class:`CrossValidator` won't do random k-fold split. Note that this column "
                                "should be integer type with range [0, numFolds) and Spark will throw exception on "
                                "out-of-range fold numbers.", TypeConverters.toString)

    @keyword_only
    def __init__(self, *, estimator=None, estimatorParamMaps=None, evaluator=None, numFolds=3, seed=None,
                 parallelism=1, collectSubModels=False, foldCol=""):
        super().__init__()
        self._setDefault(numFolds=3, foldCol="")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        est, ev = self.getOrDefault(self.estimator), self.getOrDefault(self.evaluator)
        maps = self._maps()
        k = self.getOrDefault(self.numFolds)
        fc = self.getOrDefault(self.foldCol)
        if fc:
            fold = df.column_data(fc).data.long()
        else:
            u = sampling.uniform(df._global_rows(), self.getOrDefault(self.seed), stream=3)
            fold = (u * k).long().clamp_max(k - 1)
        metrics = np.zeros(len(maps))
        subs = [[None] * len(maps) for _ in range(k)]
        for f in range(k):
            train, test = df._mask(fold != f), df._mask(fold == f)
            for i, pm in enumerate(maps):
                m = est.fit(train, _rebind(est, pm))
                metrics[i] += ev.evaluate(m.transform(test)) / k
                if self.getOrDefault(self.collectSubModels):
                    subs[f][i] = m
        best = int(np.argmax(metrics) if ev.isLargerBetter() else np.argmin(metrics))
        bm = est.fit(df, _rebind(est, maps[best]))
        cvm = CrossValidatorModel(bm, list(metrics), subs if self.getOrDefault(self.collectSubModels) else None)
        return cvm._with_parent(self)


@register("org.apache.spark.ml.tuning.CrossValidatorModel")
class CrossValidatorModel(Model, _ValidatorParams, MLWritable, MLReadable):
    numFolds = CrossValidator.numFolds

    def __init__(self, bestModel=None, avgMetrics=None, subModels=None):
        super().__init__()
        self.bestModel = bestModel
        self.avgMetrics = avgMetrics or []
        self.subModels = subModels

    def _transform(self, df):
        return self.bestModel.transform(df)


@register("org.apache.spark.ml.tuning.TrainValidationSplit")
class TrainValidationSplit(Estimator, _ValidatorParams, MLWritable, MLReadable):
    """Validation for hyper-parameter tuning. Randomly splits the input dataset into train and
    validation sets, and uses evaluation metric on the validation set to select the best model."""

    trainRatio = shared("trainRatio", "Param for ratio between train and validation data. Must be between 0 and 1.",
                        TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, estimator=None, estimatorParamMaps=None, evaluator=None, trainRatio=0.75, parallelism=1,
                 collectSubModels=False, seed=None):
        super().__init__()
        self._setDefault(trainRatio=0.75)
        self._set(**self._input_kwargs)

    def _fit(self, df):
        est, ev = self.getOrDefault(self.estimator), self.getOrDefault(self.evaluator)
        maps = self._maps()
        r = self.getOrDefault(self.trainRatio)
        train, valid = df.randomSplit([r, 1 - r], self.getOrDefault(self.seed))
        metrics = [ev.evaluate(est.fit(train, _rebind(est, pm)).transform(valid)) for pm in maps]
        best = int(np.argmax(metrics) if ev.isLargerBetter() else np.argmin(metrics))
        return TrainValidationSplitModel(est.fit(df, _rebind(est, maps[best])), metrics)._with_parent(self)


@register("org.apache.spark.ml.tuning.TrainValidationSplitModel")
class TrainValidationSplitModel(Model, _ValidatorParams, MLWritable, MLReadable):
    trainRatio = TrainValidationSplit.trainRatio

    def __init__(self, bestModel=None, validationMetrics=None):
        super().__init__()
        self.bestModel = bestModel
        self.validationMetrics = validationMetrics or []

    def _transform(self, df):
        return self.bestModel.transform(df)


_ = Evaluator
