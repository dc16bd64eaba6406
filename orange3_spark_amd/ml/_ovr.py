"""OneVsRest (``pyspark.ml.classification.OneVsRest``): reduction of K-class
classification to K binary problems.

In the reference the Classification widget lists OneVsRest but cannot configure it (its
``classifier`` param is an object that no GuiParam can type); here it is
usable from the API, the Pipeline/Tuning widgets and scripts.  Each binary fit is an
ordinary data-parallel fit of the wrapped classifier on a relabelled view of the same
sharded DataFrame (no copy of the feature column).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..frame import column as C
from . import common as U
from .base import Estimator, Model
from .param import (HasFeaturesCol, HasLabelCol, HasPredictionCol, HasRawPredictionCol, HasWeightCol,
                    TypeConverters, keyword_only, shared)
from .util import (MLReadable, MLWritable, MLWriter, apply_metadata, load_metadata, py_class, register,
                   save_metadata)


class _OneVsRestParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasRawPredictionCol, HasWeightCol):
    classifier = shared("classifier", "base binary classifier")
    parallelism = shared("parallelism", "the number of threads to use when running parallel algorithms (>= 1).",
                         TypeConverters.toInt)

    def __init__(self):
        super().__init__()
        self._setDefault(parallelism=1)


def _binary_label(k: int) -> str:
    return f"mc2b${k}"


@register("org.apache.spark.ml.classification.OneVsRest")
class OneVsRest(Estimator, _OneVsRestParams, MLWritable, MLReadable):
    """Reduction of Multiclass Classification to Binary Classification. Performs reduction
    using one against all strategy. For a multiclass classification with k classes, train k
    models (one per class). Each example is scored against all k models and the model with
    highest score is picked to label the example.
    """

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction",
                 rawPredictionCol="rawPrediction", classifier=None, weightCol=None, parallelism=1):
        super().__init__()
        self._set(**self._input_kwargs)

    @keyword_only
    def setParams(self, *, featuresCol="features", labelCol="label", predictionCol="prediction",
                  rawPredictionCol="rawPrediction", classifier=None, weightCol=None, parallelism=1):
        return self._set(**self._input_kwargs)

    def setClassifier(self, value):
        return self._set(classifier=value)

    def getClassifier(self):
        return self.getOrDefault(self.classifier)

    def _fit(self, df):
        g = self.getOrDefault
        if not self.isDefined(self.classifier) or g(self.classifier) is None:
            raise ValueError("OneVsRest requires a classifier")
        clf = g(self.classifier)
        y = U.numeric_column(df, g(self.labelCol))
        K = U.num_classes(df.comm, y)
        models = []
        for k in range(K):
            col = _binary_label(k)
            view = df.withColumnData(col, C.NumericColumn((y == k).to(torch.float64)))
            extra = {clf.getParam("labelCol"): col, clf.getParam("featuresCol"): g(self.featuresCol)}
            if self.isDefined(self.weightCol) and g(self.weightCol) and clf.hasParam("weightCol"):
                extra[clf.getParam("weightCol")] = g(self.weightCol)
            models.append(clf.fit(view, extra))
        return OneVsRestModel(models)._with_parent(self)

    def copy(self, extra=None):
        that = super().copy(extra)
        if self.isDefined(self.classifier) and self.getOrDefault(self.classifier) is not None:
            that._set(classifier=self.getOrDefault(self.classifier).copy())
        return that

    def write(self):
        return _OvrWriter(self)

    @classmethod
    def _load_impl(cls, path, meta):
        est = cls()
        apply_metadata(est, meta)
        cp = os.path.join(path, "classifier")
        if os.path.isdir(cp):
            est._set(classifier=_load_any(cp))
        return est


def _load_any(path):
    m = load_metadata(path)
    klass = py_class(m["class"])
    if hasattr(klass, "_load_impl"):
        return klass._load_impl(path, m)
    inst = klass()
    apply_metadata(inst, m)
    return inst


class _OvrWriter(MLWriter):
    def saveImpl(self, path):
        inst = self.instance
        clf = inst.getOrDefault(inst.classifier) if inst.isDefined(inst.classifier) else None
        models = getattr(inst, "models", None)
        extra = {"numClasses": len(models)} if models is not None else None
        save_metadata(inst, path, extra, paramMap=_plain_params(inst))
        if clf is not None:
            clf.write().saveImpl(os.path.join(path, "classifier"))
        for i, m in enumerate(models or []):
            m.write().saveImpl(os.path.join(path, f"model_{i}"))


def _plain_params(inst):
    from .util import _jsonable
    return {p.name: _jsonable(v) for p, v in inst._paramMap.items() if p.name != "classifier"}


@register("org.apache.spark.ml.classification.OneVsRestModel")
class OneVsRestModel(Model, _OneVsRestParams, MLWritable, MLReadable):
    """Model fitted by OneVsRest: K binary models; prediction = argmax of their scores."""

    def __init__(self, models=None):
        super().__init__()
        self.models = list(models or [])

    def _scores(self, df):
        cols = []
        for m in self.models:
            rc = m.getOrDefault(m.rawPredictionCol) if m.hasParam("rawPredictionCol") else ""
            if rc and hasattr(m, "_raw"):
                X = m._features_for_predict(df, m.getOrDefault(m.featuresCol)) \
                    if hasattr(m, "_features_for_predict") else U.dense_features(df, m.getOrDefault(m.featuresCol))
                cols.append(m._raw(X)[:, 1].to(torch.float64))
            else:
                out = m.transform(df)
                cols.append(out.column_data(rc or "rawPrediction").dense()[:, 1].to(torch.float64))
        return torch.stack(cols, dim=1)

    def _transform(self, df):
        raw = self._scores(df)
        out = df
        rc = self.getOrDefault(self.rawPredictionCol)
        if rc:
            out = out.withColumnData(rc, U.vec_out(raw))
        pc = self.getOrDefault(self.predictionCol)
        if pc:
            out = out.withColumnData(pc, U.num_out(raw.argmax(1).to(torch.float64)))
        return out

    @property
    def numClasses(self):
        return len(self.models)

    def write(self):
        return _OvrWriter(self)

    @classmethod
    def _load_impl(cls, path, meta):
        k = int(meta.get("numClasses", 0))
        models = [_load_any(os.path.join(path, f"model_{i}")) for i in range(k)]
        m = cls(models)
        apply_metadata(m, meta)
        cp = os.path.join(path, "classifier")
        if os.path.isdir(cp):
            m._set(classifier=_load_any(cp))
        return m


_ = np
