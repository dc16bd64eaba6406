"""Estimator / Transformer / Model / Evaluator / Pipeline (``pyspark.ml`` base API).

The reference's generic widgets call exactly these entry points:
``method().fit(in_df, params=paramMap)`` (orangecontrib/spark/base/spark_ml_estimator.py:19-25),
``method_instance.transform(in_df, params=paramMap)`` (base/spark_ml_transformer.py:129-139),
``model.transform(df)`` (widgets/ml/spark_ml_model.py:53) and an Evaluator's
``evaluate`` (widgets/ml/spark_ml_evaluation.py:42-78).  ``Pipeline``/``PipelineModel``
are beyond-ref (BASELINE north star).
"""
from __future__ import annotations

import os
from abc import ABC, abstractmethod

import torch

from ..runtime.tracing import trace
from .param import Param, Params, TypeConverters, keyword_only, shared
from .util import (MLReadable, MLWritable, MLWriter, apply_metadata, load_metadata, py_class, register,
                   save_metadata)


def _is_param_map(p) -> bool:
    return isinstance(p, dict)


def _pool_of(dataset):
    """The executor pool holding ``dataset`` when it is a driver-side handle (runtime/executors.py)."""
    from ..runtime.executors import remote_pool_of
    return remote_pool_of(dataset)


def _exec_fit(est, dataset, params):
    return est.fit(dataset, params)


def _exec_transform(tr, dataset, params):
    return tr.transform(dataset, params)


def _exec_evaluate(ev, dataset, params):
    return ev.evaluate(dataset, params)


class Transformer(Params, ABC):
    """Abstract: transforms one DataFrame into another.

    Called with an executor-pool handle (driver process of a multi-GPU session), the
    stage is shipped to the executors and the result stays there as a handle."""

    def transform(self, dataset, params=None):
        if params is None:
            params = {}
        if not _is_param_map(params):
            raise TypeError(f"Params must be a param map but got {type(params)}.")
        pool = _pool_of(dataset)
        if pool is not None:
            return pool.apply(_exec_transform, self, dataset, params)
        with trace(f"{type(self).__name__}.transform"):
            if params:
                return self.copy(params)._transform(dataset)
            return self._transform(dataset)

    @abstractmethod
    def _transform(self, dataset):
        raise NotImplementedError


class Estimator(Params, ABC):
    """Abstract: fits a Model to a DataFrame."""

    def fit(self, dataset, params=None, *, progress=None, cancelled=None):
        """pyspark's ``fit(dataset, params=None)``, plus two optional keywords (SURVEY
        §2.10 Q14): ``progress(percent)`` receives the fit's progress, non-decreasing
        0..100 (per iteration for the linear models, KMeans and ALS, per tree level /
        tree for the tree ensembles), and a ``cancelled()`` that returns True stops the
        fit with ``runtime.progress.FitCancelled`` at the next iteration."""
        from ..runtime import progress as P
        if progress is not None or cancelled is not None:
            with P.progress_scope(progress, cancelled):
                model = self.fit(dataset, params)
                P.report(1.0)
            return model
        if params is None:
            params = {}
        if isinstance(params, (list, tuple)):
            out = []
            for i, p in enumerate(params):
                with P.sub_range(i / len(params), (i + 1) / len(params)):
                    out.append(self.fit(dataset, p))
            return out
        if not _is_param_map(params):
            raise TypeError(f"Params must be either a param map or a list/tuple of param maps, but got {type(params)}.")
        pool = _pool_of(dataset)
        if pool is not None:                  # driver of an executor pool: fit on every executor
            P.report(0.0)
            return pool.apply_watched(_exec_fit, self, dataset, params)
        import time
        from ..parallel.comm import COMM_STATS
        from ..runtime import warmup as W
        fam = getattr(self, "_warm_family", None)
        if fam is not None:                   # first fit of a family in this process (lazy warm-up)
            W.before_fit(fam)
        with W.user_fit(fam):                 # never alongside a background warm-up fit
            c0 = {k: tuple(v) for k, v in COMM_STATS.items()}
            t0 = time.perf_counter()
            with trace(f"{type(self).__name__}.fit"):
                model = self.copy(params)._fit(dataset) if params else self._fit(dataset)
            _attach_fit_stats(model, dataset, time.perf_counter() - t0, c0, COMM_STATS)
        return model

    def fitMultiple(self, dataset, paramMaps):
        for i, pm in enumerate(paramMaps):
            yield i, self.fit(dataset, pm)

    @abstractmethod
    def _fit(self, dataset):
        raise NotImplementedError


def _attach_fit_stats(model, dataset, seconds, c0, c1):
    """``model.fitStats``: this rank's wall time of the fit, its local rows and the
    collectives it issued (calls / bytes per op) -- the per-fit observability summary
    (iterations and loss curves live on ``model.summary`` as in Spark).  Cheap: no
    device sync and no collective of its own."""
    try:
        n_local = int(len(dataset)) if hasattr(dataset, "__len__") else None
    except Exception:  # noqa: BLE001 - a dataset without a cheap local length
        n_local = None
    comm = {}
    for op, (calls, nbytes) in c1.items():
        a, b = c0.get(op, (0, 0))
        if calls - a:
            comm[op] = {"calls": calls - a, "bytes": nbytes - b}
    stats = {"seconds": seconds, "rows_local": n_local,
             "rows_per_s_local": (n_local / seconds) if (n_local and seconds > 0) else None, "collectives": comm}
    try:
        model.fitStats = stats
    except Exception:  # noqa: BLE001 - models that forbid new attributes
        pass


class Model(Transformer, ABC):
    """A fitted Transformer produced by an Estimator."""

    parent = None

    def _with_parent(self, est):
        self.parent = est
        # models inherit the estimator's param values (Spark copyValues)
        est._copyValues(self)
        return self


class Evaluator(Params, ABC):
    def evaluate(self, dataset, params=None):
        if params is None:
            params = {}
        pool = _pool_of(dataset)
        if pool is not None:
            return pool.apply(_exec_evaluate, self, dataset, params)
        with trace(f"{type(self).__name__}.evaluate"):
            if params:
                return self.copy(params)._evaluate(dataset)
            return self._evaluate(dataset)

    @abstractmethod
    def _evaluate(self, dataset):
        raise NotImplementedError

    def isLargerBetter(self) -> bool:
        return True


class UnaryTransformer(Transformer, ABC):
    """Applies a per-column function inputCol -> outputCol."""


# ------------------------------------------------------------------ pipelines
class _PipelineWriter(MLWriter):
    def saveImpl(self, path):
        inst = self.instance
        stages = inst.getStages()
        save_metadata(inst, path, paramMap={"stageUids": [s.uid for s in stages]})
        digits = len(str(len(stages)))
        for i, s in enumerate(stages):
            sp = os.path.join(path, "stages", f"{i:0{digits}d}_{s.uid}")
            s.write().saveImpl(sp) if hasattr(s, "write") else None


def _load_stages(path, meta):
    uids = meta["paramMap"]["stageUids"]
    digits = len(str(len(uids)))
    stages = []
    for i, uid in enumerate(uids):
        sp = os.path.join(path, "stages", f"{i:0{digits}d}_{uid}")
        m = load_metadata(sp)
        cls = py_class(m["class"])
        if hasattr(cls, "_load_impl"):
            stages.append(cls._load_impl(sp, m))
        else:
            inst = cls()
            apply_metadata(inst, m)
            stages.append(inst)
    return stages


@register("org.apache.spark.ml.Pipeline")
class Pipeline(Estimator, MLWritable, MLReadable):
    """A simple pipeline: a sequence of Estimator and Transformer stages."""

    stages = shared("stages", "a list of pipeline stages")

    @keyword_only
    def __init__(self, *, stages=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def setStages(self, value):
        return self._set(stages=value)

    def getStages(self):
        return list(self.getOrDefault(self.stages)) if self.isDefined(self.stages) else []

    @keyword_only
    def setParams(self, *, stages=None):
        return self._set(**self._input_kwargs)

    def _fit(self, dataset):
        stages = self.getStages()
        for s in stages:
            if not isinstance(s, (Estimator, Transformer)):
                raise TypeError(f"Cannot recognize a pipeline stage of type {type(s)}.")
        last_est = max([i for i, s in enumerate(stages) if isinstance(s, Estimator)], default=-1)
        models = []
        df = dataset
        for i, s in enumerate(stages):
            if i <= last_est:
                if isinstance(s, Transformer):
                    models.append(s)
                    df = s.transform(df)
                else:
                    from ..runtime import progress as P
                    with P.sub_range(i / (last_est + 1), (i + 1) / (last_est + 1)):
                        m = s.fit(df)
                    models.append(m)
                    if i < last_est:
                        df = m.transform(df)
            else:
                models.append(s)
        return PipelineModel(models)._with_uid(self.uid)

    def copy(self, extra=None):
        that = super().copy(extra)
        that._set(stages=[s.copy(extra) for s in self.getStages()])
        return that

    def write(self):
        return _PipelineWriter(self)

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import set_uid
        p = Pipeline(stages=_load_stages(path, meta))
        set_uid(p, meta["uid"])
        return p


@register("org.apache.spark.ml.PipelineModel")
class PipelineModel(Model, MLWritable, MLReadable):
    def __init__(self, stages=None):
        super().__init__()
        self.stages = list(stages or [])

    def _with_uid(self, uid):
        from .util import set_uid
        set_uid(self, uid)
        return self

    def _transform(self, dataset):
        df = dataset
        for s in self.stages:
            df = s.transform(df)
        return df

    def copy(self, extra=None):
        return PipelineModel([s.copy(extra) for s in self.stages])._with_uid(self.uid)

    def getStages(self):
        return list(self.stages)

    def write(self):
        w = _PipelineWriter(self)
        return w

    @classmethod
    def _load_impl(cls, path, meta):
        return PipelineModel(_load_stages(path, meta))._with_uid(meta["uid"])


# PipelineModel writer needs getStages + uid like Pipeline
_ = TypeConverters, Param, torch
