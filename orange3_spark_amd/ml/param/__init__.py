"""Param system with the ``pyspark.ml.param`` contract the reflective widgets rely on.

Contract (reference orangecontrib/spark/utils/ml_api_utils.py:20-44 and
base/spark_ml_transformer.py:117-123):

* ``inspect.signature(cls)`` lists every settable Param as a keyword argument with its
  default (constructors are keyword-only and decorated with :func:`keyword_only`);
* ``cls()`` works with no session and no device (introspection never boots anything:
  fixes reference quirk Q9);
* Param identity is ``(parent uid, name)``: the widget builds
  ``{Param(instance, name, ''): value}`` maps and passes them to ``fit``/``transform``;
* docs keep Spark's wording, including the ``"(a|b|c)"`` metric lists the Evaluation
  widget parses (widgets/ml/spark_ml_evaluation.py:43);
* a ``None`` value in a param map means "unset -> default" (fixes quirk Q10).
"""
from __future__ import annotations

import copy
import functools
import inspect
import itertools
import uuid
from typing import Any, Callable


class TypeConverters:
    @staticmethod
    def identity(v):
        return v

    @staticmethod
    def toInt(v):
        if isinstance(v, bool):
            raise TypeError(f"Could not convert {v!r} to int")
        if isinstance(v, (int,)) or (hasattr(v, "is_integer") and float(v).is_integer()):
            return int(v)
        if isinstance(v, str) and v.strip().lstrip("-").isdigit():
            return int(v)
        raise TypeError(f"Could not convert {v!r} to int")

    @staticmethod
    def toFloat(v):
        if isinstance(v, bool):
            raise TypeError(f"Could not convert {v!r} to float")
        try:
            return float(v)
        except (TypeError, ValueError):
            raise TypeError(f"Could not convert {v!r} to float")

    @staticmethod
    def toBoolean(v):
        if isinstance(v, bool):
            return v
        if isinstance(v, str) and v.lower() in ("true", "false"):
            return v.lower() == "true"
        if isinstance(v, (int, float)) and v in (0, 1):
            return bool(v)
        raise TypeError(f"Boolean Param requires value of type bool. Found {type(v)}.")

    @staticmethod
    def toString(v):
        if isinstance(v, str):
            return v
        raise TypeError(f"Could not convert {v!r} to string")

    @staticmethod
    def _split(v):
        if isinstance(v, str):
            s = v.strip()
            if s.startswith("[") and s.endswith("]"):
                s = s[1:-1]
            return [p.strip().strip("'\"") for p in s.split(",") if p.strip()]
        return list(v)

    @staticmethod
    def toListString(v):
        return [str(x) for x in TypeConverters._split(v)]

    @staticmethod
    def toListFloat(v):
        return [float(x) for x in TypeConverters._split(v)]

    @staticmethod
    def toListInt(v):
        return [int(float(x)) for x in TypeConverters._split(v)]

    @staticmethod
    def toListListFloat(v):
        return [TypeConverters.toListFloat(x) for x in v]

    @staticmethod
    def toVector(v):
        from ..linalg import DenseVector, Vector
        if isinstance(v, Vector):
            return v
        return DenseVector(TypeConverters.toListFloat(v))

    @staticmethod
    def toMatrix(v):
        return v


class Param:
    """A named parameter owned by a Params instance (identity = (parent uid, name))."""

    def __init__(self, parent, name: str, doc: str, typeConverter: Callable | None = None):
        if isinstance(parent, Params):
            parent = parent.uid
        self.parent = parent
        self.name = str(name)
        self.doc = str(doc)
        self.typeConverter = typeConverter or TypeConverters.identity

    def _copy_new_parent(self, parent: "Params") -> "Param":
        p = copy.copy(self)
        p.parent = parent.uid
        return p

    def __str__(self):
        return f"{self.parent}__{self.name}"

    def __repr__(self):
        return f"Param(parent={self.parent!r}, name={self.name!r}, doc={self.doc!r})"

    def __hash__(self):
        return hash(str(self))

    def __eq__(self, other):
        return isinstance(other, Param) and self.parent == other.parent and self.name == other.name


class Params:
    """Base of every Estimator/Transformer/Evaluator/Model."""

    _counters = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        add_accessors(cls)   # getX/setX for every Param, like pyspark's generated accessors

    def __init__(self):
        self._paramMap: dict[Param, Any] = {}
        self._defaultParamMap: dict[Param, Any] = {}
        self.uid = self._randomUID()
        self._params = None
        self._copy_params()

    @classmethod
    def _randomUID(cls) -> str:
        return f"{cls.__name__}_{uuid.uuid4().hex[:12]}"

    def _copy_params(self):
        """Bind class-level Param templates to this instance (new parent = uid)."""
        for name in dir(type(self)):
            attr = getattr(type(self), name, None)
            if isinstance(attr, Param):
                setattr(self, name, attr._copy_new_parent(self))

    @property
    def params(self) -> list[Param]:
        if self._params is None:
            self._params = sorted(
                [getattr(self, n) for n in dir(self)
                 if not n.startswith("__") and n != "params" and isinstance(getattr(type(self), n, None), Param)],
                key=lambda p: p.name)
        return self._params

    # -- introspection ---------------------------------------------------------
    def explainParam(self, param) -> str:
        param = self._resolveParam(param)
        values = []
        if self.isDefined(param):
            if param in self._defaultParamMap:
                values.append(f"default: {self._defaultParamMap[param]}")
            if param in self._paramMap:
                values.append(f"current: {self._paramMap[param]}")
        else:
            values.append("undefined")
        return f"{param.name}: {param.doc} ({', '.join(values)})"

    def explainParams(self) -> str:
        return "\n".join(self.explainParam(p) for p in self.params)

    def getParam(self, paramName: str) -> Param:
        p = getattr(self, paramName, None)
        if isinstance(p, Param):
            return p
        raise ValueError(f"Cannot find param with name {paramName}.")

    def hasParam(self, paramName: str) -> bool:
        return isinstance(getattr(self, str(paramName), None), Param)

    def isSet(self, param) -> bool:
        return self._resolveParam(param) in self._paramMap

    def hasDefault(self, param) -> bool:
        return self._resolveParam(param) in self._defaultParamMap

    def isDefined(self, param) -> bool:
        return self.isSet(param) or self.hasDefault(param)

    def getOrDefault(self, param):
        param = self._resolveParam(param)
        if param in self._paramMap:
            return self._paramMap[param]
        if param in self._defaultParamMap:
            return self._defaultParamMap[param]
        raise KeyError(f"Param {param.name} is not set and has no default")

    def extractParamMap(self, extra: dict | None = None) -> dict:
        m = dict(self._defaultParamMap)
        m.update(self._paramMap)
        if extra:
            m.update(extra)
        return m

    def _resolveParam(self, param) -> Param:
        if isinstance(param, Param):
            if param.parent != self.uid:
                p = getattr(self, param.name, None)
                if isinstance(p, Param):
                    return p
                raise ValueError(f"Param {param} does not belong to {self}.")
            return param
        if isinstance(param, str):
            return self.getParam(param)
        raise TypeError(f"Cannot resolve {param!r} as a param.")

    # -- setters ---------------------------------------------------------------
    def set(self, param, value):
        self._set(**{self._resolveParam(param).name: value})

    def _set(self, **kwargs):
        for name, value in kwargs.items():
            p = self.getParam(name)
            if value is None:
                # "unset -> default" (reference passes None for blank GUI fields)
                self._paramMap.pop(p, None)
                continue
            try:
                value = p.typeConverter(value)
            except TypeError as e:
                raise TypeError(f'Invalid param value given for param "{name}". {e}')
            self._paramMap[p] = value
        return self

    def _setDefault(self, **kwargs):
        for name, value in kwargs.items():
            p = self.getParam(name)
            if value is not None and p.typeConverter is not TypeConverters.identity:
                try:
                    value = p.typeConverter(value)
                except TypeError:
                    pass
            self._defaultParamMap[p] = value
        return self

    def clear(self, param):
        self._paramMap.pop(self._resolveParam(param), None)

    # -- copying ---------------------------------------------------------------
    def copy(self, extra: dict | None = None):
        that = copy.copy(self)
        that._paramMap = {}
        that._defaultParamMap = {}
        that._params = None
        return self._copyValues(that, extra)

    def _copyValues(self, to: "Params", extra: dict | None = None):
        paramMap = dict(self._paramMap)
        if extra:
            for k, v in extra.items():
                name = k.name if isinstance(k, Param) else str(k)
                if self.hasParam(name):
                    paramMap[self.getParam(name)] = v
        for p in self.params:
            if p in self._defaultParamMap and to.hasParam(p.name):
                to._defaultParamMap[to.getParam(p.name)] = self._defaultParamMap[p]
            if p in paramMap and to.hasParam(p.name):
                v = paramMap[p]
                if v is None:
                    continue
                to._set(**{p.name: v})
        return to

    def _shouldOwn(self, param):
        if not (self.uid == param.parent and self.hasParam(param.name)):
            raise ValueError(f"Param {param} does not belong to {self}.")

    def __repr__(self):
        return self.uid


def keyword_only(func):
    """Record keyword arguments in ``self._input_kwargs`` (pyspark idiom)."""
    @functools.wraps(func)
    def wrapper(self, *args, **kwargs):
        if args:
            raise TypeError(f"Method {func.__name__} forces keyword arguments.")
        self._input_kwargs = kwargs
        return func(self, **kwargs)
    return wrapper


def shared(name: str, doc: str, conv=None) -> Param:
    """Class-level Param template (bound per instance by Params._copy_params)."""
    return Param("undefined", name, doc, conv)


# ------------------------------------------------------------- shared param mixins
def _getter(pname):
    def g(self):
        return self.getOrDefault(getattr(self, pname))
    g.__name__ = "get" + pname[0].upper() + pname[1:]
    return g


def _setter(pname):
    def s(self, value):
        self._set(**{pname: value})
        return self
    s.__name__ = "set" + pname[0].upper() + pname[1:]
    return s


def add_accessors(cls):
    """Generate getX/setX for every Param declared on ``cls`` (if missing)."""
    for n in list(dir(cls)):
        if isinstance(getattr(cls, n, None), Param):
            cap = n[0].upper() + n[1:]
            if not hasattr(cls, "get" + cap):
                setattr(cls, "get" + cap, _getter(n))
            if not hasattr(cls, "set" + cap):
                setattr(cls, "set" + cap, _setter(n))
    return cls


_SHARED = {
    "featuresCol": ("features column name.", TypeConverters.toString, "features"),
    "labelCol": ("label column name.", TypeConverters.toString, "label"),
    "predictionCol": ("prediction column name.", TypeConverters.toString, "prediction"),
    "probabilityCol": ("Column name for predicted class conditional probabilities. Note: Not all models output "
                       "well-calibrated probability estimates! These probabilities should be treated as confidences, "
                       "not precise probabilities.", TypeConverters.toString, "probability"),
    "rawPredictionCol": ("raw prediction (a.k.a. confidence) column name.", TypeConverters.toString, "rawPrediction"),
    "weightCol": ("weight column name. If this is not set or empty, we treat all instance weights as 1.0.",
                  TypeConverters.toString, None),
    "inputCol": ("input column name.", TypeConverters.toString, None),
    "inputCols": ("input column names.", TypeConverters.toListString, None),
    "outputCol": ("output column name.", TypeConverters.toString, None),
    "outputCols": ("output column names.", TypeConverters.toListString, None),
    "maxIter": ("max number of iterations (>= 0).", TypeConverters.toInt, None),
    "regParam": ("regularization parameter (>= 0).", TypeConverters.toFloat, None),
    "elasticNetParam": ("the ElasticNet mixing parameter, in range [0, 1]. For alpha = 0, the penalty is an L2 "
                        "penalty. For alpha = 1, it is an L1 penalty.", TypeConverters.toFloat, None),
    "tol": ("the convergence tolerance for iterative algorithms (>= 0).", TypeConverters.toFloat, None),
    "fitIntercept": ("whether to fit an intercept term.", TypeConverters.toBoolean, None),
    "standardization": ("whether to standardize the training features before fitting the model.",
                        TypeConverters.toBoolean, None),
    "threshold": ("threshold in binary classification prediction, in range [0, 1].", TypeConverters.toFloat, None),
    "thresholds": ("Thresholds in multi-class classification to adjust the probability of predicting each class. "
                   "Array must have length equal to the number of classes, with values > 0, excepting that at most "
                   "one value may be 0. The class with largest value p/t is predicted, where p is the original "
                   "probability of that class and t is the class's threshold.", TypeConverters.toListFloat, None),
    "seed": ("random seed.", TypeConverters.toInt, None),
    "stepSize": ("Step size to be used for each iteration of optimization (>= 0).", TypeConverters.toFloat, None),
    "aggregationDepth": ("suggested depth for treeAggregate (>= 2).", TypeConverters.toInt, 2),
    "checkpointInterval": ("set checkpoint interval (>= 1) or disable checkpoint (-1). E.g. 10 means that the cache "
                           "will get checkpointed every 10 iterations. Note: this setting will be ignored if the "
                           "checkpoint directory is not set in the SparkContext.", TypeConverters.toInt, None),
    "handleInvalid": ("how to handle invalid entries. Options are 'skip' (which will filter out rows with bad "
                      "values), or 'error' (which will throw an error), or 'keep'.", TypeConverters.toString, None),
    "numFeatures": ("Number of features. Should be greater than 0.", TypeConverters.toInt, None),
    "k": ("the number of clusters to create. Must be > 1.", TypeConverters.toInt, None),
    "solver": ("The solver algorithm for optimization.", TypeConverters.toString, None),
    "varianceCol": ("column name for the biased sample variance of prediction.", TypeConverters.toString, None),
    "distanceMeasure": ("the distance measure. Supported options: 'euclidean' and 'cosine'.",
                        TypeConverters.toString, "euclidean"),
    "blockSize": ("block size for stacking input data in matrices. Data is stacked within partitions. If block size "
                  "is more than remaining data in a partition then it is adjusted to the size of this data.",
                  TypeConverters.toInt, None),
    "maxBlockSizeInMB": ("maximum memory in MB for stacking input data into blocks. Data is stacked within "
                         "partitions. If more than remaining data size in a partition then it is adjusted to the "
                         "data size. Default 0.0 represents choosing optimal value, depends on specific algorithm. "
                         "Must be >= 0.", TypeConverters.toFloat, 0.0),
}


def _mixin(pname):
    doc, conv, default = _SHARED[pname]
    cap = pname[0].upper() + pname[1:]

    def __init__(self):
        super(cls, self).__init__()
        if default is not None:
            self._setDefault(**{pname: default})

    cls = type("Has" + cap, (Params,), {pname: shared(pname, doc, conv), "__init__": __init__,
                                        "get" + cap: _getter(pname)})
    return cls


HasFeaturesCol = _mixin("featuresCol")
HasLabelCol = _mixin("labelCol")
HasPredictionCol = _mixin("predictionCol")
HasProbabilityCol = _mixin("probabilityCol")
HasRawPredictionCol = _mixin("rawPredictionCol")
HasWeightCol = _mixin("weightCol")
HasInputCol = _mixin("inputCol")
HasInputCols = _mixin("inputCols")
HasOutputCol = _mixin("outputCol")
HasOutputCols = _mixin("outputCols")
HasMaxIter = _mixin("maxIter")
HasRegParam = _mixin("regParam")
HasElasticNetParam = _mixin("elasticNetParam")
HasTol = _mixin("tol")
HasFitIntercept = _mixin("fitIntercept")
HasStandardization = _mixin("standardization")
HasThreshold = _mixin("threshold")
HasThresholds = _mixin("thresholds")
HasSeed = _mixin("seed")
HasStepSize = _mixin("stepSize")
HasAggregationDepth = _mixin("aggregationDepth")
HasCheckpointInterval = _mixin("checkpointInterval")
HasHandleInvalid = _mixin("handleInvalid")
HasNumFeatures = _mixin("numFeatures")
HasSolver = _mixin("solver")
HasVarianceCol = _mixin("varianceCol")
HasDistanceMeasure = _mixin("distanceMeasure")
HasBlockSize = _mixin("blockSize")
HasMaxBlockSizeInMB = _mixin("maxBlockSizeInMB")


class ParamGridBuilder:
    """Builder for a param grid used in grid search-based model selection."""

    def __init__(self):
        self._param_grid: dict[Param, list] = {}

    def addGrid(self, param: Param, values):
        self._param_grid[param] = list(values)
        return self

    def baseOn(self, *args):
        if len(args) == 1 and isinstance(args[0], dict):
            args = tuple(args[0].items())
        for p, v in args:
            self.addGrid(p, [v])
        return self

    def build(self) -> list[dict]:
        keys = list(self._param_grid.keys())
        grids = [self._param_grid[k] for k in keys]
        return [dict(zip(keys, combo)) for combo in itertools.product(*grids)]


__all__ = ["Param", "Params", "TypeConverters", "keyword_only", "shared", "add_accessors", "ParamGridBuilder"] + \
    [n for n in list(globals()) if n.startswith("Has")]
_ = inspect
