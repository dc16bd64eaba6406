"""MultilayerPerceptronClassifier (``pyspark.ml.classification``).

Reached through the Classification widget's reflection.  Network: affine
layers with sigmoid activations and a softmax output, cross-entropy loss averaged over
the (weighted) rows, trained with L-BFGS (default) or gradient descent.

MI355X mapping: every optimiser evaluation runs forward + backward over the rank's rows
as chunked fp32 GEMMs (hipBLASLt) and all-reduces ONE flat gradient vector
(models/dist_opt.py) -- data parallelism over row shards, like Spark's treeAggregate.
The flat weight layout is Spark's (per layer: the [in, out] weight block stored
column-major as an out x in matrix, then the bias), so saved ``weights`` interoperate.
"""
from __future__ import annotations

import numpy as np
import torch

from ..models import dist_opt
from . import common as U
from .base import Estimator, Model
from .linalg import DenseVector
from .param import (HasBlockSize, HasFeaturesCol, HasLabelCol, HasMaxIter, HasPredictionCol, HasProbabilityCol,
                    HasRawPredictionCol, HasSeed, HasSolver, HasStepSize, HasThresholds, HasTol, TypeConverters,
                    keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, read_data, register, vec_col, write_data


class _MLPParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasProbabilityCol, HasRawPredictionCol,
                 HasMaxIter, HasTol, HasSeed, HasStepSize, HasSolver, HasBlockSize, HasThresholds):
    layers = shared("layers", "Sizes of layers from input layer to output layer E.g., Array(780, 100, 10) means "
                              "780 inputs, one hidden layer with 100 neurons and output layer of 10 neurons.",
                    TypeConverters.toListInt)
    initialWeights = shared("initialWeights", "The initial weights of the model.", TypeConverters.toVector)

    def __init__(self):
        super().__init__()
        self._setDefault(maxIter=100, tol=1e-6, blockSize=128, stepSize=0.03, solver="l-bfgs", seed=0)


def layer_slices(layers):
    """[(w_offset, b_offset, n_in, n_out)] of the flat Spark weight vector."""
    out, off = [], 0
    for i, o in zip(layers[:-1], layers[1:]):
        out.append((off, off + i * o, i, o))
        off += i * o + o
    return out, off


def forward(theta: torch.Tensor, X: torch.Tensor, layers) -> torch.Tensor:
    """Logits of the output layer (pre-softmax), theta in Spark's flat layout."""
    h = X
    sl, _ = layer_slices(layers)
    for li, (wo, bo, i, o) in enumerate(sl):
        W = theta[wo:wo + i * o].reshape(i, o)       # out x in column-major == [in, out] row-major
        h = h @ W + theta[bo:bo + o]
        if li < len(sl) - 1:
            h = torch.sigmoid(h)
    return h


def init_weights(layers, seed: int) -> np.ndarray:
    """Uniform(-r, r), r = sqrt(6 / (in + out)) per layer, zero biases (Glorot)."""
    sl, total = layer_slices(layers)
    rng = np.random.default_rng(seed)
    x = np.zeros(total)
    for wo, bo, i, o in sl:
        r = np.sqrt(6.0 / (i + o))
        x[wo:wo + i * o] = rng.uniform(-r, r, i * o)
    return x


@register("org.apache.spark.ml.classification.MultilayerPerceptronClassifier")
class MultilayerPerceptronClassifier(Estimator, _MLPParams, MLWritable, MLReadable):
    """Classifier trainer based on the Multilayer Perceptron. Each layer has sigmoid
    activation function, output layer has softmax. Number of inputs has to be equal to the
    size of feature vectors. Number of outputs has to be equal to the total number of labels.
    """

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxIter=100,
                 tol=1e-6, seed=None, layers=None, blockSize=128, stepSize=0.03, solver="l-bfgs",
                 initialWeights=None, probabilityCol="probability", rawPredictionCol="rawPrediction"):
        super().__init__()
        self._set(**self._input_kwargs)

    @keyword_only
    def setParams(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxIter=100,
                  tol=1e-6, seed=None, layers=None, blockSize=128, stepSize=0.03, solver="l-bfgs",
                  initialWeights=None, probabilityCol="probability", rawPredictionCol="rawPrediction"):
        return self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        comm = df.comm
        X = U.dense_features(df, g(self.featuresCol))
        y = U.numeric_column(df, g(self.labelCol))
        if not self.isDefined(self.layers) or not g(self.layers):
            raise ValueError("MultilayerPerceptronClassifier requires the layers param")
        layers = [int(v) for v in g(self.layers)]
        if X.shape[1] != layers[0] and X.shape[0]:
            raise ValueError(f"Dimensions mismatch: features {X.shape[1]} vs input layer {layers[0]}")
        K = layers[-1]
        dev = X.device
        dt = dist_opt.compute_dtype(dev)
        yl = y.to(dev).long()
        if yl.numel() and int(comm.max_scalar(float(yl.max()))) >= K:
            raise ValueError(f"labels must be in [0, {K}) for an output layer of size {K}")
        n = X.shape[0]
        W = float(comm.sum_scalar(n))

        def local_loss(theta, a, b):
            logits = forward(theta, X[a:b].to(dt), layers)
            return torch.nn.functional.cross_entropy(logits, yl[a:b], reduction="sum")

        obj = dist_opt.Objective(comm, dev, n, local_loss, W, chunk=1 << 18)
        if self.isDefined(self.initialWeights) and g(self.initialWeights) is not None:
            x0 = np.asarray(g(self.initialWeights).toArray(), dtype=np.float64)
        else:
            x0 = init_weights(layers, int(g(self.seed)) & 0xFFFFFFFF)
        if g(self.solver) == "gd":
            res = dist_opt.gradient_descent(obj, x0, g(self.maxIter), g(self.stepSize), g(self.tol))
        else:
            res = dist_opt.lbfgs(obj, x0, g(self.maxIter), g(self.tol))
        m = MultilayerPerceptronClassificationModel._from(layers, res.x)
        m.summary = _TrainingSummary(res.history, res.iterations)
        return m._with_parent(self)


class _TrainingSummary:
    def __init__(self, history, iterations):
        self.objectiveHistory = list(history)
        self.totalIterations = int(iterations)


@register("org.apache.spark.ml.classification.MultilayerPerceptronClassificationModel")
class MultilayerPerceptronClassificationModel(U.ProbabilisticClassifierMixin, Model, _MLPParams, MLWritable,
                                              MLReadable):
    """Model fitted by MultilayerPerceptronClassifier."""

    def evaluate(self, df):
        """Multiclass metrics of this model's predictions on ``df`` (Spark >= 3.1)."""
        from . import _summary as S
        g = self.getOrDefault
        return S.ClassificationSummary(lambda: self.transform(df), labelCol=g(self.labelCol),
                                       predictionCol=g(self.predictionCol))

    def __init__(self):
        super().__init__()
        self._layers = []
        self._w = np.zeros(0)
        self.summary = None

    @classmethod
    def _from(cls, layers, weights):
        m = cls()
        m._layers = [int(v) for v in layers]
        m._w = np.asarray(weights, dtype=np.float64)
        m._set(layers=m._layers)
        return m

    @property
    def weights(self) -> DenseVector:
        return DenseVector(self._w)

    @property
    def numFeatures(self) -> int:
        return self._layers[0]

    @property
    def numClasses(self) -> int:
        return self._layers[-1]

    def _raw(self, X):
        dt = dist_opt.compute_dtype(X.device)
        theta = torch.from_numpy(self._w).to(X.device, dt)
        return forward(theta, X.to(dt)[:, : self.numFeatures], self._layers).to(torch.float64)

    def _save_data(self, path):
        write_data(path, {"weights": vec_col([self.weights])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        t = read_data(path).to_pylist()[0]
        layers = meta.get("paramMap", {}).get("layers")
        m = cls._from(layers, vector_from_struct(t["weights"]).toArray())
        apply_metadata(m, meta)
        return m
