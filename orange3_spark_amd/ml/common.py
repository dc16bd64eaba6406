"""Helpers shared by the ML stages: column access and prediction-model plumbing."""
from __future__ import annotations

import numpy as np
import torch

from ..frame import column as C
from ..synthetic import LineageVectorColumn
from .base import Model
from .linalg import DenseVector
from .param import Param, TypeConverters, shared


def features_column(df, name: str) -> C.Column:
    c = df.column_data(name)
    if not isinstance(c, (C.VectorColumn, C.SparseVectorColumn)):
        raise TypeError(f"Column {name} must be of type vector but was actually {c.dtype.simpleString()}.")
    return c


def dense_features(df, name: str, dtype=None) -> torch.Tensor:
    """[n, d] dense tensor of a vector column (lineage rows materialised)."""
    c = features_column(df, name)
    if isinstance(c, C.SparseVectorColumn):
        t = c.to_dense(dtype or torch.float32)
    elif isinstance(c, LineageVectorColumn):
        t = c.full()[:, : c.size]
    else:
        t = c.dense()
    return t if dtype is None else t.to(dtype)


def linear_features(df, name: str):
    """Operand of a linear model's margin: CSR rows (ops.sparse.SparseRows, never
    densified) for sparse vector columns, else the dense tensor."""
    c = features_column(df, name)
    if isinstance(c, C.SparseVectorColumn):
        from ..ops.sparse import SparseRows
        return SparseRows(c.indptr, c.indices, c.values, c.size)
    return dense_features(df, name)


def linear_margin(X, w: np.ndarray, b: float) -> torch.Tensor:
    """fp64 margins X.w + b for a dense tensor or SparseRows operand."""
    from ..ops.sparse import SparseRows
    if isinstance(X, SparseRows):
        wt = torch.from_numpy(np.asarray(w, dtype=np.float64))
        return X.margins(wt, float(b)).to(torch.float64) if X.kernel else X._margins_f64(wt, float(b))
    wt = torch.from_numpy(np.asarray(w, dtype=np.float64)).to(X.device)
    return X.to(torch.float64)[:, : wt.shape[0]] @ wt + float(b)


def numeric_column(df, name: str, dtype=torch.float64) -> torch.Tensor:
    """The column's values as a tensor of ``dtype`` (None: floating columns keep their
    storage dtype -- no full-length copy of a 1B-row label column)."""
    c = df.column_data(name)
    if isinstance(c, C.NumericColumn):
        d = c.data
        if d.device != df.device:            # a host-resident column of an out-of-core table
            d = d.to(df.device, non_blocking=d.is_pinned())
        if c.valid is not None and not bool(c.valid.all()):
            raise ValueError(f"column {name} contains null values")
        if dtype is None:
            return d if d.is_floating_point() else d.to(torch.float64)
        return d.to(dtype)
    if isinstance(c, C.StringColumn):
        return c.cast("double").data.to(dtype or torch.float64)
    raise TypeError(f"Column {name} must be numeric but was {c.dtype.simpleString()}.")


def weights_or_none(df, est) -> torch.Tensor | None:
    if est.hasParam("weightCol") and est.isDefined(est.weightCol):
        wc = est.getOrDefault(est.weightCol)
        if wc:
            return numeric_column(df, wc)
    return None


def num_classes(comm, y: torch.Tensor) -> int:
    mx = float(y.max().item()) if y.numel() else 0.0
    mx = comm.max_scalar(mx)
    return int(mx) + 1


def vec_out(t: torch.Tensor) -> C.VectorColumn:
    return C.VectorColumn(t.to(torch.float64))


def num_out(t: torch.Tensor) -> C.NumericColumn:
    return C.NumericColumn(t.to(torch.float64))


class PredictionModelMixin:
    """featuresCol -> predictionCol for regression-style models."""

    def _predict_tensor(self, X: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def _features_for_predict(self, df, name):
        return dense_features(df, name)

    def _transform(self, df):
        X = self._features_for_predict(df, self.getOrDefault(self.featuresCol))
        pred = self._predict_tensor(X)
        pc = self.getOrDefault(self.predictionCol)
        return df.withColumnData(pc, num_out(pred)) if pc else df

    def predict(self, value):
        x = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value), dtype=torch.float64)
        return float(self._predict_tensor(x[None, :])[0])


class ProbabilisticClassifierMixin:
    """rawPrediction -> probability -> prediction (Spark ProbabilisticClassificationModel)."""

    def _raw(self, X: torch.Tensor) -> torch.Tensor:            # [n, C]
        raise NotImplementedError

    def _raw2prob(self, raw: torch.Tensor) -> torch.Tensor:
        return torch.softmax(raw, dim=1)

    def _prob2pred(self, prob: torch.Tensor) -> torch.Tensor:
        if self.hasParam("thresholds") and self.isSet(self.thresholds):
            t = torch.tensor(self.getOrDefault(self.thresholds), dtype=prob.dtype, device=prob.device)
            scaled = torch.where(t > 0, prob / torch.where(t > 0, t, torch.ones_like(t)),
                                 torch.full_like(prob, float("inf")))
            return scaled.argmax(1).to(torch.float64)
        if prob.shape[1] == 2 and self.hasParam("threshold") and self.isDefined(self.threshold):
            return (prob[:, 1] > self.getOrDefault(self.threshold)).to(torch.float64)
        return prob.argmax(1).to(torch.float64)

    def _transform(self, df):
        feat = self.getOrDefault(self.featuresCol)
        X = self._features_for_predict(df, feat)
        raw = self._raw(X)
        out = df
        rc = self.getOrDefault(self.rawPredictionCol) if self.hasParam("rawPredictionCol") else ""
        pc = self.getOrDefault(self.probabilityCol) if self.hasParam("probabilityCol") else ""
        yc = self.getOrDefault(self.predictionCol)
        prob = None
        if rc:
            out = out.withColumnData(rc, vec_out(raw))
        if pc or yc:
            prob = self._raw2prob(raw)
        if pc:
            out = out.withColumnData(pc, vec_out(prob))
        if yc:
            out = out.withColumnData(yc, num_out(self._prob2pred(prob)))
        return out

    def _features_for_predict(self, df, name):
        return dense_features(df, name)

    def predictRaw(self, value):
        x = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value), dtype=torch.float64)
        return DenseVector(self._raw(x[None, :])[0].cpu().numpy())

    def predictProbability(self, value):
        x = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value), dtype=torch.float64)
        return DenseVector(self._raw2prob(self._raw(x[None, :]))[0].cpu().numpy())

    def predict(self, value):
        x = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value), dtype=torch.float64)
        return float(self._prob2pred(self._raw2prob(self._raw(x[None, :])))[0])


_ = (Model, Param, TypeConverters, shared)
