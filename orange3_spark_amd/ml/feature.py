"""Feature transformers and estimators (``pyspark.ml.feature`` surface).

The reference's Feature widget exposes this module's Transformers
(orangecontrib/spark/widgets/ml/spark_ml_feature.py:15); the Dataset Builder runs
``VectorAssembler(inputCols=features, outputCol='features')``
(widgets/ml/spark_ml_dataset.py:575-576).
"""
from __future__ import annotations

import numpy as np
import torch

from ..frame import column as C
from ..ops import glm as G
from .base import Estimator, Model, Transformer
from .param import (HasHandleInvalid, HasInputCol, HasInputCols, HasOutputCol, HasOutputCols, TypeConverters,
                    add_accessors, keyword_only, shared)
from .util import MLReadable, MLWritable, register


def to_vector_column(session, mat: torch.Tensor, size: int | None = None) -> C.VectorColumn:
    """Store a dense [n, d] matrix in the session's feature dtype (bf16 padded on GPU)."""
    dt = session.vector_dtype()
    n, d = mat.shape
    if dt == torch.bfloat16:
        ld = G.padded_width(d)
        out = torch.zeros((n, ld), dtype=torch.bfloat16, device=mat.device)
        out[:, :d] = mat
        return C.VectorColumn(out, d if size is None else size)
    return C.VectorColumn(mat.to(dt).contiguous(), d if size is None else size)


def _as_matrix(col: C.Column, n: int, device) -> torch.Tensor:
    if isinstance(col, C.NumericColumn):
        v = col.data.to(device, torch.float64)
        if col.valid is not None:
            v = torch.where(col.valid.to(device), v, torch.full_like(v, float("nan")))
        return v[:, None]
    if isinstance(col, C.SparseVectorColumn):
        return col.to_dense(torch.float64).to(device)
    if isinstance(col, C.VectorColumn):
        return col.dense().to(device, torch.float64)
    raise TypeError(f"Data type {col.dtype.simpleString()} of column is not supported.")


@add_accessors
@register("org.apache.spark.ml.feature.VectorAssembler")
class VectorAssembler(Transformer, HasInputCols, HasOutputCol, HasHandleInvalid, MLWritable, MLReadable):
    """A feature transformer that merges multiple columns into a vector column."""

    @keyword_only
    def __init__(self, *, inputCols=None, outputCol=None, handleInvalid="error"):
        super().__init__()
        self._setDefault(handleInvalid="error", outputCol=self.uid + "__output")
        self._set(**self._input_kwargs)

    @keyword_only
    def setParams(self, *, inputCols=None, outputCol=None, handleInvalid="error"):
        return self._set(**self._input_kwargs)

    def _transform(self, df):
        cols = self.getOrDefault(self.inputCols)
        n = len(df)
        dev = df.device
        mats = [_as_matrix(df.column_data(c), n, dev) for c in cols]
        mat = torch.cat(mats, dim=1) if mats else torch.zeros((n, 0), dtype=torch.float64, device=dev)
        hi = self.getOrDefault(self.handleInvalid)
        bad = torch.isnan(mat).any(1) if mat.numel() else torch.zeros(n, dtype=torch.bool, device=dev)
        if bool(bad.any()):
            if hi == "error":
                raise ValueError("Encountered null while assembling a row with handleInvalid = \"error\". "
                                 "Consider removing nulls from dataset or using handleInvalid = \"keep\" or \"skip\".")
            if hi == "skip":
                df = df._mask(~bad)
                mat = mat[~bad]
        return df.withColumnData(self.getOrDefault(self.outputCol), to_vector_column(df.session, mat))


__all__ = ["VectorAssembler", "to_vector_column"]
_ = (np, Estimator, Model, HasInputCol, HasOutputCols, TypeConverters, shared)
