"""Shared base of the feature-selector models (ChiSq, VarianceThreshold, Univariate):
keep the ``selectedFeatures`` columns of a vector column."""
from __future__ import annotations

import torch

from ..frame import column as C
from . import common as U
from .base import Model
from .param import HasFeaturesCol, HasOutputCol
from .util import MLReadable, MLWritable, apply_metadata, prim_list, read_data, write_data


def _vec(df, name) -> torch.Tensor:
    return U.dense_features(df, name, torch.float64)


class _SelectorModel(Model, HasFeaturesCol, HasOutputCol, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self.selectedFeatures = []

    def _transform(self, df):
        X = _vec(df, self.getOrDefault(self.featuresCol))
        idx = torch.tensor(self.selectedFeatures, dtype=torch.int64, device=X.device)
        return df.withColumnData(self.getOrDefault(self.outputCol), C.VectorColumn(X[:, idx]))

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"selectedFeatures": pa.array([self.selectedFeatures], prim_list(pa.int32()))})

    @classmethod
    def _load_impl(cls, path, meta):
        m = cls()
        m.selectedFeatures = read_data(path).to_pylist()[0]["selectedFeatures"]
        apply_metadata(m, meta)
        return m
