"""``pyspark.ml.functions``: conversions between ML vector columns and array columns.

Reached like the rest of the pyspark surface from the PySpark Script widget's scripts
(reference orangecontrib/spark/widgets/data/pyspark_script_console.py:331).  Vectors live
on the device as [n, d] matrices (dense) or CSR (sparse); arrays of doubles live on the
host, so ``vector_to_array`` is one device -> host copy and ``array_to_vector`` one
host -> device copy of the rank's slice.
"""
from __future__ import annotations

import numpy as np
import torch

from ..frame import column as C
from ..frame import types as T
from ..frame.expr import Expr, col

__all__ = ["vector_to_array", "array_to_vector", "predict_batch_udf"]


def _e(x) -> Expr:
    return col(x) if isinstance(x, str) else x


def vector_to_array(c, dtype: str = "float64") -> Expr:
    """Vector column -> array<double> (or array<float> with ``dtype="float32"``)."""
    if dtype not in ("float64", "float32"):
        raise ValueError(f"Unsupported dtype: {dtype}. Valid values: float64, float32.")
    e = _e(c)
    np_dt = np.float64 if dtype == "float64" else np.float32

    def f(df):
        v = e.eval(df)
        if isinstance(v, C.SparseVectorColumn):
            mat = v.to_dense(torch.float64).cpu().numpy()
        elif isinstance(v, C.VectorColumn):
            mat = v.to_numpy()
        else:
            raise TypeError(f"vector_to_array expects a vector column, got {v.dtype.simpleString()}")
        vals = np.empty(len(mat), dtype=object)
        vals[:] = [list(r.astype(np_dt).tolist()) for r in mat]
        return C.ArrayColumn(vals, T.DoubleType() if dtype == "float64" else T.FloatType())
    return Expr(f, f"vector_to_array({e.name})", e.refs)


def array_to_vector(c) -> Expr:
    """array<numeric> column (equal lengths) -> dense vector column on the session device."""
    e = _e(c)

    def f(df):
        v = e.eval(df)
        if isinstance(v, C.VectorColumn):
            return v
        if not isinstance(v, C.ArrayColumn):
            raise TypeError(f"array_to_vector expects an array column, got {v.dtype.simpleString()}")
        rows = [r for r in v.values]
        if any(r is None for r in rows):
            raise ValueError("array_to_vector: null arrays cannot become vectors")
        widths = {len(r) for r in rows}
        if len(widths) > 1:
            raise ValueError("array_to_vector: arrays of different lengths")
        d = widths.pop() if widths else 0
        mat = np.asarray(rows, dtype=np.float64).reshape(len(rows), d)
        return C.VectorColumn(torch.from_numpy(mat).to(df.device))
    return Expr(f, f"array_to_vector({e.name})", e.refs)


def predict_batch_udf(make_predict_fn, *, return_type, batch_size: int, input_tensor_shapes=None):
    """Batched inference UDF: ``make_predict_fn()`` returns ``predict(np.ndarray) -> np.ndarray``
    applied to the column's rows in batches of ``batch_size`` on this rank."""
    def udf(*cols):
        es = [_e(x) for x in cols]

        def f(df):
            predict = make_predict_fn()
            arrs = []
            for e in es:
                v = e.eval(df)
                arrs.append(v.to_numpy() if hasattr(v, "to_numpy") else np.asarray(v.to_pylist()))
            n = len(df)
            outs = []
            for s in range(0, n, batch_size):
                batch = [a[s:s + batch_size] for a in arrs]
                outs.append(np.asarray(predict(*batch)))
            out = np.concatenate(outs) if outs else np.zeros(0)
            return C.from_numpy(out, df.device)
        return Expr(f, "predict_batch_udf(" + ", ".join(e.name for e in es) + ")",
                    tuple(r for e in es for r in e.refs))
    return udf
