"""TargetEncoder / TargetEncoderModel (``pyspark.ml.feature``, Spark >= 4.0).

Reached like every feature estimator through the Feature Estimator widget (SURVEY §2.5
note, §2.7).  Encodes each categorical index column by the label statistics of its
category, blended with the global statistic:

    enc(c) = w * mean_c + (1 - w) * mean_global,   w = n_c / (n_c + smoothing)

(binary target: mean = fraction of positive labels; continuous: mean label), the formula
of Spark's ``TargetEncoder`` *(external: mllib TargetEncoder.scala)*.  Null feature values
form their own category (Spark's NULL_CATEGORY = -1); categories not seen in fit map to
the global statistic under ``handleInvalid='keep'`` and raise under ``'error'``.

The fit is one pass per column on the device: per-category counts and label sums by
``bincount`` (fp64) and ONE all-reduce of both arrays across ranks; the transform is a
gather from the encoding table.  Bit parity with Spark's incremental mean is unpinned
(same value up to fp64 rounding).
"""
from __future__ import annotations

import torch

from ..frame import column as C
from .base import Estimator, Model
from .param import (HasHandleInvalid, HasInputCol, HasInputCols, HasLabelCol, HasOutputCol, HasOutputCols,
                    TypeConverters, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, read_data, register, write_data

NULL_CATEGORY = -1
UNSEEN_CATEGORY = 2147483647


class _TargetEncoderParams(HasLabelCol, HasInputCol, HasInputCols, HasOutputCol, HasOutputCols, HasHandleInvalid):
    targetType = shared("targetType", "Type of label considered during fit(). Options are 'binary' and "
                                      "'continuous'. When 'binary', estimates are calculated as conditional "
                                      "probability of the target given each category. When 'continuous', estimates "
                                      "are calculated as the average of the target given each category. "
                                      "(binary|continuous)", TypeConverters.toString)
    smoothing = shared("smoothing", "Smoothing factor for encodings. Smoothing blends in-class estimates with overall "
                                    "estimates according to the relative size of the particular class on the whole "
                                    "dataset, reducing the risk of overfitting due to unreliable estimates",
                       TypeConverters.toFloat)

    def _io(self):
        if self.isSet(self.inputCols):
            ins = list(self.getOrDefault(self.inputCols))
            outs = list(self.getOrDefault(self.outputCols)) if self.isSet(self.outputCols) else []
        else:
            ins = [self.getOrDefault(self.inputCol)]
            outs = [self.getOrDefault(self.outputCol)] if self.isSet(self.outputCol) else []
        if len(outs) != len(ins):
            raise ValueError("TargetEncoder needs one output column per input column")
        return ins, outs


def _slots(c: C.Column, name: str) -> torch.Tensor:
    """Category index + 1 per row (0 = null); invalid values (negative / non-integral) -> -1."""
    if not isinstance(c, C.NumericColumn):
        raise TypeError(f"TargetEncoder input column {name} must be numeric category indices")
    x = c.data.to(torch.float64)
    null = c.null_mask()
    bad = ~null & ((x < 0) | (x != torch.floor(x)) | torch.isnan(x))
    s = torch.where(null, torch.zeros_like(x), x + 1).to(torch.int64)
    return torch.where(bad, torch.full_like(s, -1), s)


@register("org.apache.spark.ml.feature.TargetEncoder")
class TargetEncoder(Estimator, _TargetEncoderParams, MLWritable, MLReadable):
    """Target encoding of categorical index columns (Spark 4.0 ``TargetEncoder``)."""

    @keyword_only
    def __init__(self, *, inputCols=None, outputCols=None, inputCol=None, outputCol=None, labelCol="label",
                 handleInvalid="error", targetType="binary", smoothing=0.0):
        super().__init__()
        self._setDefault(labelCol="label", handleInvalid="error", targetType="binary", smoothing=0.0)
        self._set(**self._input_kwargs)

    def _fit(self, df):
        ins, _ = self._io()
        tt = self.getOrDefault(self.targetType)
        if tt not in ("binary", "continuous"):
            raise ValueError(f"targetType must be binary or continuous, got {tt}")
        lab = df.column_data(self.getOrDefault(self.labelCol))
        y = lab.data.to(torch.float64)
        keep = ~lab.null_mask()                      # rows with a null label do not count
        if tt == "binary" and bool(((y != 0) & (y != 1) & keep).any()):
            raise ValueError("Values of label column for binary targetType must be 0 or 1")
        comm = df.comm
        slots = [_slots(df.column_data(n), n) for n in ins]
        for n, s in zip(ins, slots):
            if bool(((s < 0) & keep).any()):
                raise ValueError(f"Values from column {n} must be indices, but got a negative or non-integral value")
        sizes = torch.tensor([int(s.max()) + 1 if s.numel() else 1 for s in slots], dtype=torch.float64)
        sizes = comm.all_reduce(sizes.to(df.device), "max").cpu().long().tolist()
        parts = []
        for s, m in zip(slots, sizes):
            s = s[keep]
            parts.append(torch.bincount(s, minlength=m).to(torch.float64))
            parts.append(torch.bincount(s, weights=y[keep], minlength=m))
        parts = comm.all_reduce_coalesced(parts, "sum") if comm.world_size > 1 else parts
        m = TargetEncoderModel()
        m.stats = [(parts[2 * i], parts[2 * i + 1]) for i in range(len(ins))]
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.TargetEncoderModel")
class TargetEncoderModel(Model, _TargetEncoderParams, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self._setDefault(labelCol="label", handleInvalid="error", targetType="binary", smoothing=0.0)
        self.stats: list = []          # per input column: (counts, label sums) by slot (0 = null category)

    def _encodings(self, i: int):
        n, tot = self.stats[i]
        s = float(self.getOrDefault(self.smoothing))
        g = float(tot.sum()) / max(float(n.sum()), 1.0)
        w = n / (n + s) if s > 0 else torch.ones_like(n)
        enc = w * (tot / n.clamp_min(1.0)) + (1 - w) * g
        return enc, n > 0, g

    @property
    def encodings(self):
        """{column: {category: encoding}} with -1 = null and 2147483647 = unseen (Spark's keys)."""
        ins, _ = self._io()
        out = {}
        for i, name in enumerate(ins):
            enc, seen, g = self._encodings(i)
            d = {(k - 1 if k else NULL_CATEGORY): float(enc[k]) for k in torch.nonzero(seen).flatten().tolist()}
            d[UNSEEN_CATEGORY] = g
            out[name] = d
        return out

    def _transform(self, df):
        ins, outs = self._io()
        keep_invalid = self.getOrDefault(self.handleInvalid) == "keep"
        for i, (name, out) in enumerate(zip(ins, outs)):
            enc, seen, g = self._encodings(i)
            s = _slots(df.column_data(name), name)
            enc, seen = enc.to(s.device), seen.to(s.device)
            inside = (s >= 0) & (s < enc.numel())
            idx = torch.where(inside, s, torch.zeros_like(s))
            known = inside & seen[idx]
            if not keep_invalid and not bool(known.all()):
                raise ValueError(f"Unseen or invalid value in column {name} with handleInvalid='error' "
                                 "(set handleInvalid='keep' to encode it with the global statistic)")
            v = torch.where(known, enc[idx], torch.full_like(enc[idx], g))
            df = df.withColumnData(out, C.NumericColumn(v))
        return df

    def _save_data(self, path):
        rows = {"index": [], "category": [], "count": [], "stat": []}
        for i, (n, tot) in enumerate(self.stats):
            for k in torch.nonzero(n > 0).flatten().tolist():
                rows["index"].append(i)
                rows["category"].append(float(k - 1 if k else NULL_CATEGORY))
                rows["count"].append(float(n[k]))
                rows["stat"].append(float(tot[k]))
            rows["index"].append(i)                # empty columns keep their slot in the list
            rows["category"].append(float(UNSEEN_CATEGORY))
            rows["count"].append(0.0)
            rows["stat"].append(0.0)
        write_data(path, rows)

    @classmethod
    def _load_impl(cls, path, meta):
        m = cls()
        apply_metadata(m, meta)
        recs = read_data(path).to_pylist()
        nfeat = max((int(r["index"]) for r in recs), default=-1) + 1
        size = [1] * nfeat
        for r in recs:
            if r["category"] != UNSEEN_CATEGORY:
                size[int(r["index"])] = max(size[int(r["index"])], int(r["category"]) + 2)
        m.stats = [(torch.zeros(k, dtype=torch.float64), torch.zeros(k, dtype=torch.float64)) for k in size]
        for r in recs:
            if r["category"] == UNSEEN_CATEGORY:
                continue
            i, k = int(r["index"]), int(r["category"]) + 1
            m.stats[i][0][k] = r["count"]
            m.stats[i][1][k] = r["stat"]
        return m
