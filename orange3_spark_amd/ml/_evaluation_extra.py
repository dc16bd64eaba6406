"""MultilabelClassificationEvaluator and RankingEvaluator (``pyspark.ml.evaluation``,
Spark >= 3.0), listed by the Evaluation widget's reflection over ``evaluation``
(orangecontrib/spark/widgets/ml/spark_ml_evaluation.py:19-22).

Both read array columns (sets of labels / ranked item lists), which live on the host;
each rank reduces its rows to a handful of sums and the sums are combined across ranks
with one small all-reduce.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .base import Evaluator
from .param import HasLabelCol, HasPredictionCol, TypeConverters, keyword_only, shared
from .util import MLReadable, MLWritable, register


def _arrays(df, name):
    return [list(v) if v is not None else [] for v in df.column_data(name).values]


def _allreduce(df, vals):
    t = torch.tensor(vals, dtype=torch.float64, device=df.session.device)
    df.comm.all_reduce(t)
    return t.cpu().numpy()


@register("org.apache.spark.ml.evaluation.MultilabelClassificationEvaluator")
class MultilabelClassificationEvaluator(Evaluator, HasLabelCol, HasPredictionCol, MLWritable, MLReadable):
    """Evaluator for Multilabel Classification, which expects two input columns:
    prediction and label (both arrays of doubles)."""

    metricName = shared("metricName", "metric name in evaluation (subsetAccuracy|accuracy|hammingLoss|precision|"
                                      "recall|f1Measure|precisionByLabel|recallByLabel|f1MeasureByLabel|"
                                      "microPrecision|microRecall|microF1Measure)", TypeConverters.toString)
    metricLabel = shared("metricLabel", "The class whose metric will be computed in precisionByLabel|"
                                        "recallByLabel|f1MeasureByLabel. Must be >= 0. The default value is 0.",
                         TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, predictionCol="prediction", labelCol="label", metricName="f1Measure", metricLabel=0.0):
        super().__init__()
        self._setDefault(metricName="f1Measure", metricLabel=0.0)
        self._set(**self._input_kwargs)

    def _evaluate(self, df):
        g = self.getOrDefault
        P = _arrays(df, g(self.predictionCol))
        L = _arrays(df, g(self.labelCol))
        lab = float(g(self.metricLabel))
        subset = acc = prec = rec = f1 = 0.0
        tp = fp = fn = 0.0
        ltp = lfp = lfn = 0.0
        hamming = 0.0
        labels = set()
        for p, l in zip(P, L):
            ps, ls = set(map(float, p)), set(map(float, l))
            labels |= ls
            inter = len(ps & ls)
            uni = len(ps | ls)
            subset += float(ps == ls)
            acc += inter / uni if uni else 1.0
            prec += inter / len(ps) if ps else 0.0
            rec += inter / len(ls) if ls else 0.0
            f1 += 2.0 * inter / (len(ps) + len(ls)) if (ps or ls) else 0.0
            hamming += len(ps ^ ls)
            tp += inter
            fp += len(ps - ls)
            fn += len(ls - ps)
            ltp += float(lab in ps and lab in ls)
            lfp += float(lab in ps and lab not in ls)
            lfn += float(lab not in ps and lab in ls)
        nlab = len(set().union(*df.comm.all_gather_object(labels))) if df.comm.world_size > 1 else len(labels)
        s = _allreduce(df, [len(P), subset, acc, prec, rec, f1, hamming, tp, fp, fn, ltp, lfp, lfn])
        n, subset, acc, prec, rec, f1, hamming, tp, fp, fn, ltp, lfp, lfn = s
        m = g(self.metricName)
        div = lambda a, b: a / b if b else 0.0  # noqa: E731
        if m == "subsetAccuracy":
            return div(subset, n)
        if m == "accuracy":
            return div(acc, n)
        if m == "hammingLoss":
            return div(hamming, n * nlab)
        if m == "precision":
            return div(prec, n)
        if m == "recall":
            return div(rec, n)
        if m == "f1Measure":
            return div(f1, n)
        if m == "precisionByLabel":
            return div(ltp, ltp + lfp)
        if m == "recallByLabel":
            return div(ltp, ltp + lfn)
        if m == "f1MeasureByLabel":
            p_, r_ = div(ltp, ltp + lfp), div(ltp, ltp + lfn)
            return div(2 * p_ * r_, p_ + r_)
        if m == "microPrecision":
            return div(tp, tp + fp)
        if m == "microRecall":
            return div(tp, tp + fn)
        if m == "microF1Measure":
            return div(2 * tp, 2 * tp + fp + fn)
        raise ValueError(f"unsupported metric {m}")

    def isLargerBetter(self):
        return self.getOrDefault(self.metricName) != "hammingLoss"


@register("org.apache.spark.ml.evaluation.RankingEvaluator")
class RankingEvaluator(Evaluator, HasLabelCol, HasPredictionCol, MLWritable, MLReadable):
    """Evaluator for Ranking, which expects two input columns: prediction (ranked item list)
    and label (relevant items)."""

    metricName = shared("metricName", "metric name in evaluation (meanAveragePrecision|meanAveragePrecisionAtK|"
                                      "precisionAtK|ndcgAtK|recallAtK)", TypeConverters.toString)
    k = shared("k", "The ranking position value used in meanAveragePrecisionAtK|precisionAtK|ndcgAtK|recallAtK. "
                    "Must be > 0. The default value is 10.", TypeConverters.toInt)

    @keyword_only
    def __init__(self, *, predictionCol="prediction", labelCol="label", metricName="meanAveragePrecision", k=10):
        super().__init__()
        self._setDefault(metricName="meanAveragePrecision", k=10)
        self._set(**self._input_kwargs)

    def _evaluate(self, df):
        g = self.getOrDefault
        P = _arrays(df, g(self.predictionCol))
        L = _arrays(df, g(self.labelCol))
        k = int(g(self.k))
        m = g(self.metricName)
        total = 0.0
        for pred, lab in zip(P, L):
            rel = set(lab)
            if not rel:
                continue                                   # Spark logs a warning and scores 0
            if m in ("meanAveragePrecision", "meanAveragePrecisionAtK"):
                upto = len(pred) if m == "meanAveragePrecision" else min(k, len(pred))
                hits, s = 0, 0.0
                for i, p in enumerate(pred[:upto]):
                    if p in rel:
                        hits += 1
                        s += hits / (i + 1)
                total += s / (len(rel) if m == "meanAveragePrecision" else min(len(rel), k))
            elif m == "precisionAtK":
                total += sum(1 for p in pred[:k] if p in rel) / k
            elif m == "recallAtK":
                total += sum(1 for p in pred[:k] if p in rel) / len(rel)
            elif m == "ndcgAtK":
                dcg = sum(1.0 / math.log2(i + 2) for i, p in enumerate(pred[:k]) if p in rel)
                idcg = sum(1.0 / math.log2(i + 2) for i in range(min(len(rel), k)))
                total += dcg / idcg if idcg else 0.0
            else:
                raise ValueError(f"unsupported metric {m}")
        n, total = _allreduce(df, [len(P), total])
        return total / n if n else 0.0


_ = np
