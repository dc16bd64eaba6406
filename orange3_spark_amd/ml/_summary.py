"""Model summaries (``pyspark.ml.classification`` / ``regression`` summary classes).

Spark attaches a training summary to LogisticRegression / LinearSVC / LinearRegression
/ RandomForest / MLP / FM models and returns the same summary type from
``model.evaluate(df)``.  Here every metric is computed lazily from global sufficient
statistics on the device:

* per-label metrics from one k x k confusion matrix (``ops.evaluation.confusion``
  kernel + one all-reduce);
* binary curves (roc / pr / metric-by-threshold) from :func:`evaluation.binary_curve`
  (exact at small n, the 2^20-bin score-histogram kernel at large n);
* regression metrics from the 7-sum ``regression_stats`` kernel, and coefficient
  standard errors / t / p values from the all-reduced weighted Gram matrix
  (Spark: only for the "normal" solver; here whenever the Gram fits, D <= 4096).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame import column as C


def _frame(session_df, cols: dict):
    """Small replicated result table -> DataFrame (sharded like every other output)."""
    from collections import OrderedDict
    full = OrderedDict((k, C.NumericColumn(torch.as_tensor(np.asarray(v, dtype=np.float64)))) for k, v in cols.items())
    return session_df._from_full(full)


class _Lazy:
    def __init__(self, fn):
        self.fn, self.val, self.done = fn, None, False

    def get(self):
        if not self.done:
            self.val, self.done = self.fn(), True
        return self.val


class TrainingSummaryMixin:
    def _init_training(self, objectiveHistory=(), totalIterations=0, trainingSeconds=0.0, dataPasses=0):
        self.objectiveHistory = list(objectiveHistory)
        self.totalIterations = int(totalIterations)
        self.trainingSeconds = float(trainingSeconds)
        self.dataPasses = int(dataPasses)


class ClassificationSummary:
    """Multiclass metrics of a predictions DataFrame (Spark ClassificationSummary)."""

    def __init__(self, predictions, labelCol="label", predictionCol="prediction", weightCol=None):
        self._pred = _Lazy(predictions) if callable(predictions) else _Lazy(lambda: predictions)
        self.labelCol, self.predictionCol, self.weightCol = labelCol, predictionCol, weightCol
        self._cm = _Lazy(self._confusion)

    @property
    def predictions(self):
        return self._pred.get()

    def _confusion(self):
        from ..ops import evaluation as EV
        df = self.predictions
        y = df.column_data(self.labelCol).data
        p = df.column_data(self.predictionCol).data.to(y.device)
        w = df.column_data(self.weightCol).data.to(y.device) if self.weightCol else None
        k = int(df.comm.max_scalar(float(max(y.max().item() if y.numel() else 0,
                                                p.max().item() if p.numel() else 0)))) + 1
        cm = EV.confusion(y, p, k, w).reshape(-1)
        df.comm.all_reduce(cm)
        return cm.reshape(k, k).cpu().numpy()          # rows = label, cols = prediction

    # -- per label -------------------------------------------------------------------
    @property
    def labels(self):
        return [float(i) for i in range(self._cm.get().shape[0])]

    def _tp_fp_fn(self):
        cm = self._cm.get()
        tp = np.diag(cm)
        return tp, cm.sum(0) - tp, cm.sum(1) - tp, cm

    @property
    def truePositiveRateByLabel(self):
        return self.recallByLabel

    @property
    def falsePositiveRateByLabel(self):
        tp, fp, fn, cm = self._tp_fp_fn()
        neg = cm.sum() - cm.sum(1)
        return [float(f / n) if n > 0 else 0.0 for f, n in zip(fp, neg)]

    @property
    def precisionByLabel(self):
        tp, fp, _, _ = self._tp_fp_fn()
        return [float(t / (t + f)) if t + f > 0 else 0.0 for t, f in zip(tp, fp)]

    @property
    def recallByLabel(self):
        tp, _, fn, _ = self._tp_fp_fn()
        return [float(t / (t + f)) if t + f > 0 else 0.0 for t, f in zip(tp, fn)]

    def fMeasureByLabel(self, beta: float = 1.0):
        b2 = beta * beta
        out = []
        for p, r in zip(self.precisionByLabel, self.recallByLabel):
            out.append(float((1 + b2) * p * r / (b2 * p + r)) if p + r > 0 else 0.0)
        return out

    @property
    def accuracy(self):
        cm = self._cm.get()
        return float(np.trace(cm) / cm.sum()) if cm.sum() > 0 else 0.0

    def _weighted(self, vals):
        cm = self._cm.get()
        frac = cm.sum(1) / max(cm.sum(), 1e-300)
        return float(np.dot(frac, vals))

    @property
    def weightedTruePositiveRate(self):
        return self._weighted(self.truePositiveRateByLabel)

    @property
    def weightedFalsePositiveRate(self):
        return self._weighted(self.falsePositiveRateByLabel)

    @property
    def weightedRecall(self):
        return self._weighted(self.recallByLabel)

    @property
    def weightedPrecision(self):
        return self._weighted(self.precisionByLabel)

    def weightedFMeasure(self, beta: float = 1.0):
        return self._weighted(self.fMeasureByLabel(beta))


class BinaryClassificationSummary(ClassificationSummary):
    """Adds the threshold curves of a binary classifier (Spark BinaryClassificationSummary)."""

    def __init__(self, predictions, scoreCol="probability", **kw):
        super().__init__(predictions, **kw)
        self.scoreCol = scoreCol
        self._curve = _Lazy(self._compute_curve)

    def _compute_curve(self):
        from .evaluation import binary_curve
        df = self.predictions
        raw = df.column_data(self.scoreCol)
        s = raw.data[:, 1] if isinstance(raw, C.VectorColumn) and raw.data.shape[1] > 1 else \
            (raw.data[:, 0] if isinstance(raw, C.VectorColumn) else raw.data)
        y = df.column_data(self.labelCol).data.to(s.device)
        w = df.column_data(self.weightCol).data.to(s.device) if self.weightCol else None
        return binary_curve(df.comm, s, y, w)

    @property
    def areaUnderROC(self):
        from .evaluation import curve_areas
        _, tp, fp, P, N = self._curve.get()
        return curve_areas(tp, fp, P, N)[0]

    @property
    def roc(self):
        _, tp, fp, P, N = self._curve.get()
        fpr = np.concatenate([[0.0], fp / N if N > 0 else np.zeros_like(fp), [1.0]])
        tpr = np.concatenate([[0.0], tp / P if P > 0 else np.zeros_like(tp), [1.0]])
        return _frame(self.predictions, {"FPR": fpr, "TPR": tpr})

    def _pr_arrays(self):
        thr, tp, fp, P, N = self._curve.get()
        recall = tp / P if P > 0 else np.zeros_like(tp)
        precision = np.where(tp + fp > 0, tp / np.maximum(tp + fp, 1e-300), 1.0)
        return thr, recall, precision

    @property
    def pr(self):
        _, recall, precision = self._pr_arrays()
        first = precision[0] if len(precision) else 1.0
        return _frame(self.predictions, {"recall": np.concatenate([[0.0], recall]),
                                         "precision": np.concatenate([[first], precision])})

    @property
    def precisionByThreshold(self):
        thr, _, precision = self._pr_arrays()
        return _frame(self.predictions, {"threshold": thr, "precision": precision})

    @property
    def recallByThreshold(self):
        thr, recall, _ = self._pr_arrays()
        return _frame(self.predictions, {"threshold": thr, "recall": recall})

    @property
    def fMeasureByThreshold(self):
        thr, recall, precision = self._pr_arrays()
        f = np.where(precision + recall > 0, 2 * precision * recall / np.maximum(precision + recall, 1e-300), 0.0)
        return _frame(self.predictions, {"threshold": thr, "F-Measure": f})


class LogisticRegressionSummary(ClassificationSummary):
    def __init__(self, predictions, probabilityCol="probability", featuresCol="features", **kw):
        super().__init__(predictions, **kw)
        self.probabilityCol, self.featuresCol = probabilityCol, featuresCol


class LogisticRegressionTrainingSummary(LogisticRegressionSummary, TrainingSummaryMixin):
    def __init__(self, predictions, history=(), iterations=0, seconds=0.0, passes=0, **kw):
        super().__init__(predictions, **kw)
        self._init_training(history, iterations, seconds, passes)


class BinaryLogisticRegressionSummary(BinaryClassificationSummary):
    def __init__(self, predictions, probabilityCol="probability", featuresCol="features", **kw):
        super().__init__(predictions, scoreCol=probabilityCol, **kw)
        self.probabilityCol, self.featuresCol = probabilityCol, featuresCol


class BinaryLogisticRegressionTrainingSummary(BinaryLogisticRegressionSummary, TrainingSummaryMixin):
    def __init__(self, predictions, history=(), iterations=0, seconds=0.0, passes=0, **kw):
        super().__init__(predictions, **kw)
        self._init_training(history, iterations, seconds, passes)


class LinearSVCSummary(BinaryClassificationSummary):
    def __init__(self, predictions, **kw):
        super().__init__(predictions, scoreCol="rawPrediction", **kw)


class LinearSVCTrainingSummary(LinearSVCSummary, TrainingSummaryMixin):
    def __init__(self, predictions, history=(), iterations=0, seconds=0.0, passes=0, **kw):
        super().__init__(predictions, **kw)
        self._init_training(history, iterations, seconds, passes)


class LinearRegressionSummary:
    """Spark LinearRegressionSummary: error metrics, residuals and (when the weighted Gram
    matrix is available) coefficient standard errors, t- and p-values."""

    def __init__(self, predictions, labelCol="label", predictionCol="prediction", featuresCol="features",
                 weightCol=None, coefficients=None, intercept=0.0, fitIntercept=True, regParam=0.0):
        self._pred = _Lazy(predictions) if callable(predictions) else _Lazy(lambda: predictions)
        self.labelCol, self.predictionCol, self.featuresCol, self.weightCol = labelCol, predictionCol, featuresCol, \
            weightCol
        self._coef = None if coefficients is None else np.asarray(coefficients, dtype=np.float64)
        self._intercept, self._fit_intercept, self._reg = float(intercept), bool(fitIntercept), float(regParam)
        self._st = _Lazy(self._stats)
        self._inf = _Lazy(self._inference)

    @property
    def predictions(self):
        return self._pred.get()

    def _stats(self):
        from ..ops import evaluation as EV
        df = self.predictions
        y = df.column_data(self.labelCol).data
        p = df.column_data(self.predictionCol).data.to(y.device)
        w = df.column_data(self.weightCol).data.to(y.device) if self.weightCol else None
        st = EV.regression_stats(y, p, w)
        df.comm.all_reduce(st)
        W, se, ae, sy, syy, sp, spp = st.cpu().tolist()
        n = df.count()
        return dict(W=W, se=se, ae=ae, sy=sy, syy=syy, sp=sp, spp=spp, n=n)

    @property
    def numInstances(self):
        return int(self._st.get()["n"])

    @property
    def degreesOfFreedom(self):
        k = 0 if self._coef is None else len(self._coef)
        return int(self.numInstances - k - (1 if self._fit_intercept else 0))

    @property
    def meanSquaredError(self):
        s = self._st.get()
        return s["se"] / s["W"]

    @property
    def rootMeanSquaredError(self):
        return math.sqrt(self.meanSquaredError)

    @property
    def meanAbsoluteError(self):
        s = self._st.get()
        return s["ae"] / s["W"]

    @property
    def r2(self):
        s = self._st.get()
        ss_tot = s["syy"] - s["sy"] ** 2 / s["W"] if self._fit_intercept else s["syy"]
        return 1 - s["se"] / ss_tot if ss_tot else float("nan")

    @property
    def r2adj(self):
        n = self.numInstances
        k = 0 if self._coef is None else len(self._coef)
        i = 1 if self._fit_intercept else 0
        return 1 - (1 - self.r2) * (n - i) / max(n - k - i, 1)

    @property
    def explainedVariance(self):
        s = self._st.get()
        mean_y = s["sy"] / s["W"]
        # sum w (p - mean_y)^2 / W  (Spark RegressionMetrics.explainedVariance)
        return (s["spp"] - 2 * mean_y * s["sp"] + mean_y * mean_y * s["W"]) / s["W"]

    @property
    def residuals(self):
        from ..frame import expr as E
        return self.predictions.select((E.col(self.labelCol) - E.col(self.predictionCol)).alias("residuals"))

    @property
    def devianceResiduals(self):
        r = self.residuals
        c = r.column_data("residuals").data
        mn = r.comm.all_gather_object(float(c.min()) if c.numel() else math.inf)
        mx = r.comm.all_gather_object(float(c.max()) if c.numel() else -math.inf)
        return [min(mn), max(mx)]

    def _inference(self):
        """(std errors, t values, p values), intercept last (Spark order)."""
        from scipy import stats
        if self._coef is None:
            raise RuntimeError("coefficient statistics need the model coefficients")
        df = self.predictions
        X = df.column_data(self.featuresCol)
        Xd = (X.dense() if isinstance(X, C.VectorColumn) else X.to_dense(torch.float64)).to(torch.float64)
        w = df.column_data(self.weightCol).data.to(Xd.device, torch.float64) if self.weightCol else None
        if self._fit_intercept:
            Xd = torch.cat([Xd, torch.ones(Xd.shape[0], 1, dtype=torch.float64, device=Xd.device)], 1)
        Xw = Xd if w is None else Xd * w[:, None]
        from ..ops.gram import rows_t_matmul
        G = rows_t_matmul(Xw, Xd)
        df.comm.all_reduce(G)
        G = G.cpu().numpy()
        dof = self.degreesOfFreedom
        sigma2 = self._st.get()["se"] / max(dof, 1)
        cov = np.linalg.pinv(G) * sigma2
        se = np.sqrt(np.clip(np.diag(cov), 0, None))
        beta = np.concatenate([self._coef, [self._intercept]]) if self._fit_intercept else self._coef
        t = np.where(se > 0, beta / np.maximum(se, 1e-300), np.nan)
        pv = 2 * stats.t.sf(np.abs(t), max(dof, 1))
        return se.tolist(), t.tolist(), pv.tolist()

    @property
    def coefficientStandardErrors(self):
        return self._inf.get()[0]

    @property
    def tValues(self):
        return self._inf.get()[1]

    @property
    def pValues(self):
        return self._inf.get()[2]


class LinearRegressionTrainingSummary(LinearRegressionSummary, TrainingSummaryMixin):
    def __init__(self, predictions, history=(), iterations=0, **kw):
        super().__init__(predictions, **kw)
        self._init_training(history, iterations)
