"""Statistics (``pyspark.ml.stat``): ChiSquareTest, Correlation, Summarizer, KolmogorovSmirnovTest.

Sufficient statistics are computed per rank on device and all-reduced; the small final
computations (p-values) run on the host with scipy.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from ..runtime.executors import ship

from ..frame import column as C
from ..frame.dataframe import DataFrame
from . import common as U
from .linalg import DenseMatrix, DenseVector
from ._clustering_extra import MultivariateGaussian  # noqa: F401  (pyspark.ml.stat export)


def chi_square_pvalues(comm, X: torch.Tensor, y: torch.Tensor, return_all=False):
    """Pearson chi-square independence test of each (categorical) feature vs the label."""
    from scipy.stats import chi2
    pv, stats, dofs = [], [], []
    yl = y.long()
    ky = int(comm.max_scalar(float(yl.max().item()) if yl.numel() else 0.0)) + 1
    for j in range(X.shape[1]):
        xv = X[:, j]
        vals = torch.unique(xv)
        allv = torch.unique(comm.all_gather_v(vals)) if comm.world_size > 1 else vals
        xi = torch.searchsorted(allv, xv)
        kx = allv.numel()
        tab = torch.zeros(kx * ky, dtype=torch.float64, device=X.device).index_add_(
            0, xi * ky + yl, torch.ones_like(xv, dtype=torch.float64))
        comm.all_reduce(tab)
        t = tab.reshape(kx, ky).cpu().numpy()
        n = t.sum()
        exp = t.sum(1, keepdims=True) * t.sum(0, keepdims=True) / max(n, 1)
        with np.errstate(divide="ignore", invalid="ignore"):
            st = float(np.nansum(np.where(exp > 0, (t - exp) ** 2 / exp, 0.0)))
        dof = (kx - 1) * (ky - 1)
        stats.append(st)
        dofs.append(dof)
        pv.append(float(chi2.sf(st, dof)) if dof > 0 else 1.0)
    if return_all:
        return np.array(pv), np.array(stats), np.array(dofs)
    return np.array(pv)


class ChiSquareTest:
    @staticmethod
    @ship
    def test(dataset, featuresCol, labelCol, flatten=False):
        X = U.dense_features(dataset, featuresCol, torch.float64)
        y = U.numeric_column(dataset, labelCol)
        p, s, d = chi_square_pvalues(dataset.comm, X, y, True)
        s_ = dataset.session
        if flatten:
            import pandas as pd
            return s_.createDataFrame(pd.DataFrame({"featureIndex": np.arange(len(p)), "pValue": p,
                                                    "degreesOfFreedom": d.astype(np.int64), "statistic": s}))
        cols = OrderedDict(pValues=C.VectorColumn(torch.from_numpy(p)[None, :]),
                           degreesOfFreedom=C.ArrayColumn([[int(v) for v in d]]),
                           statistics=C.VectorColumn(torch.from_numpy(s)[None, :]))
        return DataFrame(s_.local_view(), cols)


class Correlation:
    @staticmethod
    @ship
    def corr(dataset, column, method="pearson"):
        X = U.dense_features(dataset, column, torch.float64)
        comm = dataset.comm
        if method == "spearman":
            X = comm.all_gather_v(X) if comm.world_size > 1 else X
            X = X.argsort(0).argsort(0).to(torch.float64)   # ranks (ties broken by order)
            comm_ = None
        else:
            comm_ = comm
        d = X.shape[1]
        from ..ops.gram import rows_t_matmul
        st = torch.cat([rows_t_matmul(X, X).reshape(-1), X.sum(0), torch.tensor([float(X.shape[0])], dtype=torch.float64,
                                                                       device=X.device)])
        if comm_ is not None:
            comm_.all_reduce(st)
        G, s, n = st[: d * d].reshape(d, d), st[d * d: d * d + d], st[-1]
        cov = (G - torch.outer(s, s) / n) / (n - 1)
        sd = torch.sqrt(torch.diag(cov))
        corr = cov / torch.outer(sd, sd)
        m = DenseMatrix.from_array(corr.cpu().numpy())
        cols = OrderedDict()
        cols[f"{method}({column})"] = C.HostColumn([m]) if False else _matrix_col(m)
        return DataFrame(dataset.session.local_view(), cols)


def _matrix_col(m):
    arr = np.empty(1, dtype=object)
    arr[0] = m
    c = C.HostColumn(arr)
    c.dtype = C.T.StringType()
    return c


class SummaryBuilder:
    def __init__(self, metrics):
        self.metrics = list(metrics)

    def summary(self, featuresCol, weightCol=None):
        return _SummaryExpr(self.metrics, featuresCol, weightCol)


class _SummaryExpr:
    def __init__(self, metrics, featuresCol, weightCol):
        self.metrics, self.featuresCol, self.weightCol = metrics, featuresCol, weightCol
        self.name = "aggregate_metrics(" + str(featuresCol) + ")"


class Summarizer:
    """Vector column summary statistics (mean, variance, count, numNonZeros, max, min, normL1, normL2, sum, std)."""

    @staticmethod
    def metrics(*metrics):
        return SummaryBuilder(metrics)

    @staticmethod
    @ship
    def compute(dataset, featuresCol, metrics, weightCol=None):
        X = U.dense_features(dataset, featuresCol, torch.float64)
        w = torch.ones(X.shape[0], dtype=torch.float64, device=X.device) if weightCol is None else \
            U.numeric_column(dataset, weightCol).to(X.device)
        comm = dataset.comm
        d = X.shape[1]
        st = torch.cat([w @ X, w @ (X * X), (X != 0).sum(0).double(), (w[:, None] * X.abs()).sum(0),
                        torch.stack([w.sum(), (w * w).sum(), torch.tensor(float(X.shape[0]), dtype=torch.float64,
                                                                             device=X.device)])])
        comm.all_reduce(st)
        mx = X.max(0).values.contiguous() if X.shape[0] else torch.full((d,), -np.inf, dtype=torch.float64,
                                                                         device=X.device)
        mn = X.min(0).values.contiguous() if X.shape[0] else torch.full((d,), np.inf, dtype=torch.float64,
                                                                         device=X.device)
        comm.all_reduce(mx, "max")
        comm.all_reduce(mn, "min")
        s1, s2, nnz, l1 = st[:d], st[d:2 * d], st[2 * d:3 * d], st[3 * d:4 * d]
        W, W2, cnt = st[4 * d], st[4 * d + 1], st[4 * d + 2]
        mean = s1 / W
        var = (s2 / W - mean * mean) * (W * W / (W * W - W2)) if float(W * W - W2) > 0 else torch.zeros_like(mean)
        out = {"mean": mean, "variance": var, "std": var.sqrt(), "count": int(cnt), "numNonZeros": nnz,
               "max": mx, "min": mn, "normL1": l1, "normL2": s2.sqrt(), "sum": s1}
        res = {}
        for m in metrics:
            v = out[m]
            res[m] = v if isinstance(v, int) else DenseVector(v.cpu().numpy())
        return res

    @staticmethod
    def mean(col, weightCol=None):
        return _SummaryExpr(["mean"], col, weightCol)


class KolmogorovSmirnovTest:
    @staticmethod
    @ship
    def test(dataset, sampleCol, distName="norm", *params):
        from scipy import stats
        x = U.numeric_column(dataset, sampleCol)
        x = dataset.comm.all_gather_v(x) if dataset.comm.world_size > 1 else x
        r = stats.kstest(x.cpu().numpy(), distName, args=params)
        return dataset.session.createDataFrame([(float(r.pvalue), float(r.statistic))], ["pValue", "statistic"])


def _test_frame(dataset, p, dof, stat, flatten):
    s_ = dataset.session
    if flatten:
        import pandas as pd
        return s_.createDataFrame(pd.DataFrame({"featureIndex": np.arange(len(p)), "pValue": p,
                                                "degreesOfFreedom": np.asarray(dof, dtype=np.int64),
                                                "fValue": stat}))
    cols = OrderedDict(pValues=C.VectorColumn(torch.from_numpy(np.asarray(p, dtype=np.float64))[None, :]),
                       degreesOfFreedom=C.ArrayColumn([[int(v) for v in dof]]),
                       fValues=C.VectorColumn(torch.from_numpy(np.asarray(stat, dtype=np.float64))[None, :]))
    return DataFrame(s_.local_view(), cols)


class ANOVATest:
    """ANOVA F-test of continuous features against a categorical label (Spark >= 3.1)."""

    @staticmethod
    @ship
    def test(dataset, featuresCol, labelCol, flatten=False):
        from ._feature_extra import anova_f
        X = U.dense_features(dataset, featuresCol, torch.float64)
        y = U.numeric_column(dataset, labelCol)
        F, p, dof = anova_f(dataset.comm, X, y)
        return _test_frame(dataset, p, dof, F, flatten)


class FValueTest:
    """F-value regression test of continuous features against a continuous label."""

    @staticmethod
    @ship
    def test(dataset, featuresCol, labelCol, flatten=False):
        from ._feature_extra import f_regression
        X = U.dense_features(dataset, featuresCol, torch.float64)
        y = U.numeric_column(dataset, labelCol)
        F, p, dof = f_regression(dataset.comm, X, y)
        return _test_frame(dataset, p, dof, F, flatten)
