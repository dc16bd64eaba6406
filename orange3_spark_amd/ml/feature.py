"""Feature transformers and estimators (``pyspark.ml.feature`` surface).

The reference's Feature widget exposes this module's Transformers
(orangecontrib/spark/widgets/ml/spark_ml_feature.py:15); the Dataset Builder runs
``VectorAssembler(inputCols=features, outputCol='features')``
(widgets/ml/spark_ml_dataset.py:575-576).  Feature *Estimators* (StandardScaler,
StringIndexer, IDF, PCA, ...) are exposed by the add-on's "Feature Estimator" widget
(the reference could not reach them).

Dense numeric work is torch on the session device (memory-bound elementwise/GEMM ops);
term hashing runs the MurmurHash3 HIP kernel (ops/text.py); column statistics are
all-reduced over the session communicator.
"""
from __future__ import annotations

import math
import re
from collections import Counter, OrderedDict

import numpy as np
import torch

from ..frame import column as C
from ..frame.spill import SpilledVectorColumn, block_moments, map_blocks
from ..ops import glm as G
from ..ops import text as TX
from . import common as U
from .base import Estimator, Model, Transformer
from .linalg import DenseMatrix, DenseVector
from .param import (HasFeaturesCol, HasHandleInvalid, HasInputCol, HasInputCols, HasLabelCol, HasMaxIter,
                    HasNumFeatures, HasOutputCol, HasOutputCols, HasSeed, HasStepSize, HasTol, HasWeightCol,
                    TypeConverters, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, prim_list, read_data, register, vec_col, write_data


# ----------------------------------------------------------------------------- helpers
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


from ._selector import _SelectorModel  # noqa: E402


def _vec(df, name) -> torch.Tensor:
    return U.dense_features(df, name, torch.float64)


def _out_vec(df, name, mat):
    return df.withColumnData(name, to_vector_column(df.session, mat) if df.session.device.type == "cuda"
                             else C.VectorColumn(mat.to(torch.float64)))


def _strings(df, name) -> list:
    c = df.column_data(name)
    if isinstance(c, C.HostColumn):
        return list(c.values)
    return [None if v is None else _num_str(v) for v in c.to_pylist()]


def _num_str(v):
    return repr(float(v)) if isinstance(v, float) else str(v)


def _value_counts(df, name) -> dict:
    """{string form: count} of the non-null values of a column, without a per-row Python
    loop: numeric columns count their distinct values on device (torch.unique) and format
    only those; string columns use pandas' hash table."""
    import pandas as pd
    c = df.column_data(name)
    if isinstance(c, C.HostColumn):
        vc = pd.Series(c.values, dtype=object).value_counts(dropna=True)
        return dict(zip(vc.index.tolist(), vc.values.tolist()))
    if isinstance(c, C.NumericColumn):
        data = c.data if c.valid is None else c.data[c.valid.to(c.data.device)]
        vals, counts = torch.unique(data, return_counts=True)
        out: dict = {}
        for v, k in zip(vals.tolist(), counts.tolist()):
            key = _num_str(v)
            out[key] = out.get(key, 0) + int(k)
        return out
    return Counter(v for v in _strings(df, name) if v is not None)


def _index_values(df, name, idx: dict):
    """(float64 label index per row, NaN for null / unseen; first unseen value or None)."""
    import pandas as pd
    c = df.column_data(name)
    if isinstance(c, C.NumericColumn):
        uniq, inv = torch.unique(c.data, return_inverse=True)
        lut = np.array([idx.get(_num_str(v), np.nan) for v in uniq.tolist()], dtype=np.float64)
        res = lut[inv.cpu().numpy()]
        if c.valid is not None:
            res[~c.valid.cpu().numpy()] = np.nan
        bad_u = [v for v, l in zip(uniq.tolist(), lut) if np.isnan(l)]
        return res, (_num_str(bad_u[0]) if bad_u else None)
    vals = c.values if isinstance(c, C.HostColumn) else np.asarray(_strings(df, name), dtype=object)
    res = pd.Series(vals, dtype=object).map(idx).to_numpy(dtype=np.float64, na_value=np.nan)
    bad = np.isnan(res)
    return res, (vals[int(np.argmax(bad))] if bad.any() else None)


class _InOut(HasInputCol, HasOutputCol):
    def __init__(self):
        super().__init__()
        self._setDefault(outputCol=self.uid + "__output")


class _Simple(Transformer, _InOut, MLWritable, MLReadable):
    """Base for stateless inputCol -> outputCol transformers."""

    def _transform(self, df):
        return df.withColumnData(self.getOrDefault(self.outputCol), self._apply(df, self.getOrDefault(self.inputCol)))


# ============================================================================ assemblers
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
        streamed = self._transform_streamed(df, cols, n)
        if streamed is not None:
            return streamed
        fused = self._transform_fused(df, cols, n)
        if fused is not None:
            return fused
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

    def _transform_streamed(self, df, cols, n):
        """Out-of-core assembly (frame/spill.assemble_streamed): when an input column is
        host-resident (a table larger than the HBM budget) or the assembled matrix would
        not fit the budget, the rows are assembled chunk by chunk into a
        SpilledVectorColumn -- resident prefix up to the budget, the rest in pinned host
        memory; nothing of full length is materialised on the device."""
        from ..frame import spill
        from ..synthetic import LineageVectorColumn
        if not cols or n == 0:
            return None
        srcs = []
        host_in = False
        for c in cols:
            col = df.column_data(c)
            if isinstance(col, C.NumericColumn) and col.data.dim() == 1:
                srcs.append((col.data, col.valid, 1))
            elif type(col) is C.VectorColumn and col.data.dim() == 2:
                srcs.append((col.data, None, int(col.size)))
            else:
                return None
            host_in |= col.data.device != df.device
        budget = spill.ingest_budget(df.session)
        explicit = df.session.conf.get("o3s.storage.hbmBudget", None) not in (None, "", "auto")
        D = sum(w for _, _, w in srcs)
        esz = torch.empty((), dtype=df.session.vector_dtype()).element_size()
        too_big = budget is not None and n * D * esz > budget and (explicit or df.device.type == "cuda")
        if not host_in and not too_big:
            return None
        _ = LineageVectorColumn
        hi = self.getOrDefault(self.handleInvalid)
        got = spill.assemble_streamed(srcs, n, df.session, budget, want_bad=hi == "skip")
        out, nbad = got[0], got[1]
        if nbad:
            if hi == "error":
                raise ValueError("Encountered null while assembling a row with handleInvalid = \"error\". "
                                 "Consider removing nulls from dataset or using handleInvalid = \"keep\" or \"skip\".")
            if hi == "skip":             # drop the flagged rows from every column, layout kept
                return df.withColumnData(self.getOrDefault(self.outputCol), out)._mask(~got[2])
        return df.withColumnData(self.getOrDefault(self.outputCol), out)

    def _transform_fused(self, df, cols, n):
        """GPU, bf16 feature storage: ONE gather kernel (ops/assemble.py) reads every input
        column once (any numeric dtype, null masks, vector columns) and writes the padded
        bf16 matrix once, flagging invalid rows in the same pass; None -> torch path."""
        from ..ops import assemble as A
        from ..synthetic import LineageVectorColumn
        if df.device.type != "cuda" or df.session.vector_dtype() != torch.bfloat16 or not cols or n == 0 \
                or len(cols) > A.MAX_SOURCES:
            return None
        srcs = []
        for c in cols:
            col = df.column_data(c)
            if isinstance(col, C.NumericColumn) and A.supported(col.data) and col.data.dim() == 1:
                srcs.append((col.data.contiguous(), col.valid, 1))
            elif isinstance(col, C.VectorColumn) and not isinstance(col, (C.SparseVectorColumn, LineageVectorColumn)) \
                    and A.supported(col.data) and col.data.dim() == 2:
                srcs.append((col.data, None, int(col.size)))
            else:
                return None
        out, bad, nbad, D = A.assemble_bf16(srcs, n, df.device)
        nb = int(nbad.item())
        if nb:
            hi = self.getOrDefault(self.handleInvalid)
            if hi == "error":
                raise ValueError("Encountered null while assembling a row with handleInvalid = \"error\". "
                                 "Consider removing nulls from dataset or using handleInvalid = \"keep\" or \"skip\".")
            if hi == "skip":
                keep = bad == 0
                df = df._mask(keep)
                out = out[keep]
        return df.withColumnData(self.getOrDefault(self.outputCol), C.VectorColumn(out, D))


@register("org.apache.spark.ml.feature.VectorSlicer")
class VectorSlicer(_Simple):
    """Slices a vector column by feature indices."""

    indices = shared("indices", "An array of indices to select features from a vector column. There can be no "
                                "overlap with names.", TypeConverters.toListInt)
    names = shared("names", "An array of feature names to select features from a vector column. These names must "
                            "be specified by ML org.apache.spark.ml.attribute.Attribute. There can be no overlap "
                            "with indices.", TypeConverters.toListString)

    @keyword_only
    def __init__(self, *, inputCol=None, outputCol=None, indices=None, names=None):
        super().__init__()
        self._setDefault(indices=[], names=[])
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        idx = torch.tensor(self.getOrDefault(self.indices), dtype=torch.int64, device=df.device)
        return C.VectorColumn(_vec(df, name)[:, idx])


@register("org.apache.spark.ml.feature.VectorSizeHint")
class VectorSizeHint(Transformer, HasInputCol, HasHandleInvalid, MLWritable, MLReadable):
    """Checks the size of vectors in a column."""

    size = shared("size", "Size of vectors in column.", TypeConverters.toInt)

    @keyword_only
    def __init__(self, *, inputCol=None, size=None, handleInvalid="error"):
        super().__init__()
        self._setDefault(handleInvalid="error")
        self._set(**self._input_kwargs)

    def _transform(self, df):
        c = df.column_data(self.getOrDefault(self.inputCol))
        if getattr(c, "size", None) != self.getOrDefault(self.size) and self.getOrDefault(self.handleInvalid) == "error":
            raise ValueError(f"vector size {getattr(c, 'size', None)} != {self.getOrDefault(self.size)}")
        return df


# ============================================================================ elementwise
@register("org.apache.spark.ml.feature.Binarizer")
class Binarizer(_Simple):
    """Binarize a column of continuous features given a threshold."""

    threshold = shared("threshold", "Param for threshold used to binarize continuous features. The features "
                                    "greater than the threshold will be binarized to 1.0. The features equal to or "
                                    "less than the threshold will be binarized to 0.0", TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, threshold=0.0, inputCol=None, outputCol=None):
        super().__init__()
        self._setDefault(threshold=0.0)
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        c = df.column_data(name)
        t = self.getOrDefault(self.threshold)
        if isinstance(c, C.NumericColumn):
            return C.NumericColumn((c.data.to(torch.float64) > t).to(torch.float64))
        return C.VectorColumn((_vec(df, name) > t).to(torch.float64))


@register("org.apache.spark.ml.feature.Bucketizer")
class Bucketizer(_Simple, HasHandleInvalid):
    """Maps a column of continuous features to a column of feature buckets."""

    splits = shared("splits", "Split points for mapping continuous features into buckets. With n+1 splits, there "
                              "are n buckets. A bucket defined by splits x,y holds values in the range [x,y) except "
                              "the last bucket, which also includes y. The splits should be of length >= 3 and "
                              "strictly increasing. Values at -inf, inf must be explicitly provided to cover all "
                              "Double values; otherwise, values outside the splits specified will be treated as "
                              "errors.", TypeConverters.toListFloat)

    @keyword_only
    def __init__(self, *, splits=None, inputCol=None, outputCol=None, handleInvalid="error"):
        super().__init__()
        self._setDefault(handleInvalid="error")
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        x = df.column_data(name).data.to(torch.float64)
        s = torch.tensor(self.getOrDefault(self.splits), dtype=torch.float64, device=x.device)
        b = torch.bucketize(x, s, right=True) - 1
        b = torch.where(x == s[-1], torch.full_like(b, s.numel() - 2), b)
        bad = torch.isnan(x) | (b < 0) | (b > s.numel() - 2)
        hi = self.getOrDefault(self.handleInvalid)
        if bool(bad.any()):
            if hi == "error":
                raise ValueError("Bucketizer: value out of splits range or NaN (handleInvalid='error')")
            b = torch.where(bad, torch.full_like(b, s.numel() - 1), b)
            if hi == "skip":
                return C.NumericColumn(b.to(torch.float64), ~bad)
        return C.NumericColumn(b.to(torch.float64))


@register("org.apache.spark.ml.feature.Normalizer")
class Normalizer(_Simple):
    """Normalize a vector to have unit norm using the given p-norm."""

    p = shared("p", "the p norm value.", TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, p=2.0, inputCol=None, outputCol=None):
        super().__init__()
        self._setDefault(p=2.0)
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        X = _vec(df, name)
        nrm = torch.linalg.vector_norm(X, ord=self.getOrDefault(self.p), dim=1, keepdim=True)
        return C.VectorColumn(torch.where(nrm > 0, X / nrm, X))


@register("org.apache.spark.ml.feature.ElementwiseProduct")
class ElementwiseProduct(_Simple):
    """Hadamard product of each input vector with a provided "weight" vector."""

    scalingVec = shared("scalingVec", "Vector for hadamard product.", TypeConverters.toVector)

    @keyword_only
    def __init__(self, *, scalingVec=None, inputCol=None, outputCol=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        v = torch.from_numpy(self.getOrDefault(self.scalingVec).toArray()).to(df.device)
        return C.VectorColumn(_vec(df, name) * v[None, :])


@register("org.apache.spark.ml.feature.PolynomialExpansion")
class PolynomialExpansion(_Simple):
    """Expand the features into a polynomial space (Spark ordering)."""

    degree = shared("degree", "the polynomial degree to expand (>= 1)", TypeConverters.toInt)

    @keyword_only
    def __init__(self, *, degree=2, inputCol=None, outputCol=None):
        super().__init__()
        self._setDefault(degree=2)
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        X = _vec(df, name)
        return C.VectorColumn(_poly_expand(X, self.getOrDefault(self.degree)))


def _poly_expand(X: torch.Tensor, degree: int) -> torch.Tensor:
    """Spark PolynomialExpansion order: recursive over features (last feature outermost)."""
    n, d = X.shape

    def expand(k, deg):
        # all monomials of features[0..k) with total degree in [0, deg], Spark's order
        if k == 0:
            return [torch.ones(n, dtype=X.dtype, device=X.device)]
        out = []
        x = X[:, k - 1]
        p = torch.ones(n, dtype=X.dtype, device=X.device)
        for e in range(deg + 1):
            out += [m * p for m in expand(k - 1, deg - e)]
            p = p * x
        return out
    terms = expand(d, degree)[1:]
    return torch.stack(terms, 1)


@register("org.apache.spark.ml.feature.DCT")
class DCT(_Simple):
    """Discrete cosine transform (DCT-II, orthonormal scaling as in Spark/JTransforms)."""

    inverse = shared("inverse", "Set transformer to perform inverse DCT, default False.", TypeConverters.toBoolean)

    @keyword_only
    def __init__(self, *, inverse=False, inputCol=None, outputCol=None):
        super().__init__()
        self._setDefault(inverse=False)
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        X = _vec(df, name)
        N_ = X.shape[1]
        k = torch.arange(N_, dtype=torch.float64, device=X.device)
        M = torch.cos(math.pi / N_ * (k[None, :] + 0.5) * k[:, None])   # [k, n]
        M = M * math.sqrt(2.0 / N_)
        M[0] = M[0] / math.sqrt(2.0)
        return C.VectorColumn(X @ (M if self.getOrDefault(self.inverse) else M.T))


@register("org.apache.spark.ml.feature.Interaction")
class Interaction(Transformer, HasInputCols, HasOutputCol, MLWritable, MLReadable):
    """All-pairs products of the input columns' values (one vector per row)."""

    @keyword_only
    def __init__(self, *, inputCols=None, outputCol=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _transform(self, df):
        mats = [_as_matrix(df.column_data(c), len(df), df.device) for c in self.getOrDefault(self.inputCols)]
        out = mats[0]
        for m in mats[1:]:
            out = (out[:, :, None] * m[:, None, :]).reshape(out.shape[0], -1)
        return df.withColumnData(self.getOrDefault(self.outputCol), C.VectorColumn(out))


@register("org.apache.spark.ml.feature.SQLTransformer")
class SQLTransformer(Transformer, MLWritable, MLReadable):
    """Implements the transforms which are defined by SQL statement ("SELECT ... FROM __THIS__")."""

    statement = shared("statement", "SQL statement", TypeConverters.toString)

    @keyword_only
    def __init__(self, *, statement=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _transform(self, df):
        name = "__THIS__"
        df.session.catalog.registerTempView(name, df)
        try:
            return df.session.sql(self.getOrDefault(self.statement))
        finally:
            df.session.catalog.dropTempView(name)


# ============================================================================ text
@register("org.apache.spark.ml.feature.Tokenizer")
class Tokenizer(_Simple):
    """A tokenizer that converts the input string to lowercase and then splits it by white spaces."""

    @keyword_only
    def __init__(self, *, inputCol=None, outputCol=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        vals = _strings(df, name)
        dev = TX.device_tokenize(np.asarray(vals, dtype=object), df.device) if df.device.type == "cuda" else None
        return dev if dev is not None else C.ArrayColumn(TX.tokenize_lower_ws(vals))


@register("org.apache.spark.ml.feature.RegexTokenizer")
class RegexTokenizer(_Simple):
    """A regex based tokenizer that extracts tokens either by using the provided regex pattern
    (in Java dialect) to split the text (default) or repeatedly matching the regex (if gaps is false)."""

    minTokenLength = shared("minTokenLength", "minimum token length (>= 0)", TypeConverters.toInt)
    gaps = shared("gaps", "whether regex splits on gaps (True) or matches tokens (False)", TypeConverters.toBoolean)
    pattern = shared("pattern", "regex pattern (Java dialect) used for tokenizing", TypeConverters.toString)
    toLowercase = shared("toLowercase", "whether to convert all characters to lowercase before tokenizing",
                         TypeConverters.toBoolean)

    @keyword_only
    def __init__(self, *, minTokenLength=1, gaps=True, pattern="\\s+", inputCol=None, outputCol=None,
                 toLowercase=True):
        super().__init__()
        self._setDefault(minTokenLength=1, gaps=True, pattern="\\s+", toLowercase=True)
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        rx = re.compile(self.getOrDefault(self.pattern))
        gaps, low, mn = self.getOrDefault(self.gaps), self.getOrDefault(self.toLowercase), \
            self.getOrDefault(self.minTokenLength)
        out = []
        for s in _strings(df, name):
            if s is None:
                out.append(None)
                continue
            s = s.lower() if low else s
            toks = rx.split(s) if gaps else rx.findall(s)
            out.append([t for t in toks if len(t) >= mn])
        return C.ArrayColumn(out)


_EN_STOP = ("i me my myself we our ours ourselves you your yours yourself yourselves he him his himself she her "
            "hers herself it its itself they them their theirs themselves what which who whom this that these "
            "those am is are was were be been being have has had having do does did doing a an the and but if or "
            "because as until while of at by for with about against between into through during before after "
            "above below to from up down in out on off over under again further then once here there when where "
            "why how all any both each few more most other some such no nor not only own same so than too very s "
            "t can will just don should now i'll you'll he'll she'll we'll they'll i'd you'd he'd she'd we'd "
            "they'd i'm you're he's she's it's we're they're i've we've you've they've isn't aren't wasn't "
            "weren't haven't hasn't hadn't don't doesn't didn't won't wouldn't shan't shouldn't mustn't can't "
            "couldn't cannot could here's how's let's ought that's there's what's when's where's who's why's "
            "would").split()


@register("org.apache.spark.ml.feature.StopWordsRemover")
class StopWordsRemover(_Simple, HasInputCols, HasOutputCols):
    """A feature transformer that filters out stop words from input."""

    stopWords = shared("stopWords", "The words to be filtered out", TypeConverters.toListString)
    caseSensitive = shared("caseSensitive", "whether to do a case sensitive comparison over the stop words",
                           TypeConverters.toBoolean)
    locale = shared("locale", "locale of the input. ignored when case sensitive is true", TypeConverters.toString)

    @keyword_only
    def __init__(self, *, inputCol=None, outputCol=None, stopWords=None, caseSensitive=False, locale=None,
                 inputCols=None, outputCols=None):
        super().__init__()
        self._setDefault(stopWords=list(_EN_STOP), caseSensitive=False, locale="en_US")
        self._set(**self._input_kwargs)

    @staticmethod
    def loadDefaultStopWords(language="english"):
        return list(_EN_STOP)

    def _apply(self, df, name):
        cs = self.getOrDefault(self.caseSensitive)
        sw = set(self.getOrDefault(self.stopWords)) if cs else {w.lower() for w in self.getOrDefault(self.stopWords)}
        vals = df.column_data(name).values
        return C.ArrayColumn([None if v is None else [t for t in v if (t if cs else t.lower()) not in sw] for v in vals])


@register("org.apache.spark.ml.feature.NGram")
class NGram(_Simple):
    """A feature transformer that converts the input array of strings into an array of n-grams."""

    n = shared("n", "number of elements per n-gram (>=1)", TypeConverters.toInt)

    @keyword_only
    def __init__(self, *, n=2, inputCol=None, outputCol=None):
        super().__init__()
        self._setDefault(n=2)
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        k = self.getOrDefault(self.n)
        vals = df.column_data(name).values
        return C.ArrayColumn([None if v is None else [" ".join(v[i:i + k]) for i in range(len(v) - k + 1)]
                              for v in vals])


def _terms_to_csr(rows_terms: list, num_features: int, device, binary: bool) -> C.SparseVectorColumn:
    flat = [t for ts in rows_terms for t in (ts or [])]
    counts = [len(ts or []) for ts in rows_terms]
    n = len(rows_terms)
    dev = torch.device(device)
    _, bucket = TX.murmur3_buckets(flat, num_features, dev)
    return _buckets_to_csr(bucket.to(dev), torch.tensor(counts, device=dev), n, num_features, binary)


def _buckets_to_csr(bucket: torch.Tensor, counts: torch.Tensor, n: int, num_features: int,
                    binary: bool) -> C.SparseVectorColumn:
    """Per-row term buckets (row-major, ``counts`` per row) -> CSR term frequencies."""
    dev = bucket.device
    row = torch.repeat_interleave(torch.arange(n, device=dev), counts.to(dev))
    key = row * num_features + bucket
    uk, cnt = torch.unique(key, return_counts=True)         # sorted by (row, bucket)
    r = uk // num_features
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    indptr[1:] = torch.cumsum(torch.bincount(r, minlength=n), 0)
    vals = torch.ones_like(cnt, dtype=torch.float64) if binary else cnt.to(torch.float64)
    return C.SparseVectorColumn(indptr, (uk % num_features).to(torch.int32), vals, num_features)


@register("org.apache.spark.ml.feature.HashingTF")
class HashingTF(_Simple, HasNumFeatures):
    """Maps a sequence of terms to their term frequencies using the hashing trick
    (MurmurHash3_x86_32, seed 42, nonNegativeMod -- Spark's exact bucket assignment;
    hashed on the GPU by the murmur3 HIP kernel)."""

    binary = shared("binary", "If True, all non zero counts are set to 1. This is useful for discrete probabilistic "
                              "models that model binary events rather than integer counts. Default False.",
                    TypeConverters.toBoolean)

    @keyword_only
    def __init__(self, *, numFeatures=1 << 18, binary=False, inputCol=None, outputCol=None):
        super().__init__()
        self._setDefault(numFeatures=1 << 18, binary=False)
        self._set(**self._input_kwargs)

    def indexOf(self, term):
        _, b = TX.murmur3_buckets([str(term)], self.getOrDefault(self.numFeatures))
        return int(b[0])

    def _apply(self, df, name):
        col = df.column_data(name)
        nf = self.getOrDefault(self.numFeatures)
        if isinstance(col, C.DeviceTokensColumn) and col.data.is_cuda:
            # device tokens: hash the spans in place and count per document, one wave per
            # row (hashing_tf_*_kernel) -> CSR on device, no global sort
            indptr, idx, val = TX.hashing_tf_csr(col, nf, self.getOrDefault(self.binary))
            return C.SparseVectorColumn(indptr, idx, val, nf)
        vals = col.values
        return _terms_to_csr([None if v is None else [str(t) for t in v] for v in vals],
                             nf, df.device, self.getOrDefault(self.binary))


@register("org.apache.spark.ml.feature.FeatureHasher")
class FeatureHasher(Transformer, HasInputCols, HasOutputCol, HasNumFeatures, MLWritable, MLReadable):
    """Feature hashing of numeric/categorical columns (Spark FeatureHasher semantics: numeric
    -> hash(name) with value, string -> hash(name=value) with 1.0)."""

    categoricalCols = shared("categoricalCols", "numeric columns to treat as categorical",
                             TypeConverters.toListString)

    @keyword_only
    def __init__(self, *, numFeatures=1 << 18, inputCols=None, outputCol=None, categoricalCols=None):
        super().__init__()
        self._setDefault(numFeatures=1 << 18, categoricalCols=[])
        self._set(**self._input_kwargs)

    def _transform(self, df):
        nf = self.getOrDefault(self.numFeatures)
        cat = set(self.getOrDefault(self.categoricalCols))
        n = len(df)
        rows_idx, rows_val = [[] for _ in range(n)], [[] for _ in range(n)]
        for name in self.getOrDefault(self.inputCols):
            c = df.column_data(name)
            if isinstance(c, C.NumericColumn) and name not in cat:
                if isinstance(c.dtype, type(C.T.BooleanType())):
                    vals = c.to_pylist()
                    terms = [f"{name}={str(bool(v)).lower()}" for v in vals]
                    _, b = TX.murmur3_buckets(terms, nf)
                    for i in range(n):
                        rows_idx[i].append(int(b[i]))
                        rows_val[i].append(1.0)
                    continue
                _, b = TX.murmur3_buckets([name], nf)
                vals = c.data.to(torch.float64).cpu().numpy()
                for i in range(n):
                    if vals[i] != 0:
                        rows_idx[i].append(int(b[0]))
                        rows_val[i].append(float(vals[i]))
            else:
                vals = _strings(df, name)
                terms = [f"{name}={v}" for v in vals]
                _, b = TX.murmur3_buckets(terms, nf)
                for i in range(n):
                    if vals[i] is not None:
                        rows_idx[i].append(int(b[i]))
                        rows_val[i].append(1.0)
        ptr, ind, val = [0], [], []
        for ii, vv in zip(rows_idx, rows_val):
            acc = OrderedDict()
            for a, b in zip(ii, vv):
                acc[a] = acc.get(a, 0.0) + b
            items = sorted(acc.items())
            ind += [a for a, _ in items]
            val += [b for _, b in items]
            ptr.append(len(ind))
        dev = df.device
        col = C.SparseVectorColumn(torch.tensor(ptr, dtype=torch.int64, device=dev),
                                   torch.tensor(ind, dtype=torch.int32, device=dev),
                                   torch.tensor(val, dtype=torch.float64, device=dev), nf)
        return df.withColumnData(self.getOrDefault(self.outputCol), col)


@register("org.apache.spark.ml.feature.CountVectorizer")
class CountVectorizer(Estimator, _InOut, MLWritable, MLReadable):
    """Extracts a vocabulary from document collections and generates a CountVectorizerModel."""

    minTF = shared("minTF", "Filter to ignore rare words in a document. For each document, terms with frequency/"
                            "count less than the given threshold are ignored.", TypeConverters.toFloat)
    minDF = shared("minDF", "Specifies the minimum number of different documents a term must appear in to be "
                            "included in the vocabulary.", TypeConverters.toFloat)
    maxDF = shared("maxDF", "Specifies the maximum number of different documents a term could appear in to be "
                            "included in the vocabulary.", TypeConverters.toFloat)
    vocabSize = shared("vocabSize", "max size of the vocabulary. Default 1 << 18.", TypeConverters.toInt)
    binary = shared("binary", "Binary toggle to control the output vector values.", TypeConverters.toBoolean)

    @keyword_only
    def __init__(self, *, minTF=1.0, minDF=1.0, maxDF=2 ** 63 - 1, vocabSize=1 << 18, binary=False, inputCol=None,
                 outputCol=None):
        super().__init__()
        self._setDefault(minTF=1.0, minDF=1.0, maxDF=float(2 ** 63 - 1), vocabSize=1 << 18, binary=False)
        self._set(**self._input_kwargs)

    def _fit(self, df):
        docs = df.column_data(self.getOrDefault(self.inputCol)).values
        tf, dfc = Counter(), Counter()
        for d in docs:
            if d is None:
                continue
            tf.update(d)
            dfc.update(set(d))
        parts = df.comm.all_gather_object((tf, dfc, len(docs)))
        tf, dfc, ndocs = Counter(), Counter(), 0
        for a, b, c in parts:
            tf.update(a)
            dfc.update(b)
            ndocs += c
        mindf, maxdf = self.getOrDefault(self.minDF), self.getOrDefault(self.maxDF)
        mind = mindf if mindf >= 1 else mindf * ndocs
        maxd = maxdf if maxdf >= 1 else maxdf * ndocs
        terms = [t for t in tf if mind <= dfc[t] <= maxd]
        terms.sort(key=lambda t: (-tf[t], t))
        vocab = terms[: self.getOrDefault(self.vocabSize)]
        return CountVectorizerModel._from(vocab)._with_parent(self)


@register("org.apache.spark.ml.feature.CountVectorizerModel")
class CountVectorizerModel(Model, _InOut, MLWritable, MLReadable):
    minTF = CountVectorizer.minTF
    binary = CountVectorizer.binary

    def __init__(self):
        super().__init__()
        self._setDefault(minTF=1.0, binary=False)
        self.vocabulary = []

    @classmethod
    def _from(cls, vocab):
        m = cls()
        m.vocabulary = list(vocab)
        return m

    @classmethod
    def from_vocabulary(cls, vocabulary, inputCol, outputCol=None, minTF=None, binary=None):
        m = cls._from(vocabulary)
        m._set(inputCol=inputCol, outputCol=outputCol, minTF=minTF, binary=binary)
        return m

    def _transform(self, df):
        idx = {t: i for i, t in enumerate(self.vocabulary)}
        docs = df.column_data(self.getOrDefault(self.inputCol)).values
        mintf, binary = self.getOrDefault(self.minTF), self.getOrDefault(self.binary)
        ptr, ind, val = [0], [], []
        for d in docs:
            cnt = Counter(t for t in (d or []) if t in idx)
            thr = mintf if mintf >= 1 else mintf * max(len(d or []), 1)
            items = sorted((idx[t], c) for t, c in cnt.items() if c >= thr)
            ind += [a for a, _ in items]
            val += [1.0 if binary else float(c) for _, c in items]
            ptr.append(len(ind))
        dev = df.device
        col = C.SparseVectorColumn(torch.tensor(ptr, dtype=torch.int64, device=dev),
                                   torch.tensor(ind, dtype=torch.int32, device=dev),
                                   torch.tensor(val, dtype=torch.float64, device=dev), len(self.vocabulary))
        return df.withColumnData(self.getOrDefault(self.outputCol), col)

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"vocabulary": pa.array([self.vocabulary], type=pa.list_(pa.string()))})

    @classmethod
    def _load_impl(cls, path, meta):
        m = cls._from(read_data(path).to_pylist()[0]["vocabulary"])
        apply_metadata(m, meta)
        return m


@register("org.apache.spark.ml.feature.IDF")
class IDF(Estimator, _InOut, MLWritable, MLReadable):
    """Compute the Inverse Document Frequency (IDF) given a collection of documents."""

    minDocFreq = shared("minDocFreq", "minimum number of documents in which a term should appear for filtering",
                        TypeConverters.toInt)

    @keyword_only
    def __init__(self, *, minDocFreq=0, inputCol=None, outputCol=None):
        super().__init__()
        self._setDefault(minDocFreq=0)
        self._set(**self._input_kwargs)

    def _fit(self, df):
        c = df.column_data(self.getOrDefault(self.inputCol))
        if isinstance(c, C.SparseVectorColumn):
            d = c.size
            dfreq = torch.zeros(d, dtype=torch.float64, device=c.values.device).index_add_(
                0, c.indices.long(), (c.values != 0).to(torch.float64))
        else:
            X = _vec(df, self.getOrDefault(self.inputCol))
            d = X.shape[1]
            dfreq = (X != 0).sum(0).to(torch.float64)
        m = torch.tensor([float(len(df))], dtype=torch.float64, device=dfreq.device)
        buf = torch.cat([dfreq, m])
        df.comm.all_reduce(buf)
        dfreq, m = buf[:d], buf[d]
        idf = torch.log((m + 1.0) / (dfreq + 1.0))
        idf = torch.where(dfreq >= self.getOrDefault(self.minDocFreq), idf, torch.zeros_like(idf))
        return IDFModel._from(idf.cpu().numpy(), dfreq.cpu().numpy(), int(m))._with_parent(self)


@register("org.apache.spark.ml.feature.IDFModel")
class IDFModel(Model, _InOut, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self._idf = np.zeros(0)
        self.docFreq = []
        self.numDocs = 0

    @classmethod
    def _from(cls, idf, dfreq, m):
        x = cls()
        x._idf, x.docFreq, x.numDocs = np.asarray(idf), [int(v) for v in dfreq], m
        return x

    @property
    def idf(self):
        return DenseVector(self._idf)

    def _transform(self, df):
        c = df.column_data(self.getOrDefault(self.inputCol))
        w = torch.from_numpy(self._idf)
        if isinstance(c, C.SparseVectorColumn):
            out = C.SparseVectorColumn(c.indptr, c.indices, c.values.to(torch.float64) *
                                       w.to(c.values.device)[c.indices.long()], c.size)
        else:
            out = C.VectorColumn(_vec(df, self.getOrDefault(self.inputCol)) * w.to(df.device)[None, :])
        return df.withColumnData(self.getOrDefault(self.outputCol), out)

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"idf": vec_col([self.idf]), "docFreq": pa.array([self.docFreq], prim_list(pa.int64())),
                          "numDocs": pa.array([self.numDocs], pa.int64())})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls._from(vector_from_struct(t["idf"]).toArray(), t["docFreq"], t["numDocs"])
        apply_metadata(m, meta)
        return m


# ============================================================================ scalers
def _col_moments(df, X):
    """Column summary (mean, unbiased std, min, max, max |x|) of the vector column named
    ``X`` (or of the matrix ``X``), reduced over ranks.  An out-of-core (spilled) column is
    summarised block by block (frame/spill.py ``block_moments``)."""
    if isinstance(X, str):
        c = df.column_data(X)
        if isinstance(c, SpilledVectorColumn):
            s_, ss_, n_, mx_, lo_, hi_ = block_moments(c)
            dev = s_.device
            st = torch.cat([s_, ss_, torch.tensor([n_], dtype=torch.float64, device=dev)])
            d = s_.numel()
            df.comm.all_reduce(st)
            mx = mx_.contiguous()
            df.comm.all_reduce(mx, "max")
            mins, maxs = lo_.contiguous(), hi_.contiguous()
            df.comm.all_reduce(mins, "min")
            df.comm.all_reduce(maxs, "max")
            return _finish_moments(st[:d], st[d:2 * d], st[2 * d], mins, maxs, mx)
        X = _vec(df, X)
    n = torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device)
    st = torch.cat([X.sum(0), (X * X).sum(0), n,
                    torch.where(torch.isfinite(X), X, torch.zeros_like(X)).abs().max(0).values if X.shape[0]
                    else torch.zeros(X.shape[1], dtype=X.dtype, device=X.device)])
    d = X.shape[1]
    df.comm.all_reduce(st[: 2 * d + 1])
    mx = st[2 * d + 1:].contiguous()
    df.comm.all_reduce(mx, "max")
    mins = X.min(0).values if X.shape[0] else torch.full((d,), math.inf, dtype=X.dtype, device=X.device)
    maxs = X.max(0).values if X.shape[0] else torch.full((d,), -math.inf, dtype=X.dtype, device=X.device)
    mins, maxs = mins.contiguous(), maxs.contiguous()
    df.comm.all_reduce(mins, "min")
    df.comm.all_reduce(maxs, "max")
    return _finish_moments(st[:d], st[d:2 * d], st[2 * d], mins, maxs, mx)


def _finish_moments(s, ss, m, mins, maxs, mx):
    mean = s / m
    var = ((ss - m * mean * mean) / (m - 1)).clamp_min(0) if m > 1 else torch.zeros_like(mean)
    return mean, var.sqrt(), mins, maxs, mx


def _rowwise(df, in_name, out_name, fn):
    """``df`` with ``out_name`` = the row-wise fp64 map ``fn`` of vector column ``in_name``.
    An out-of-core (spilled) input maps block by block into a spilled output of the same
    resident / host split and dtype (frame/spill.py ``map_blocks``); otherwise fp64 rows,
    as Spark's double vectors."""
    c = df.column_data(in_name)
    if isinstance(c, SpilledVectorColumn):
        return df.withColumnData(out_name, map_blocks(c, fn))
    return df.withColumnData(out_name, C.VectorColumn(fn(_vec(df, in_name).to(df.device))))


class _ScalerModelBase(Model, _InOut, MLWritable, MLReadable):
    _fields: tuple = ()

    def _save_data(self, path):
        write_data(path, {k: vec_col([DenseVector(getattr(self, "_" + k))]) for k in self._fields})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls()
        for k in cls._fields:
            setattr(m, "_" + k, vector_from_struct(t[k]).toArray())
        apply_metadata(m, meta)
        return m


@register("org.apache.spark.ml.feature.StandardScaler")
class StandardScaler(Estimator, _InOut, MLWritable, MLReadable):
    """Standardizes features by removing the mean and scaling to unit variance using column
    summary statistics on the samples in the training set (unbiased sample std, as Spark)."""

    withMean = shared("withMean", "Center data with mean", TypeConverters.toBoolean)
    withStd = shared("withStd", "Scale to unit standard deviation", TypeConverters.toBoolean)

    @keyword_only
    def __init__(self, *, withMean=False, withStd=True, inputCol=None, outputCol=None):
        super().__init__()
        self._setDefault(withMean=False, withStd=True)
        self._set(**self._input_kwargs)

    def _fit(self, df):
        mean, std, *_ = _col_moments(df, self.getOrDefault(self.inputCol))
        m = StandardScalerModel()
        m._mean, m._std = mean.cpu().numpy(), std.cpu().numpy()
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.StandardScalerModel")
class StandardScalerModel(_ScalerModelBase):
    withMean = StandardScaler.withMean
    withStd = StandardScaler.withStd
    _fields = ("std", "mean")

    @property
    def mean(self):
        return DenseVector(self._mean)

    @property
    def std(self):
        return DenseVector(self._std)

    def _transform(self, df):
        mean = torch.from_numpy(self._mean).to(df.device)
        s = torch.from_numpy(self._std).to(df.device)
        with_mean, with_std = self.getOrDefault(self.withMean), self.getOrDefault(self.withStd)

        def f(X):
            if with_mean:
                X = X - mean
            if with_std:
                X = torch.where(s > 0, X / torch.where(s > 0, s, torch.ones_like(s)), torch.zeros_like(X))
            return X
        return _rowwise(df, self.getOrDefault(self.inputCol), self.getOrDefault(self.outputCol), f)


@register("org.apache.spark.ml.feature.MinMaxScaler")
class MinMaxScaler(Estimator, _InOut, MLWritable, MLReadable):
    """Rescale each feature individually to a common range [min, max] linearly using column summary statistics."""

    min = shared("min", "Lower bound of the output feature range", TypeConverters.toFloat)
    max = shared("max", "Upper bound of the output feature range", TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, min=0.0, max=1.0, inputCol=None, outputCol=None):  # noqa: A002
        super().__init__()
        self._setDefault(min=0.0, max=1.0)
        self._set(**self._input_kwargs)

    def _fit(self, df):
        _, _, mins, maxs, _ = _col_moments(df, self.getOrDefault(self.inputCol))
        m = MinMaxScalerModel()
        m._originalMin, m._originalMax = mins.cpu().numpy(), maxs.cpu().numpy()
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.MinMaxScalerModel")
class MinMaxScalerModel(_ScalerModelBase):
    min = MinMaxScaler.min
    max = MinMaxScaler.max
    _fields = ("originalMin", "originalMax")

    @property
    def originalMin(self):
        return DenseVector(self._originalMin)

    @property
    def originalMax(self):
        return DenseVector(self._originalMax)

    def _transform(self, df):
        lo = torch.from_numpy(self._originalMin).to(df.device)
        rng = torch.from_numpy(self._originalMax - self._originalMin).to(df.device)
        a, b = self.getOrDefault(self.min), self.getOrDefault(self.max)

        def f(X):
            scaled = torch.where(rng != 0, (X - lo) / torch.where(rng != 0, rng, torch.ones_like(rng)),
                                 torch.full_like(X, 0.5))
            return scaled * (b - a) + a
        return _rowwise(df, self.getOrDefault(self.inputCol), self.getOrDefault(self.outputCol), f)


@register("org.apache.spark.ml.feature.MaxAbsScaler")
class MaxAbsScaler(Estimator, _InOut, MLWritable, MLReadable):
    """Rescale each feature individually to range [-1, 1] by dividing through the largest maximum absolute value."""

    @keyword_only
    def __init__(self, *, inputCol=None, outputCol=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        *_, mx = _col_moments(df, self.getOrDefault(self.inputCol))
        m = MaxAbsScalerModel()
        m._maxAbs = mx.cpu().numpy()
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.MaxAbsScalerModel")
class MaxAbsScalerModel(_ScalerModelBase):
    _fields = ("maxAbs",)

    @property
    def maxAbs(self):
        return DenseVector(self._maxAbs)

    def _transform(self, df):
        m = torch.from_numpy(self._maxAbs).to(df.device)
        return _rowwise(df, self.getOrDefault(self.inputCol), self.getOrDefault(self.outputCol),
                        lambda X: torch.where(m > 0, X / torch.where(m > 0, m, torch.ones_like(m)), X))


@register("org.apache.spark.ml.feature.RobustScaler")
class RobustScaler(Estimator, _InOut, MLWritable, MLReadable):
    """Removes the median and scales the data according to the quantile range."""

    lower = shared("lower", "Lower quantile to calculate quantile range", TypeConverters.toFloat)
    upper = shared("upper", "Upper quantile to calculate quantile range", TypeConverters.toFloat)
    withCentering = shared("withCentering", "Whether to center data with median", TypeConverters.toBoolean)
    withScaling = shared("withScaling", "Whether to scale the data to quantile range", TypeConverters.toBoolean)
    relativeError = shared("relativeError", "The target relative error for quantile computation",
                           TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, lower=0.25, upper=0.75, withCentering=False, withScaling=True, inputCol=None,
                 outputCol=None, relativeError=0.001):
        super().__init__()
        self._setDefault(lower=0.25, upper=0.75, withCentering=False, withScaling=True, relativeError=0.001)
        self._set(**self._input_kwargs)

    def _fit(self, df):
        X = _vec(df, self.getOrDefault(self.inputCol))
        X = df.comm.all_gather_v(X) if df.comm.world_size > 1 else X
        q = torch.quantile(X, torch.tensor([self.getOrDefault(self.lower), 0.5, self.getOrDefault(self.upper)],
                                           dtype=X.dtype, device=X.device), dim=0)
        m = RobustScalerModel()
        m._median, m._range = q[1].cpu().numpy(), (q[2] - q[0]).cpu().numpy()
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.RobustScalerModel")
class RobustScalerModel(_ScalerModelBase):
    withCentering = RobustScaler.withCentering
    withScaling = RobustScaler.withScaling
    _fields = ("range", "median")

    @property
    def median(self):
        return DenseVector(self._median)

    @property
    def range(self):
        return DenseVector(self._range)

    def _transform(self, df):
        X = _vec(df, self.getOrDefault(self.inputCol))
        if self.getOrDefault(self.withCentering):
            X = X - torch.from_numpy(self._median).to(X.device)
        if self.getOrDefault(self.withScaling):
            r = torch.from_numpy(self._range).to(X.device)
            X = torch.where(r > 0, X / torch.where(r > 0, r, torch.ones_like(r)), torch.zeros_like(X))
        return df.withColumnData(self.getOrDefault(self.outputCol), C.VectorColumn(X))


# ============================================================================ categorical
@register("org.apache.spark.ml.feature.StringIndexer")
class StringIndexer(Estimator, _InOut, HasInputCols, HasOutputCols, HasHandleInvalid, MLWritable, MLReadable):
    """A label indexer that maps a string column of labels to an ML column of label indices
    (frequencyDesc ordering by default, ties broken alphabetically, as Spark)."""

    stringOrderType = shared("stringOrderType", "How to order labels of string column. The first label after "
                             "ordering is assigned an index of 0. Supported options: frequencyDesc, frequencyAsc, "
                             "alphabetDesc, alphabetAsc.", TypeConverters.toString)

    @keyword_only
    def __init__(self, *, inputCol=None, outputCol=None, inputCols=None, outputCols=None, handleInvalid="error",
                 stringOrderType="frequencyDesc"):
        super().__init__()
        self._setDefault(handleInvalid="error", stringOrderType="frequencyDesc")
        self._set(**self._input_kwargs)

    def _cols(self):
        if self.isSet(self.inputCols):
            return list(self.getOrDefault(self.inputCols)), list(self.getOrDefault(self.outputCols))
        return [self.getOrDefault(self.inputCol)], [self.getOrDefault(self.outputCol)]

    def _fit(self, df):
        ins, _ = self._cols()
        labels = []
        for name in ins:
            cnt = _value_counts(df, name)
            total = Counter()
            for part in df.comm.all_gather_object(cnt):
                total.update(part)
            o = self.getOrDefault(self.stringOrderType)
            keys = list(total)
            if o == "frequencyDesc":
                keys.sort(key=lambda k: (-total[k], k))
            elif o == "frequencyAsc":
                keys.sort(key=lambda k: (total[k], k))
            elif o == "alphabetDesc":
                keys.sort(reverse=True)
            else:
                keys.sort()
            labels.append(keys)
        return StringIndexerModel._from(labels)._with_parent(self)


@register("org.apache.spark.ml.feature.StringIndexerModel")
class StringIndexerModel(Model, _InOut, HasInputCols, HasOutputCols, HasHandleInvalid, MLWritable, MLReadable):
    stringOrderType = StringIndexer.stringOrderType

    def __init__(self):
        super().__init__()
        self._setDefault(handleInvalid="error")
        self.labelsArray = []

    @classmethod
    def _from(cls, labels_array):
        m = cls()
        m.labelsArray = [list(l) for l in labels_array]
        return m

    @classmethod
    def from_labels(cls, labels, inputCol, outputCol=None, handleInvalid=None):
        m = cls._from([labels])
        m._set(inputCol=inputCol, outputCol=outputCol, handleInvalid=handleInvalid)
        return m

    @property
    def labels(self):
        return self.labelsArray[0]

    def _transform(self, df):
        if self.isSet(self.inputCols):
            ins, outs = list(self.getOrDefault(self.inputCols)), list(self.getOrDefault(self.outputCols))
        else:
            ins, outs = [self.getOrDefault(self.inputCol)], [self.getOrDefault(self.outputCol)]
        hi = self.getOrDefault(self.handleInvalid)
        keep = torch.ones(len(df), dtype=torch.bool)
        cols = []
        for name, out, labels in zip(ins, outs, self.labelsArray):
            idx = {l: i for i, l in enumerate(labels)}
            res, first_bad = _index_values(df, name, idx)        # NaN = null or unseen
            bad = np.isnan(res)
            if bad.any():
                if hi == "keep":
                    res[bad] = len(labels)
                elif hi == "skip":
                    keep &= torch.from_numpy(~bad)
                else:
                    raise ValueError(f"Unseen label: {first_bad}. To handle unseen labels, set Param handleInvalid "
                                     f"to keep.")
            cols.append((out, torch.from_numpy(res)))
        for out, t in cols:
            df = df.withColumnData(out, C.NumericColumn(t.to(df.device)))
        return df._mask(keep) if not bool(keep.all()) else df

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"labelsArray": pa.array([self.labelsArray], type=pa.list_(pa.list_(pa.string())))})

    @classmethod
    def _load_impl(cls, path, meta):
        m = cls._from(read_data(path).to_pylist()[0]["labelsArray"])
        apply_metadata(m, meta)
        return m


@register("org.apache.spark.ml.feature.IndexToString")
class IndexToString(_Simple):
    """A Transformer that maps a column of indices back to a new column of corresponding string values."""

    labels = shared("labels", "Optional array of labels specifying index-string mapping. If not provided or if "
                              "empty, then metadata from inputCol is used instead.", TypeConverters.toListString)

    @keyword_only
    def __init__(self, *, inputCol=None, outputCol=None, labels=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _apply(self, df, name):
        labels = self.getOrDefault(self.labels)
        vals = df.column_data(name).data.cpu().numpy()
        return C.StringColumn(np.array([labels[int(v)] for v in vals], dtype=object))


@register("org.apache.spark.ml.feature.OneHotEncoder")
class OneHotEncoder(Estimator, HasInputCol, HasOutputCol, HasInputCols, HasOutputCols, HasHandleInvalid,
                    MLWritable, MLReadable):
    """Maps a column of category indices to a column of binary vectors (dropLast by default)."""

    dropLast = shared("dropLast", "whether to drop the last category", TypeConverters.toBoolean)

    @keyword_only
    def __init__(self, *, inputCols=None, outputCols=None, handleInvalid="error", dropLast=True, inputCol=None,
                 outputCol=None):
        super().__init__()
        self._setDefault(handleInvalid="error", dropLast=True)
        self._set(**self._input_kwargs)

    def _io(self):
        if self.isSet(self.inputCols):
            return list(self.getOrDefault(self.inputCols)), list(self.getOrDefault(self.outputCols))
        return [self.getOrDefault(self.inputCol)], [self.getOrDefault(self.outputCol)]

    def _fit(self, df):
        ins, _ = self._io()
        sizes = []
        for name in ins:
            mx = df.comm.max_scalar(float(df.column_data(name).data.max().item()) if len(df) else 0.0)
            sizes.append(int(mx) + 1)
        m = OneHotEncoderModel()
        m.categorySizes = sizes
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.OneHotEncoderModel")
class OneHotEncoderModel(Model, HasInputCol, HasOutputCol, HasInputCols, HasOutputCols, HasHandleInvalid,
                         MLWritable, MLReadable):
    dropLast = OneHotEncoder.dropLast

    def __init__(self):
        super().__init__()
        self._setDefault(handleInvalid="error", dropLast=True)
        self.categorySizes = []

    def _transform(self, df):
        if self.isSet(self.inputCols):
            ins, outs = list(self.getOrDefault(self.inputCols)), list(self.getOrDefault(self.outputCols))
        else:
            ins, outs = [self.getOrDefault(self.inputCol)], [self.getOrDefault(self.outputCol)]
        keep_invalid = self.getOrDefault(self.handleInvalid) == "keep"
        for name, out, k in zip(ins, outs, self.categorySizes):
            v = df.column_data(name).data.long()
            size = k + (1 if keep_invalid else 0) - (1 if self.getOrDefault(self.dropLast) else 0)
            bad = (v < 0) | (v >= k)
            if bool(bad.any()) and not keep_invalid:
                raise ValueError("OneHotEncoder: invalid category index (handleInvalid='error')")
            v = torch.where(bad, torch.full_like(v, k), v)
            hit = v < size
            n = v.numel()
            ptr = torch.zeros(n + 1, dtype=torch.int64, device=v.device)
            ptr[1:] = torch.cumsum(hit.long(), 0)
            col = C.SparseVectorColumn(ptr, v[hit].to(torch.int32), torch.ones(int(hit.sum()), dtype=torch.float64,
                                                                                device=v.device), size)
            df = df.withColumnData(out, col)
        return df

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"categorySizes": pa.array([self.categorySizes], prim_list(pa.int32()))})

    @classmethod
    def _load_impl(cls, path, meta):
        m = cls()
        m.categorySizes = read_data(path).to_pylist()[0]["categorySizes"]
        apply_metadata(m, meta)
        return m


@register("org.apache.spark.ml.feature.VectorIndexer")
class VectorIndexer(Estimator, _InOut, HasHandleInvalid, MLWritable, MLReadable):
    """Class for indexing categorical feature columns in a dataset of Vector."""

    maxCategories = shared("maxCategories", "Threshold for the number of values a categorical feature can take "
                           "(>= 2). If a feature is found to have > maxCategories values, then it is declared "
                           "continuous.", TypeConverters.toInt)

    @keyword_only
    def __init__(self, *, maxCategories=20, inputCol=None, outputCol=None, handleInvalid="error"):
        super().__init__()
        self._setDefault(maxCategories=20, handleInvalid="error")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        X = _vec(df, self.getOrDefault(self.inputCol))
        X = df.comm.all_gather_v(X) if df.comm.world_size > 1 else X
        maps = {}
        for j in range(X.shape[1]):
            u = torch.unique(X[:, j])
            if u.numel() <= self.getOrDefault(self.maxCategories):
                vals = sorted(u.tolist())
                if 0.0 in vals:
                    vals.remove(0.0)
                    vals = [0.0] + vals
                maps[j] = {v: i for i, v in enumerate(vals)}
        m = VectorIndexerModel()
        m.categoryMaps, m.numFeatures = maps, X.shape[1]
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.VectorIndexerModel")
class VectorIndexerModel(Model, _InOut, HasHandleInvalid, MLWritable, MLReadable):
    maxCategories = VectorIndexer.maxCategories

    def __init__(self):
        super().__init__()
        self.categoryMaps, self.numFeatures = {}, 0

    def _transform(self, df):
        X = _vec(df, self.getOrDefault(self.inputCol)).clone()
        for j, mp in self.categoryMaps.items():
            col = X[:, j]
            out = torch.full_like(col, float(len(mp)))
            for v, i in mp.items():
                out = torch.where(col == v, torch.full_like(col, float(i)), out)
            X[:, j] = out
        return df.withColumnData(self.getOrDefault(self.outputCol), C.VectorColumn(X))


@register("org.apache.spark.ml.feature.QuantileDiscretizer")
class QuantileDiscretizer(Estimator, _InOut, HasHandleInvalid, MLWritable, MLReadable):
    """Takes a column with continuous features and outputs a column with binned categorical features."""

    numBuckets = shared("numBuckets", "Maximum number of buckets (quantiles, or categories) into which data "
                                      "points are grouped. Must be >= 2.", TypeConverters.toInt)
    relativeError = shared("relativeError", "The relative target precision for the approximate quantile "
                                            "algorithm used to generate buckets. Must be in the range [0, 1].",
                           TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, numBuckets=2, inputCol=None, outputCol=None, relativeError=0.001, handleInvalid="error"):
        super().__init__()
        self._setDefault(numBuckets=2, relativeError=0.001, handleInvalid="error")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        x = df.column_data(self.getOrDefault(self.inputCol)).data.to(torch.float64)
        x = df.comm.all_gather_v(x) if df.comm.world_size > 1 else x
        x = x[~torch.isnan(x)]
        k = self.getOrDefault(self.numBuckets)
        q = torch.quantile(x, torch.linspace(0, 1, k + 1, dtype=torch.float64, device=x.device)[1:-1]).cpu().numpy()
        splits = [-math.inf] + sorted(set(q.tolist())) + [math.inf]
        return Bucketizer(splits=splits, inputCol=self.getOrDefault(self.inputCol),
                          outputCol=self.getOrDefault(self.outputCol), handleInvalid=self.getOrDefault(self.handleInvalid))


@register("org.apache.spark.ml.feature.Imputer")
class Imputer(Estimator, HasInputCols, HasOutputCols, HasInputCol, HasOutputCol, MLWritable, MLReadable):
    """Imputation estimator for completing missing values (mean, median or mode)."""

    strategy = shared("strategy", "strategy for imputation. If mean, then replace missing values using the mean "
                                  "value of the feature. If median, then replace missing values using the median "
                                  "value of the feature. If mode, then replace missing using the most frequent value "
                                  "of the feature.", TypeConverters.toString)
    missingValue = shared("missingValue", "The placeholder for the missing values. All occurrences of missingValue "
                                          "will be imputed.", TypeConverters.toFloat)
    relativeError = shared("relativeError", "the relative target precision for the approximate quantile algorithm. "
                                            "Must be in the range [0, 1]", TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, strategy="mean", missingValue=float("nan"), inputCols=None, outputCols=None, inputCol=None,
                 outputCol=None, relativeError=0.001):
        super().__init__()
        self._setDefault(strategy="mean", missingValue=float("nan"), relativeError=0.001)
        self._set(**self._input_kwargs)

    def _io(self):
        if self.isSet(self.inputCols):
            return list(self.getOrDefault(self.inputCols)), list(self.getOrDefault(self.outputCols))
        return [self.getOrDefault(self.inputCol)], [self.getOrDefault(self.outputCol)]

    def _fit(self, df):
        ins, _ = self._io()
        mv = self.getOrDefault(self.missingValue)
        surrogates = {}
        for name in ins:
            c = df.column_data(name)
            x = c.data.to(torch.float64)
            miss = c.null_mask() | (torch.isnan(x) if math.isnan(mv) else (x == mv))
            v = x[~miss]
            v = df.comm.all_gather_v(v) if df.comm.world_size > 1 else v
            s = self.getOrDefault(self.strategy)
            if v.numel() == 0:
                raise ValueError(f"surrogate cannot be computed. All the values in {name} are Null, Nan or missingValue")
            if s == "mean":
                surrogates[name] = float(v.mean())
            elif s == "median":
                surrogates[name] = float(torch.quantile(v, 0.5, interpolation="lower"))
            else:
                u, cnt = torch.unique(v, return_counts=True)
                surrogates[name] = float(u[cnt.argmax()])
        m = ImputerModel()
        m.surrogates = surrogates
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.ImputerModel")
class ImputerModel(Model, HasInputCols, HasOutputCols, HasInputCol, HasOutputCol, MLWritable, MLReadable):
    strategy = Imputer.strategy
    missingValue = Imputer.missingValue

    def __init__(self):
        super().__init__()
        self._setDefault(missingValue=float("nan"))
        self.surrogates = {}

    @property
    def surrogateDF(self):
        from ..session import Session
        return Session.getOrCreate().createDataFrame([tuple(self.surrogates.values())], list(self.surrogates))

    def _transform(self, df):
        if self.isSet(self.inputCols):
            ins, outs = list(self.getOrDefault(self.inputCols)), list(self.getOrDefault(self.outputCols))
        else:
            ins, outs = [self.getOrDefault(self.inputCol)], [self.getOrDefault(self.outputCol)]
        mv = self.getOrDefault(self.missingValue)
        for name, out in zip(ins, outs):
            c = df.column_data(name)
            x = c.data.to(torch.float64)
            miss = c.null_mask() | (torch.isnan(x) if math.isnan(mv) else (x == mv))
            df = df.withColumnData(out, C.NumericColumn(torch.where(miss, torch.full_like(x, self.surrogates[name]), x)))
        return df

    def _save_data(self, path):
        write_data(path, {k: [v] for k, v in self.surrogates.items()})

    @classmethod
    def _load_impl(cls, path, meta):
        m = cls()
        m.surrogates = {k: v for k, v in read_data(path).to_pylist()[0].items()}
        apply_metadata(m, meta)
        return m


# ============================================================================ projection / selection
@register("org.apache.spark.ml.feature.PCA")
class PCA(Estimator, _InOut, MLWritable, MLReadable):
    """PCA trains a model to project vectors to a lower dimensional space of the top k principal
    components (covariance via one all-reduced Gram GEMM, eigendecomposition on device)."""

    k = shared("k", "the number of principal components", TypeConverters.toInt)

    @keyword_only
    def __init__(self, *, k=None, inputCol=None, outputCol=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        X = _vec(df, self.getOrDefault(self.inputCol))
        d = X.shape[1]
        from ..ops.gram import rows_t_matmul
        st = torch.cat([rows_t_matmul(X, X).reshape(-1), X.sum(0), torch.tensor([float(X.shape[0])], dtype=X.dtype,
                                                                                 device=X.device)])
        df.comm.all_reduce(st)
        G_, s, n = st[: d * d].reshape(d, d), st[d * d: d * d + d], st[-1]
        mean = s / n
        cov = (G_ - n * torch.outer(mean, mean)) / (n - 1)
        evals, evecs = torch.linalg.eigh(cov)
        order = torch.argsort(evals, descending=True)
        k = self.getOrDefault(self.k)
        pc = evecs[:, order[:k]]
        # sign convention: largest-|component| positive (deterministic)
        sign = torch.sign(pc[pc.abs().argmax(0), torch.arange(k)])
        pc = pc * torch.where(sign == 0, torch.ones_like(sign), sign)
        ev = evals[order]
        m = PCAModel()
        m._pc, m._ev = pc.cpu().numpy(), (ev[:k] / ev.clamp_min(0).sum()).cpu().numpy()
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.PCAModel")
class PCAModel(Model, _InOut, MLWritable, MLReadable):
    k = PCA.k

    def __init__(self):
        super().__init__()
        self._pc, self._ev = np.zeros((0, 0)), np.zeros(0)

    @property
    def pc(self):
        return DenseMatrix.from_array(self._pc)

    @property
    def explainedVariance(self):
        return DenseVector(self._ev)

    def _transform(self, df):
        X = _vec(df, self.getOrDefault(self.inputCol))
        return df.withColumnData(self.getOrDefault(self.outputCol),
                                 C.VectorColumn(X @ torch.from_numpy(self._pc).to(X.device)))

    def _save_data(self, path):
        from .util import mat_col
        write_data(path, {"pc": mat_col([self.pc]), "explainedVariance": vec_col([self.explainedVariance])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import matrix_from_struct, vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls()
        m._pc = matrix_from_struct(t["pc"]).toArray()
        m._ev = vector_from_struct(t["explainedVariance"]).toArray()
        apply_metadata(m, meta)
        return m


@register("org.apache.spark.ml.feature.VarianceThresholdSelector")
class VarianceThresholdSelector(Estimator, HasFeaturesCol, HasOutputCol, MLWritable, MLReadable):
    """Feature selector that removes all low-variance features."""

    varianceThreshold = shared("varianceThreshold", "Param for variance threshold. Features with a variance not "
                               "greater than this threshold will be removed. The default value is 0.0.",
                               TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, featuresCol="features", outputCol=None, varianceThreshold=0.0):
        super().__init__()
        self._setDefault(varianceThreshold=0.0, featuresCol="features")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        _, std, *_ = _col_moments(df, _vec(df, self.getOrDefault(self.featuresCol)))
        m = VarianceThresholdSelectorModel()
        m.selectedFeatures = [int(i) for i in torch.nonzero(std * std > self.getOrDefault(self.varianceThreshold)).
                              reshape(-1).tolist()]
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.VarianceThresholdSelectorModel")
class VarianceThresholdSelectorModel(_SelectorModel):
    varianceThreshold = VarianceThresholdSelector.varianceThreshold


@register("org.apache.spark.ml.feature.ChiSqSelector")
class ChiSqSelector(Estimator, HasFeaturesCol, HasOutputCol, HasLabelCol, MLWritable, MLReadable):
    """Chi-Squared feature selection, which selects categorical features to use for predicting a categorical label."""

    selectorType = shared("selectorType", "The selector type. Supported options: numTopFeatures (default), "
                          "percentile, fpr, fdr, fwe.", TypeConverters.toString)
    numTopFeatures = shared("numTopFeatures", "Number of features that selector will select, ordered by ascending "
                            "p-value. If the number of features is < numTopFeatures, then this will select all "
                            "features.", TypeConverters.toInt)
    percentile = shared("percentile", "Percentile of features that selector will select, ordered by ascending "
                                      "p-value.", TypeConverters.toFloat)
    fpr = shared("fpr", "The highest p-value for features to be kept.", TypeConverters.toFloat)
    fdr = shared("fdr", "The upper bound of the expected false discovery rate.", TypeConverters.toFloat)
    fwe = shared("fwe", "The upper bound of the expected family-wise error rate.", TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, numTopFeatures=50, featuresCol="features", outputCol=None, labelCol="label",
                 selectorType="numTopFeatures", percentile=0.1, fpr=0.05, fdr=0.05, fwe=0.05):
        super().__init__()
        self._setDefault(numTopFeatures=50, selectorType="numTopFeatures", percentile=0.1, fpr=0.05, fdr=0.05,
                         fwe=0.05, featuresCol="features", labelCol="label")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        from ..ml.stat import chi_square_pvalues
        X = _vec(df, self.getOrDefault(self.featuresCol))
        y = U.numeric_column(df, self.getOrDefault(self.labelCol))
        p = chi_square_pvalues(df.comm, X, y)
        order = np.argsort(p, kind="stable")
        t = self.getOrDefault(self.selectorType)
        F = len(p)
        if t == "numTopFeatures":
            sel = order[: self.getOrDefault(self.numTopFeatures)]
        elif t == "percentile":
            sel = order[: int(F * self.getOrDefault(self.percentile))]
        elif t == "fpr":
            sel = np.nonzero(p < self.getOrDefault(self.fpr))[0]
        elif t == "fdr":
            thr = self.getOrDefault(self.fdr)
            ps = p[order]
            ok = np.nonzero(ps <= thr * (np.arange(F) + 1) / F)[0]
            sel = order[: ok.max() + 1] if ok.size else np.array([], dtype=int)
        else:
            sel = np.nonzero(p < self.getOrDefault(self.fwe) / F)[0]
        m = ChiSqSelectorModel()
        m.selectedFeatures = sorted(int(i) for i in sel)
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.ChiSqSelectorModel")
class ChiSqSelectorModel(_SelectorModel):
    pass


# ============================================================================ LSH
class _LSHParams(_InOut, HasSeed):
    numHashTables = shared("numHashTables", "number of hash tables, where increasing number of hash tables lowers "
                                            "the false negative rate, and decreasing it improves the running "
                                            "performance.", TypeConverters.toInt)

    def __init__(self):
        super().__init__()
        self._setDefault(numHashTables=1, seed=0)


class _LSHModel(Model, _LSHParams, MLWritable, MLReadable):
    def _hash(self, X):
        raise NotImplementedError

    def _dist(self, A_, b):
        raise NotImplementedError

    def _transform(self, df):
        X = _vec(df, self.getOrDefault(self.inputCol))
        return df.withColumnData(self.getOrDefault(self.outputCol), C.VectorColumn(self._hash(X)))

    def approxNearestNeighbors(self, dataset, key, numNearestNeighbors, distCol="distCol"):
        X = _vec(dataset, self.getOrDefault(self.inputCol))
        k = torch.as_tensor(np.asarray(key.toArray() if hasattr(key, "toArray") else key), dtype=torch.float64,
                            device=X.device)
        d = self._dist(X, k)
        idx = torch.argsort(d)[:numNearestNeighbors]
        out = dataset._take(idx)
        return out.withColumnData(distCol, C.NumericColumn(d[idx]))

    def approxSimilarityJoin(self, datasetA, datasetB, threshold, distCol="distCol"):
        A_ = _vec(datasetA, self.getOrDefault(self.inputCol))
        B_ = _vec(datasetB, self.getOrDefault(self.inputCol))
        rows = []
        for i in range(A_.shape[0]):
            d = self._dist(B_, A_[i])
            for j in torch.nonzero(d < threshold).reshape(-1).tolist():
                rows.append((i, j, float(d[j])))
        import pandas as pd
        from ..session import Session
        return Session.getOrCreate().createDataFrame(pd.DataFrame(rows, columns=["idA", "idB", distCol]))


@register("org.apache.spark.ml.feature.BucketedRandomProjectionLSH")
class BucketedRandomProjectionLSH(Estimator, _LSHParams, MLWritable, MLReadable):
    """LSH class for Euclidean distance metrics."""

    bucketLength = shared("bucketLength", "the length of each hash bucket, a larger bucket lowers the false "
                                          "negative rate.", TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, inputCol=None, outputCol=None, seed=None, numHashTables=1, bucketLength=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        d = U.features_column(df, self.getOrDefault(self.inputCol)).size
        g = torch.Generator().manual_seed(self.getOrDefault(self.seed))
        R = torch.randn((self.getOrDefault(self.numHashTables), d), generator=g, dtype=torch.float64)
        R = R / R.norm(dim=1, keepdim=True)
        m = BucketedRandomProjectionLSHModel()
        m._R = R.numpy()
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.BucketedRandomProjectionLSHModel")
class BucketedRandomProjectionLSHModel(_LSHModel):
    bucketLength = BucketedRandomProjectionLSH.bucketLength

    def _hash(self, X):
        return torch.floor(X @ torch.from_numpy(self._R).to(X.device).T / self.getOrDefault(self.bucketLength))

    def _dist(self, X, k):
        return ((X - k[None, :]) ** 2).sum(1).sqrt()


@register("org.apache.spark.ml.feature.MinHashLSH")
class MinHashLSH(Estimator, _LSHParams, MLWritable, MLReadable):
    """LSH class for Jaccard distance (inputs are binary vectors)."""

    @keyword_only
    def __init__(self, *, inputCol=None, outputCol=None, seed=None, numHashTables=1):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        rng = np.random.default_rng(self.getOrDefault(self.seed))
        p = 2038074743
        m = MinHashLSHModel()
        m._ab = np.stack([rng.integers(1, p, self.getOrDefault(self.numHashTables)),
                          rng.integers(0, p, self.getOrDefault(self.numHashTables))], 1)
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.MinHashLSHModel")
class MinHashLSHModel(_LSHModel):
    def _hash(self, X):
        p = 2038074743
        idx = torch.arange(X.shape[1], dtype=torch.float64, device=X.device)
        out = []
        for a, b in self._ab:
            h = torch.remainder((1 + idx) * float(a) + float(b), p)
            hv = torch.where(X != 0, h[None, :], torch.full_like(X, float("inf")))
            out.append(hv.min(1).values)
        return torch.stack(out, 1)

    def _dist(self, X, k):
        a = X != 0
        b = (k != 0)[None, :]
        inter = (a & b).sum(1).to(torch.float64)
        union = (a | b).sum(1).to(torch.float64)
        return 1 - inter / union.clamp_min(1)


from ._feature_extra import (RFormula, RFormulaModel, UnivariateFeatureSelector,  # noqa: E402,F401
                             UnivariateFeatureSelectorModel, Word2Vec, Word2VecModel)
from ._target_encoder import TargetEncoder, TargetEncoderModel  # noqa: E402,F401

__all__ = [n for n, v in list(globals().items()) if isinstance(v, type) and issubclass(v, (Transformer, Estimator))
           and not n.startswith("_")] + ["to_vector_column"]
_ = (HasMaxIter, HasStepSize, HasTol, HasWeightCol)

