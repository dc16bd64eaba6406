"""RFormula, UnivariateFeatureSelector and Word2Vec (``pyspark.ml.feature``), plus the
ANOVA / F-value univariate tests they share with ``ml.stat``.

Reached in the reference through the Feature widget (transformers) and, for the
estimators, this framework's Feature Estimator widget (SURVEY §2.5 note, §2.7).

* Univariate tests are one pass: the per-class sums are the one-hot GEMM used by
  NaiveBayes (ml/_nb.py), correlations are one Gram GEMM; one all-reduce each.
* Word2Vec is skip-gram with negative sampling (Mikolov et al.) trained as batched
  gather -> dot -> scatter-add updates on the device; ranks train on their own sentences
  and average the embedding tables after every epoch (one all-reduce per table), the
  MI355X analogue of Spark's per-partition training + merge.  Spark trains with
  hierarchical softmax, so vectors are not bit-comparable (parity unpinned); the API,
  vocabulary rules (minCount, frequency order) and persistence layout follow Spark.
"""
from __future__ import annotations

import math
import re
from collections import Counter, OrderedDict

import numpy as np
import torch

from ..frame import column as C
from ..frame.dataframe import DataFrame
from . import common as U
from ._nb import class_sums
from ._selector import _SelectorModel
from .base import Estimator, Model
from .linalg import DenseVector
from .param import (HasFeaturesCol, HasHandleInvalid, HasInputCol, HasLabelCol, HasMaxIter, HasOutputCol, HasSeed,
                    HasStepSize, TypeConverters, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, prim_list, read_data, register, write_data


# ====================================================== univariate statistics
def anova_f(comm, X: torch.Tensor, y: torch.Tensor):
    """One-way ANOVA F statistic and p-value of each continuous feature vs a categorical label."""
    from scipy.stats import f as fdist
    X = X.to(torch.float64)
    K = U.num_classes(comm, y)
    S, S2, cnt = class_sums(comm, X, y, None, K, squares=True)
    S, S2, cnt = S.cpu().numpy(), S2.cpu().numpy(), cnt.cpu().numpy()
    n = cnt.sum()
    k = int((cnt > 0).sum())
    tot = S.sum(0)
    between = (S ** 2 / np.maximum(cnt, 1)[:, None]).sum(0)
    ssb = between - tot ** 2 / n
    ssw = S2.sum(0) - between
    dfb, dfw = max(k - 1, 1), max(n - k, 1)
    with np.errstate(divide="ignore", invalid="ignore"):
        F = (ssb / dfb) / (ssw / dfw)
    F = np.where(np.isfinite(F), F, 0.0)
    return F, fdist.sf(F, dfb, dfw), np.full(F.shape, dfb + dfw, dtype=np.int64)


def f_regression(comm, X: torch.Tensor, y: torch.Tensor):
    """F statistic of the univariate linear regression of y on each feature."""
    from scipy.stats import f as fdist
    X = X.to(torch.float64)
    y = y.to(X.device, torch.float64)
    d = X.shape[1]
    st = torch.cat([X.sum(0), (X * X).sum(0), y @ X, torch.stack([y.sum(), (y * y).sum(),
                                                                   torch.tensor(float(X.shape[0]), dtype=torch.float64,
                                                                                device=X.device)])])
    comm.all_reduce(st)
    st = st.cpu().numpy()
    sx, sxx, sxy = st[:d], st[d:2 * d], st[2 * d:3 * d]
    sy, syy, n = st[3 * d], st[3 * d + 1], st[3 * d + 2]
    cov = sxy - sx * sy / n
    vx = sxx - sx * sx / n
    vy = syy - sy * sy / n
    with np.errstate(divide="ignore", invalid="ignore"):
        r2 = np.where((vx > 0) & (vy > 0), cov * cov / (vx * vy), 0.0)
        F = np.where(r2 < 1, r2 / (1 - r2) * (n - 2), np.inf)
    return F, fdist.sf(F, 1, max(n - 2, 1)), np.full(d, int(n - 1), dtype=np.int64)


def select_by_pvalues(p: np.ndarray, mode: str, threshold: float) -> list:
    order = np.argsort(p, kind="stable")
    F = len(p)
    if mode == "numTopFeatures":
        sel = order[: int(threshold)]
    elif mode == "percentile":
        sel = order[: int(F * threshold)]
    elif mode == "fpr":
        sel = np.nonzero(p < threshold)[0]
    elif mode == "fdr":
        ps = p[order]
        ok = np.nonzero(ps <= threshold * (np.arange(F) + 1) / F)[0]
        sel = order[: ok.max() + 1] if ok.size else np.array([], dtype=int)
    elif mode == "fwe":
        sel = np.nonzero(p < threshold / F)[0]
    else:
        raise ValueError(f"unknown selectionMode {mode}")
    return sorted(int(i) for i in sel)


@register("org.apache.spark.ml.feature.UnivariateFeatureSelector")
class UnivariateFeatureSelector(Estimator, HasFeaturesCol, HasOutputCol, HasLabelCol, MLWritable, MLReadable):
    """Feature selector based on univariate statistical tests against labels.  The test is
    chosen by (featureType, labelType): categorical/categorical -> chi-squared,
    continuous/categorical -> ANOVA F-test, continuous/continuous -> F-value regression."""

    featureType = shared("featureType", "The feature type. Supported options: categorical, continuous.",
                         TypeConverters.toString)
    labelType = shared("labelType", "The label type. Supported options: categorical, continuous.",
                       TypeConverters.toString)
    selectionMode = shared("selectionMode", "The selection mode. Supported options: numTopFeatures (default), "
                                            "percentile, fpr, fdr, fwe.", TypeConverters.toString)
    selectionThreshold = shared("selectionThreshold", "The upper bound of the features that selector will "
                                                      "select.", TypeConverters.toFloat)

    @keyword_only
    def __init__(self, *, featuresCol="features", outputCol=None, labelCol="label", selectionMode="numTopFeatures"):
        super().__init__()
        self._setDefault(selectionMode="numTopFeatures", featuresCol="features", labelCol="label")
        self._set(**self._input_kwargs)

    def setFeatureType(self, value):
        return self._set(featureType=value)

    def setLabelType(self, value):
        return self._set(labelType=value)

    def setSelectionThreshold(self, value):
        return self._set(selectionThreshold=value)

    def _fit(self, df):
        from .stat import chi_square_pvalues
        g = self.getOrDefault
        X = U.dense_features(df, g(self.featuresCol), torch.float64)
        y = U.numeric_column(df, g(self.labelCol))
        ft, lt = g(self.featureType), g(self.labelType)
        if ft == "categorical" and lt == "categorical":
            p = chi_square_pvalues(df.comm, X, y)
        elif ft == "continuous" and lt == "categorical":
            p = anova_f(df.comm, X, y)[1]
        elif ft == "continuous" and lt == "continuous":
            p = f_regression(df.comm, X, y)[1]
        else:
            raise ValueError(f"Unsupported featureType {ft} with labelType {lt}")
        mode = g(self.selectionMode)
        default = {"numTopFeatures": 50, "percentile": 0.1, "fpr": 0.05, "fdr": 0.05, "fwe": 0.05}[mode]
        thr = g(self.selectionThreshold) if self.isDefined(self.selectionThreshold) else default
        m = UnivariateFeatureSelectorModel()
        m.selectedFeatures = select_by_pvalues(np.asarray(p), mode, thr)
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.UnivariateFeatureSelectorModel")
class UnivariateFeatureSelectorModel(_SelectorModel):
    """Model fitted by UnivariateFeatureSelector."""


# ==================================================================== RFormula
_TERM = re.compile(r"\s*([^+\-]+|[+\-])\s*")


def parse_formula(formula: str, columns: list, label_hint: str | None = None):
    """R model formula subset: ``y ~ a + b + a:b + . - c``, ``+ 0`` / ``- 1`` drop the
    intercept.  Returns (label, [terms as tuples of column names], has_intercept)."""
    if "~" not in formula:
        raise ValueError(f"RFormula requires a '~': {formula!r}")
    lhs, rhs = (s.strip() for s in formula.split("~", 1))
    label = lhs or label_hint
    terms: list = []
    removed: list = []
    intercept = True
    sign = "+"
    for tok in _TERM.findall(rhs):
        tok = tok.strip()
        if tok in "+-":
            sign = tok
            continue
        if tok in ("0", "1"):
            intercept = (tok == "1") if sign == "+" else (tok != "1")
            continue
        parts = []
        for fac in tok.split(":"):
            fac = fac.strip()
            if fac == ".":
                parts.append([c for c in columns if c != label])
            else:
                if fac not in columns:
                    raise ValueError(f"column {fac!r} of formula not found in {columns}")
                parts.append([fac])
        expanded = [()]
        for p in parts:
            expanded = [e + (c,) for e in expanded for c in p]
        if sign == "+":
            for t in expanded:
                if t not in terms:
                    terms.append(t)
        else:
            removed.extend(expanded)
    terms = [t for t in terms if t not in removed]
    return label, terms, intercept


class _RFormulaParams(HasFeaturesCol, HasLabelCol, HasHandleInvalid):
    formula = shared("formula", "R model formula", TypeConverters.toString)
    forceIndexLabel = shared("forceIndexLabel", "Force to index label whether it is numeric or string",
                             TypeConverters.toBoolean)
    stringIndexerOrderType = shared("stringIndexerOrderType", "How to order categories of a string feature column "
                                                              "used by StringIndexer. The last category after "
                                                              "ordering is dropped when encoding strings. Supported "
                                                              "options: frequencyDesc, frequencyAsc, alphabetDesc, "
                                                              "alphabetAsc. The default value is frequencyDesc.",
                                    TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(featuresCol="features", labelCol="label", forceIndexLabel=False,
                         stringIndexerOrderType="frequencyDesc", handleInvalid="error")


def _order_levels(cnt: Counter, order: str) -> list:
    keys = list(cnt)
    if order == "frequencyDesc":
        keys.sort(key=lambda k: (-cnt[k], k))
    elif order == "frequencyAsc":
        keys.sort(key=lambda k: (cnt[k], k))
    elif order == "alphabetDesc":
        keys.sort(reverse=True)
    else:
        keys.sort()
    return keys


def _is_string(col) -> bool:
    return isinstance(col, C.StringColumn) or (isinstance(col, C.HostColumn) and not isinstance(col, C.ArrayColumn))


@register("org.apache.spark.ml.feature.RFormula")
class RFormula(Estimator, _RFormulaParams, MLWritable, MLReadable):
    """Implements the transforms required for fitting a dataset against an R model formula.
    Currently we support a limited subset of the R operators, including '~', '.', ':', '+',
    '-'. String features are one-hot encoded (last category dropped when the formula has an
    intercept), numeric features are used as is, interactions are products."""

    @keyword_only
    def __init__(self, *, formula=None, featuresCol="features", labelCol="label", forceIndexLabel=False,
                 handleInvalid="error", stringIndexerOrderType="frequencyDesc"):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        label, terms, intercept = parse_formula(g(self.formula), df.columns)
        levels = {}
        order = g(self.stringIndexerOrderType)
        for c in sorted({c for t in terms for c in t}):
            if _is_string(df.column_data(c)):
                cnt = Counter(v for v in df.column_data(c).values if v is not None)
                tot = Counter()
                for part in df.comm.all_gather_object(cnt):
                    tot.update(part)
                levels[c] = _order_levels(tot, order)
        label_levels = None
        if label and label in df.columns and (_is_string(df.column_data(label)) or g(self.forceIndexLabel)):
            col = df.column_data(label)
            vals = col.values if _is_string(col) else [repr(float(v)) for v in col.to_pylist()]
            cnt = Counter(v for v in vals if v is not None)
            tot = Counter()
            for part in df.comm.all_gather_object(cnt):
                tot.update(part)
            label_levels = _order_levels(tot, order)
        m = RFormulaModel._from(label, terms, intercept, levels, label_levels)
        return m._with_parent(self)


@register("org.apache.spark.ml.feature.RFormulaModel")
class RFormulaModel(Model, _RFormulaParams, MLWritable, MLReadable):
    """Model fitted by RFormula: fixed terms, string levels and label indexing."""

    def __init__(self):
        super().__init__()
        self._label, self._terms, self._intercept = None, [], True
        self._levels: dict = {}
        self._label_levels = None

    @classmethod
    def _from(cls, label, terms, intercept, levels, label_levels):
        m = cls()
        m._label, m._terms, m._intercept = label, [tuple(t) for t in terms], bool(intercept)
        m._levels, m._label_levels = dict(levels), label_levels
        return m

    @property
    def resolvedFormula(self) -> str:
        rhs = " + ".join(":".join(t) for t in self._terms) or "0"
        return f"{self._label or ''} ~ {rhs}" + ("" if self._intercept else " - 1")

    def __str__(self):
        return f"RFormulaModel({self.resolvedFormula}) (uid={self.uid})"

    def _encode(self, df, c, drop_last, dev):
        col = df.column_data(c)
        n = len(df)
        if c in self._levels:
            lv = self._levels[c]
            idx = {v: i for i, v in enumerate(lv)}
            hi = self.getOrDefault(self.handleInvalid)
            codes = []
            for v in col.values:
                if v in idx:
                    codes.append(idx[v])
                elif hi == "keep":
                    codes.append(len(lv))
                elif hi == "skip":
                    codes.append(-1)
                else:
                    raise ValueError(f"Unseen label: {v} in column {c}. To handle unseen labels, set "
                                     "handleInvalid to 'keep' or 'skip'.")
            width = len(lv) + (1 if hi == "keep" else 0)
            width_out = width - 1 if drop_last else width
            t = torch.tensor(codes, dtype=torch.int64, device=dev)
            M = torch.zeros((n, width), dtype=torch.float64, device=dev)
            ok = t >= 0
            M[torch.nonzero(ok).reshape(-1), t[ok]] = 1.0
            return M[:, :width_out], ok
        if isinstance(col, C.NumericColumn):
            return col.data.to(dev, torch.float64)[:, None], torch.ones(n, dtype=torch.bool, device=dev)
        X = U.dense_features(df, c, torch.float64).to(dev)
        return X, torch.ones(n, dtype=torch.bool, device=dev)

    def _transform(self, df):
        dev = df.session.device
        n = len(df)
        blocks = []
        keep = torch.ones(n, dtype=torch.bool, device=dev)
        first_string = True
        for t in self._terms:
            M = torch.ones((n, 1), dtype=torch.float64, device=dev)
            for c in t:
                drop = True
                if c in self._levels and not self._intercept and first_string and len(t) == 1:
                    drop = False                        # no intercept: first factor keeps all levels
                    first_string = False
                E, ok = self._encode(df, c, drop, dev)
                keep &= ok
                M = (M[:, :, None] * E[:, None, :]).reshape(n, -1)
            blocks.append(M)
        X = torch.cat(blocks, dim=1) if blocks else torch.zeros((n, 0), dtype=torch.float64, device=dev)
        out = df
        if not bool(keep.all()):
            out = out._mask(keep)
            X = X[keep]
        from .feature import _out_vec
        out = _out_vec(out, self.getOrDefault(self.featuresCol), X)
        lab = self._label
        if lab and lab in out.columns:
            col = out.column_data(lab)
            if self._label_levels is not None:
                vals = col.values if _is_string(col) else [repr(float(v)) for v in col.to_pylist()]
                idx = {v: i for i, v in enumerate(self._label_levels)}
                y = torch.tensor([float(idx.get(v, np.nan)) for v in vals], dtype=torch.float64, device=dev)
            else:
                y = col.data.to(dev, torch.float64) if isinstance(col, C.NumericColumn) else \
                    U.numeric_column(out, lab).to(dev)
            out = out.withColumnData(self.getOrDefault(self.labelCol), C.NumericColumn(y))
        return out

    def _save_data(self, path):
        import json

        import pyarrow as pa
        write_data(path, {"label": pa.array([self._label or ""]),
                          "terms": pa.array([[list(t) for t in self._terms]], pa.list_(pa.list_(pa.string()))),
                          "hasIntercept": pa.array([self._intercept]),
                          "levels": pa.array([json.dumps(self._levels)]),
                          "labelLevels": pa.array([json.dumps(self._label_levels)])})

    @classmethod
    def _load_impl(cls, path, meta):
        import json
        t = read_data(path).to_pylist()[0]
        m = cls._from(t["label"] or None, [tuple(x) for x in t["terms"]], t["hasIntercept"],
                      json.loads(t["levels"]), json.loads(t["labelLevels"]))
        apply_metadata(m, meta)
        return m


# ==================================================================== Word2Vec
class _Word2VecParams(HasInputCol, HasOutputCol, HasMaxIter, HasSeed, HasStepSize):
    vectorSize = shared("vectorSize", "the dimension of codes after transforming from words", TypeConverters.toInt)
    numPartitions = shared("numPartitions", "number of partitions for sentences of words", TypeConverters.toInt)
    minCount = shared("minCount", "the minimum number of times a token must appear to be included in the "
                                  "word2vec model's vocabulary", TypeConverters.toInt)
    windowSize = shared("windowSize", "the window size (context words from [-window, window]). Default value "
                                      "is 5", TypeConverters.toInt)
    maxSentenceLength = shared("maxSentenceLength", "Maximum length (in words) of each sentence in the input data. "
                                                    "Any sentence longer than this threshold will be divided into "
                                                    "chunks up to the size.", TypeConverters.toInt)

    def __init__(self):
        super().__init__()
        self._setDefault(vectorSize=100, minCount=5, numPartitions=1, stepSize=0.025, maxIter=1, windowSize=5,
                         maxSentenceLength=1000, seed=0)


def _sentences(df, name):
    return [list(v) if v is not None else [] for v in df.column_data(name).values]


def train_sgns(comm, sents: list, vocab: dict, dim: int, window: int, epochs: int, lr0: float, seed: int,
               max_len: int, device, negatives: int = 5, batch: int = 8192):
    """Skip-gram negative sampling; returns the [V, dim] input embedding table."""
    V = len(vocab)
    g = torch.Generator(device="cpu").manual_seed(seed)
    syn0 = ((torch.rand((V, dim), generator=g, dtype=torch.float64) - 0.5) / dim).to(device, torch.float32)
    syn1 = torch.zeros((V, dim), dtype=torch.float32, device=device)
    ids, sid = [], []
    chunk_id = 0
    for s in sents:
        w = [vocab[t] for t in s if t in vocab]
        for a in range(0, len(w), max_len):          # long sentences are cut into chunks
            piece = w[a:a + max_len]
            ids.extend(piece)
            sid.extend([chunk_id] * len(piece))
            chunk_id += 1
    tok = torch.tensor(ids, dtype=torch.int64)
    sent = torch.tensor(sid, dtype=torch.int64)
    counts = torch.bincount(tok, minlength=V).to(device, torch.float64)
    comm.all_reduce(counts)
    noise = counts.cpu().clamp_min(1) ** 0.75
    noise = (noise / noise.sum()).to(torch.float32)
    n = tok.shape[0]
    total_steps = max(1, epochs * max(1, n))
    done = 0
    for ep in range(epochs):
        # dynamic window: every centre draws b in [1, window]
        b = torch.randint(1, window + 1, (n,), generator=g)
        cen, ctx = [], []
        for o in range(-window, window + 1):
            if o == 0:
                continue
            i = torch.arange(max(0, -o), min(n, n - o))
            j = i + o
            ok = (sent[i] == sent[j]) & (b[i] >= abs(o))
            cen.append(tok[i[ok]])
            ctx.append(tok[j[ok]])
        cen = torch.cat(cen) if cen else torch.zeros(0, dtype=torch.int64)
        ctx = torch.cat(ctx) if ctx else torch.zeros(0, dtype=torch.int64)
        perm = torch.randperm(cen.shape[0], generator=g)
        cen, ctx = cen[perm].to(device), ctx[perm].to(device)
        P = cen.shape[0]
        for a in range(0, P, batch):
            c = cen[a:a + batch]
            o = ctx[a:a + batch]
            m = c.shape[0]
            lr = lr0 * max(1e-4, 1.0 - (done + (ep * n) + a / max(P, 1) * n) / total_steps)
            neg = torch.multinomial(noise, m * negatives, replacement=True, generator=g).to(device).reshape(
                m, negatives)
            tgt = torch.cat([o[:, None], neg], dim=1)                      # [m, 1+neg]
            lbl = torch.zeros((m, 1 + negatives), dtype=torch.float32, device=device)
            lbl[:, 0] = 1.0
            v = syn0[c]                                                    # [m, dim]
            u = syn1[tgt]                                                  # [m, 1+neg, dim]
            sc = torch.sigmoid((u * v[:, None, :]).sum(-1))
            gcoef = (lbl - sc) * lr                                        # [m, 1+neg]
            dv = (gcoef[:, :, None] * u).sum(1)
            du = gcoef[:, :, None] * v[:, None, :]
            # a word hit k times in one batch gets its summed update scaled by 1/sqrt(k):
            # the plain sum (k SGD steps taken at once) diverges for frequent words, the
            # mean starves them of progress
            tf = tgt.reshape(-1)
            k1 = torch.bincount(tf, minlength=V).clamp_min(1).to(torch.float32).sqrt()
            k0 = torch.bincount(c, minlength=V).clamp_min(1).to(torch.float32).sqrt()
            syn1.index_add_(0, tf, du.reshape(-1, dim) / k1[tf, None])
            syn0.index_add_(0, c, dv / k0[c, None])
        done = (ep + 1) * n
        if comm.world_size > 1:
            for t in (syn0, syn1):
                comm.all_reduce(t)
                t /= comm.world_size
    return syn0.to(torch.float64)


@register("org.apache.spark.ml.feature.Word2Vec")
class Word2Vec(Estimator, _Word2VecParams, MLWritable, MLReadable):
    """Word2Vec trains a model of `Map(String, Vector)`, i.e. transforms a word into a code
    for further natural language processing or machine learning process."""

    @keyword_only
    def __init__(self, *, vectorSize=100, minCount=5, numPartitions=1, stepSize=0.025, maxIter=1, seed=None,
                 inputCol=None, outputCol=None, windowSize=5, maxSentenceLength=1000):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        sents = _sentences(df, g(self.inputCol))
        cnt = Counter(t for s in sents for t in s)
        tot = Counter()
        for part in df.comm.all_gather_object(cnt):
            tot.update(part)
        words = [w for w, c in tot.items() if c >= g(self.minCount)]
        words.sort(key=lambda w: (-tot[w], w))
        vocab = {w: i for i, w in enumerate(words)}
        if not vocab:
            raise ValueError("The vocabulary size should be > 0. You may need to check the setting of minCount, "
                             "which could be large enough to remove all your words in sentences.")
        E = train_sgns(df.comm, sents, vocab, g(self.vectorSize), g(self.windowSize), g(self.maxIter),
                       g(self.stepSize), int(g(self.seed)) & 0x7FFFFFFF, g(self.maxSentenceLength),
                       df.session.device)
        return Word2VecModel._from(words, E.cpu().numpy())._with_parent(self)


@register("org.apache.spark.ml.feature.Word2VecModel")
class Word2VecModel(Model, _Word2VecParams, MLWritable, MLReadable):
    """Model fitted by Word2Vec."""

    def __init__(self):
        super().__init__()
        self._words: list = []
        self._E = np.zeros((0, 0))

    @classmethod
    def _from(cls, words, E):
        m = cls()
        m._words, m._E = list(words), np.asarray(E, dtype=np.float64)
        m._index = {w: i for i, w in enumerate(m._words)}
        return m

    def getVectors(self):
        from ..session import Session
        s = Session.getOrCreate()
        w = np.empty(len(self._words), dtype=object)
        w[:] = self._words
        return DataFrame(s.local_view(), OrderedDict(word=C.StringColumn(w),
                                                     vector=C.VectorColumn(torch.from_numpy(self._E))))

    def _query(self, word):
        if isinstance(word, str):
            if word not in self._index:
                raise ValueError(f"{word} not in vocabulary")
            return self._E[self._index[word]], word
        return np.asarray(word.toArray() if hasattr(word, "toArray") else word, dtype=np.float64), None

    def findSynonymsArray(self, word, num):
        q, self_word = self._query(word)
        norms = np.linalg.norm(self._E, axis=1) * max(np.linalg.norm(q), 1e-300)
        sims = self._E @ q / np.maximum(norms, 1e-300)
        order = np.argsort(-sims, kind="stable")
        out = [(self._words[i], float(sims[i])) for i in order if self._words[i] != self_word]
        return out[:num]

    def findSynonyms(self, word, num):
        from ..session import Session
        s = Session.getOrCreate()
        pairs = self.findSynonymsArray(word, num)
        w = np.empty(len(pairs), dtype=object)
        w[:] = [p[0] for p in pairs]
        return DataFrame(s.local_view(), OrderedDict(word=C.StringColumn(w), similarity=C.NumericColumn(
            torch.tensor([p[1] for p in pairs], dtype=torch.float64))))

    def _transform(self, df):
        sents = _sentences(df, self.getOrDefault(self.inputCol))
        dev = df.session.device
        E = torch.from_numpy(self._E).to(dev)
        rows, cols = [], []
        for r, s in enumerate(sents):
            for t in s:
                j = self._index.get(t)
                if j is not None:
                    rows.append(r)
                    cols.append(j)
        n = len(sents)
        out = torch.zeros((n, E.shape[1]), dtype=torch.float64, device=dev)
        if rows:
            r = torch.tensor(rows, dtype=torch.int64, device=dev)
            out.index_add_(0, r, E[torch.tensor(cols, dtype=torch.int64, device=dev)])
        lens = torch.tensor([max(len(s), 1) for s in sents], dtype=torch.float64, device=dev)
        out = out / lens[:, None]
        from .feature import _out_vec
        return _out_vec(df, self.getOrDefault(self.outputCol), out)

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"word": pa.array(self._words),
                          "vector": pa.array([list(map(float, v)) for v in self._E], prim_list(pa.float32()))})

    @classmethod
    def _load_impl(cls, path, meta):
        t = read_data(path).to_pydict()
        m = cls._from(t["word"], np.asarray(t["vector"], dtype=np.float64))
        apply_metadata(m, meta)
        return m


_ = (math, DenseVector)
