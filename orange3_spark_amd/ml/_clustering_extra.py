"""BisectingKMeans, GaussianMixture, LDA and PowerIterationClustering
(``pyspark.ml.clustering``), reached through the Clustering widget's reflection
(orangecontrib/spark/widgets/ml/spark_ml_clustering.py:14; SURVEY §2.7 lists them as
Spark >= 2.0 additions).  Engines: models/clustering_extra.py.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch

from ..frame import column as C
from ..frame.dataframe import DataFrame
from ..models import clustering_extra as CE
from . import common as U
from .base import Estimator, Model
from .linalg import DenseMatrix, DenseVector
from .param import (HasCheckpointInterval, HasDistanceMeasure, HasFeaturesCol, HasMaxIter, HasPredictionCol,
                    HasProbabilityCol, HasSeed, HasTol, HasWeightCol, Params, TypeConverters, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, mat_col, prim_list, read_data, register, vec_col, write_data


def _float_features(df, name):
    X = U.dense_features(df, name)
    return X.to(torch.float64)


class _Summary:
    def __init__(self, **kw):
        self.__dict__.update(kw)


# ============================================================ BisectingKMeans
class _BisectingKMeansParams(HasFeaturesCol, HasPredictionCol, HasMaxIter, HasSeed, HasDistanceMeasure,
                             HasWeightCol):
    k = shared("k", "The desired number of leaf clusters. Must be > 1.", TypeConverters.toInt)
    minDivisibleClusterSize = shared("minDivisibleClusterSize", "The minimum number of points (if >= 1.0) or the "
                                                                "minimum proportion of points (if < 1.0) of a "
                                                                "divisible cluster.", TypeConverters.toFloat)

    def __init__(self):
        super().__init__()
        self._setDefault(k=4, maxIter=20, minDivisibleClusterSize=1.0, distanceMeasure="euclidean", seed=0)


@register("org.apache.spark.ml.clustering.BisectingKMeans")
class BisectingKMeans(Estimator, _BisectingKMeansParams, MLWritable, MLReadable):
    """A bisecting k-means algorithm based on the paper "A comparison of document clustering
    techniques" by Steinbach, Karypis, and Kumar, with modification to fit Spark. The
    algorithm starts from a single cluster that contains all points. Iteratively it finds
    divisible clusters on the bottom level and bisects each of them using k-means, until
    there are `k` leaf clusters in total or no leaf clusters are divisible."""

    @keyword_only
    def __init__(self, *, featuresCol="features", predictionCol="prediction", maxIter=20, seed=None, k=4,
                 minDivisibleClusterSize=1.0, distanceMeasure="euclidean", weightCol=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        X = _float_features(df, g(self.featuresCol))
        r = CE.fit_bisecting(df.comm, X, g(self.k), g(self.maxIter), int(g(self.seed)) & 0xFFFFFFFF,
                             g(self.minDivisibleClusterSize), g(self.distanceMeasure) == "cosine")
        m = BisectingKMeansModel._from(r.centers, r.children)
        m.summary = _Summary(k=len(r.leaves), clusterSizes=r.sizes, trainingCost=r.cost, numIter=g(self.maxIter))
        return m._with_parent(self)


@register("org.apache.spark.ml.clustering.BisectingKMeansModel")
class BisectingKMeansModel(Model, _BisectingKMeansParams, MLWritable, MLReadable):
    """Model fitted by BisectingKMeans (keeps the whole bisection tree for prediction)."""

    def __init__(self):
        super().__init__()
        self._centers: dict = {}
        self._children: dict = {}
        self._leaves: list = []
        self.summary = None

    @classmethod
    def _from(cls, centers, children):
        m = cls()
        m._centers = {int(i): np.asarray(c, float) for i, c in centers.items()}
        m._children = {int(i): (int(a), int(b)) for i, (a, b) in children.items()}
        m._leaves = CE.leaf_order(m._children)
        return m

    @property
    def hasSummary(self):
        return self.summary is not None

    def clusterCenters(self):
        return [self._centers[i].copy() for i in self._leaves]

    def _predict_tensor(self, X):
        return CE.bisecting_predict(X, self._centers, self._children, self._leaves,
                                    self.getOrDefault(self.distanceMeasure) == "cosine")

    def _transform(self, df):
        X = _float_features(df, self.getOrDefault(self.featuresCol))
        return df.withColumnData(self.getOrDefault(self.predictionCol),
                                 C.NumericColumn(self._predict_tensor(X).to(torch.int32)))

    def predict(self, value):
        x = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value), dtype=torch.float64)
        return int(self._predict_tensor(x[None, :])[0])

    def computeCost(self, df):
        X = _float_features(df, self.getOrDefault(self.featuresCol))
        a = self._predict_tensor(X)
        Cm = torch.from_numpy(np.stack(self.clusterCenters())).to(X.device)
        d = ((X - Cm[a]) ** 2).sum()
        df.comm.all_reduce(d)
        return float(d)

    def _save_data(self, path):
        import pyarrow as pa
        idx = sorted(self._centers)
        write_data(path, {"index": pa.array(idx, pa.int32()),
                          "center": vec_col([DenseVector(self._centers[i]) for i in idx]),
                          "children": pa.array([list(self._children.get(i, ())) for i in idx], prim_list(pa.int32()))})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import vector_from_struct
        rows = read_data(path).to_pylist()
        centers = {r["index"]: vector_from_struct(r["center"]).toArray() for r in rows}
        children = {r["index"]: tuple(r["children"]) for r in rows if r["children"]}
        m = cls._from(centers, children)
        apply_metadata(m, meta)
        return m


# ============================================================ GaussianMixture
class MultivariateGaussian:
    def __init__(self, mean, cov):
        self.mean = DenseVector(mean)
        self.cov = DenseMatrix.from_array(np.asarray(cov))


class _GaussianMixtureParams(HasFeaturesCol, HasPredictionCol, HasProbabilityCol, HasMaxIter, HasSeed, HasTol,
                             HasWeightCol):
    k = shared("k", "Number of independent Gaussians in the mixture model. Must be > 1.", TypeConverters.toInt)
    aggregationDepth = shared("aggregationDepth", "suggested depth for treeAggregate (>= 2).", TypeConverters.toInt)

    def __init__(self):
        super().__init__()
        self._setDefault(k=2, tol=0.01, maxIter=100, aggregationDepth=2, seed=0)


@register("org.apache.spark.ml.clustering.GaussianMixture")
class GaussianMixture(Estimator, _GaussianMixtureParams, MLWritable, MLReadable):
    """GaussianMixture clustering. This class performs expectation maximization for
    multivariate Gaussian Mixture Models (GMMs)."""

    @keyword_only
    def __init__(self, *, featuresCol="features", predictionCol="prediction", k=2, probabilityCol="probability",
                 tol=0.01, maxIter=100, seed=None, aggregationDepth=2, weightCol=None):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        X = _float_features(df, g(self.featuresCol))
        r = CE.fit_gmm(df.comm, X, g(self.k), g(self.maxIter), g(self.tol), int(g(self.seed)) & 0xFFFFFFFF,
                       U.weights_or_none(df, self))
        m = GaussianMixtureModel._from(r.weights, r.means, r.covs)
        a = m._predict_tensor(X)
        sizes = torch.bincount(a, minlength=g(self.k)).to(torch.float64)
        df.comm.all_reduce(sizes)
        m.summary = _Summary(k=g(self.k), logLikelihood=r.log_likelihood, numIter=r.iterations,
                             clusterSizes=[int(v) for v in sizes.tolist()], objectiveHistory=r.history)
        return m._with_parent(self)


@register("org.apache.spark.ml.clustering.GaussianMixtureModel")
class GaussianMixtureModel(Model, _GaussianMixtureParams, MLWritable, MLReadable):
    """Model fitted by GaussianMixture."""

    def __init__(self):
        super().__init__()
        self._w = np.zeros(0)
        self._mu = np.zeros((0, 0))
        self._cov = np.zeros((0, 0, 0))
        self.summary = None

    @classmethod
    def _from(cls, w, mu, cov):
        m = cls()
        m._w, m._mu, m._cov = np.asarray(w, float), np.asarray(mu, float), np.asarray(cov, float)
        return m

    @property
    def hasSummary(self):
        return self.summary is not None

    @property
    def weights(self):
        return self._w.tolist()

    @property
    def gaussians(self):
        return [MultivariateGaussian(self._mu[i], self._cov[i]) for i in range(len(self._w))]

    @property
    def gaussiansDF(self):
        from ..session import Session
        s = Session.getOrCreate()
        mean = np.empty(len(self._w), dtype=object)
        mean[:] = [DenseVector(v) for v in self._mu]
        cov = np.empty(len(self._w), dtype=object)
        cov[:] = [DenseMatrix.from_array(c) for c in self._cov]
        return DataFrame(s.local_view(), OrderedDict(mean=C.ArrayColumn(mean), cov=C.ArrayColumn(cov)))

    def _prob(self, X):
        dev = X.device
        lp = CE.gmm_log_prob(X.to(torch.float64), torch.from_numpy(self._mu).to(dev),
                             torch.from_numpy(self._cov).to(dev), torch.log(torch.from_numpy(self._w).to(dev)))
        return torch.softmax(lp, dim=1)

    def _predict_tensor(self, X):
        return self._prob(X).argmax(1)

    def predict(self, value):
        x = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value), dtype=torch.float64)
        return int(self._predict_tensor(x[None, :])[0])

    def predictProbability(self, value):
        x = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value), dtype=torch.float64)
        return DenseVector(self._prob(x[None, :])[0].cpu().numpy())

    def _transform(self, df):
        X = _float_features(df, self.getOrDefault(self.featuresCol))
        P = self._prob(X)
        out = df
        if self.getOrDefault(self.probabilityCol):
            out = out.withColumnData(self.getOrDefault(self.probabilityCol), U.vec_out(P))
        if self.getOrDefault(self.predictionCol):
            out = out.withColumnData(self.getOrDefault(self.predictionCol), C.NumericColumn(P.argmax(1).to(torch.int32)))
        return out

    def _save_data(self, path):
        import pyarrow as pa
        from ..io import vector_arrow_type
        from .util import matrix_arrow_type, matrix_struct, vector_struct
        write_data(path, {
            "weights": pa.array([self._w.tolist()], prim_list(pa.float64())),
            "mus": pa.array([[vector_struct(DenseVector(v)) for v in self._mu]], pa.list_(vector_arrow_type())),
            "sigmas": pa.array([[matrix_struct(DenseMatrix.from_array(c)) for c in self._cov]],
                               pa.list_(matrix_arrow_type())),
        })

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import matrix_from_struct, vector_from_struct
        t = read_data(path).to_pylist()[0]
        m = cls._from(t["weights"], [vector_from_struct(v).toArray() for v in t["mus"]],
                      [matrix_from_struct(c).toArray() for c in t["sigmas"]])
        apply_metadata(m, meta)
        return m


# ======================================================================== LDA
class _LDAParams(HasFeaturesCol, HasMaxIter, HasSeed, HasCheckpointInterval):
    k = shared("k", "The number of topics (clusters) to infer. Must be > 1.", TypeConverters.toInt)
    optimizer = shared("optimizer", "Optimizer or inference algorithm used to estimate the LDA model. Supported: "
                                    "online, em", TypeConverters.toString)
    learningOffset = shared("learningOffset", "A (positive) learning parameter that downweights early iterations."
                                              " Larger values make early iterations count less",
                            TypeConverters.toFloat)
    learningDecay = shared("learningDecay", "Learning rate, set as anexponential decay rate. This should be "
                                            "between (0.5, 1.0] to guarantee asymptotic convergence.",
                           TypeConverters.toFloat)
    subsamplingRate = shared("subsamplingRate", "Fraction of the corpus to be sampled and used in each iteration "
                                                "of mini-batch gradient descent, in range (0, 1].",
                             TypeConverters.toFloat)
    optimizeDocConcentration = shared("optimizeDocConcentration", "Indicates whether the docConcentration "
                                                                  "(Dirichlet parameter for document-topic "
                                                                  "distribution) will be optimized during "
                                                                  "training.", TypeConverters.toBoolean)
    docConcentration = shared("docConcentration", 'Concentration parameter (commonly named "alpha") for the '
                                                  'prior placed on documents\' distributions over topics ("theta").',
                              TypeConverters.toListFloat)
    topicConcentration = shared("topicConcentration", 'Concentration parameter (commonly named "beta" or "eta") '
                                                      'for the prior placed on topic\' distributions over terms.',
                                TypeConverters.toFloat)
    topicDistributionCol = shared("topicDistributionCol", "Output column with estimates of the topic mixture "
                                                          "distribution for each document (often called \"theta\" "
                                                          "in the literature). Returns a vector of zeros for an "
                                                          "empty document.", TypeConverters.toString)
    keepLastCheckpoint = shared("keepLastCheckpoint", "(For EM optimizer) If using checkpointing, this indicates "
                                                      "whether to keep the last checkpoint. If false, then the "
                                                      "checkpoint will be deleted. Deleting the checkpoint can "
                                                      "cause failures if a data partition is lost, so set this "
                                                      "bit with care.", TypeConverters.toBoolean)

    def __init__(self):
        super().__init__()
        self._setDefault(k=10, maxIter=20, optimizer="online", learningOffset=1024.0, learningDecay=0.51,
                         subsamplingRate=0.05, optimizeDocConcentration=True, checkpointInterval=10,
                         topicDistributionCol="topicDistribution", keepLastCheckpoint=True, seed=0)


def _doc_chunks(col, chunk=4096):
    """Yield (row offset, rows, cols, vals, ndocs) nonzero triplets of a term-count column."""
    if isinstance(col, C.SparseVectorColumn):
        n = len(col)
        for a in range(0, n, chunk):
            b = min(n, a + chunk)
            sub = col.take(torch.arange(a, b))
            counts = (sub.indptr[1:] - sub.indptr[:-1])
            rows = torch.repeat_interleave(torch.arange(b - a, device=counts.device), counts)
            yield a, rows.to(sub.values.device), sub.indices.long().to(sub.values.device), \
                sub.values.to(torch.float64), b - a
    else:
        X = col.dense() if hasattr(col, "dense") else col
        X = X.to(torch.float64)
        for a in range(0, X.shape[0], chunk):
            Xc = X[a:a + chunk]
            nz = Xc.nonzero()
            yield a, nz[:, 0], nz[:, 1], Xc[nz[:, 0], nz[:, 1]], Xc.shape[0]


def _vocab(col) -> int:
    return int(col.size)


@register("org.apache.spark.ml.clustering.LDA")
class LDA(Estimator, _LDAParams, MLWritable, MLReadable):
    """Latent Dirichlet Allocation (LDA), a topic model designed for text documents.
    Terminology: "term" = "word": an element of the vocabulary; "token": instance of a term
    appearing in a document; "topic": multinomial distribution over terms representing some
    concept; "document": one piece of text, corresponding to one row in the input data.

    Inference is online variational Bayes (Hoffman, Blei and Bach 2010) for both
    ``optimizer`` values here; ``em`` runs it full-batch (subsamplingRate = 1, rho = 1).
    """

    @keyword_only
    def __init__(self, *, featuresCol="features", maxIter=20, seed=None, checkpointInterval=10, k=10,
                 optimizer="online", learningOffset=1024.0, learningDecay=0.51, subsamplingRate=0.05,
                 optimizeDocConcentration=True, docConcentration=None, topicConcentration=None,
                 topicDistributionCol="topicDistribution", keepLastCheckpoint=True):
        super().__init__()
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        comm = df.comm
        col = U.features_column(df, g(self.featuresCol))
        V = _vocab(col)
        K = g(self.k)
        dev = df.session.device if hasattr(df, "session") else torch.device("cpu")
        seed = int(g(self.seed)) & 0xFFFFFFFF
        gen = np.random.default_rng([seed, comm.rank])
        alpha = torch.full((K,), 1.0 / K, dtype=torch.float64, device=dev)
        if self.isDefined(self.docConcentration) and g(self.docConcentration):
            dc = list(g(self.docConcentration))
            alpha = torch.tensor(dc if len(dc) == K else dc * K, dtype=torch.float64, device=dev)[:K]
        eta = float(g(self.topicConcentration)) if self.isDefined(self.topicConcentration) and \
            g(self.topicConcentration) is not None else 1.0 / K
        g0 = np.random.default_rng(seed)
        lam = torch.from_numpy(g0.gamma(100.0, 1.0 / 100.0, size=(K, V))).to(dev)
        state = CE.LDAState(lam, alpha, eta)
        n_local = len(col)
        corpus = float(comm.sum_scalar(n_local))
        em = g(self.optimizer).lower() == "em"
        frac = 1.0 if em else float(g(self.subsamplingRate))
        tau0, kappa = float(g(self.learningOffset)), float(g(self.learningDecay))
        for it in range(1, g(self.maxIter) + 1):
            Eb = torch.exp(CE._dirichlet_expectation(state.lam))
            sst = torch.zeros((K, V), dtype=torch.float64, device=dev)
            gammas = []
            nb = 0
            keep = np.random.default_rng([seed, it, comm.rank]).random(n_local) < frac
            sel = torch.from_numpy(np.nonzero(keep)[0])
            sub = col.take(sel) if isinstance(col, C.SparseVectorColumn) else \
                C.VectorColumn(U.dense_features(df, g(self.featuresCol))[sel.to(dev)].to(torch.float64))
            for _, rows, cols, vals, nd in _doc_chunks(sub):
                gm, s = CE.lda_e_step(rows.to(dev), cols.to(dev), vals.to(dev), nd, Eb, state.alpha, gen)
                sst += s
                gammas.append(gm)
                nb += nd
            buf = torch.cat([sst.reshape(-1), torch.tensor([float(nb)], dtype=torch.float64, device=dev)])
            comm.all_reduce(buf)
            sst, batch = buf[:-1].reshape(K, V), float(buf[-1])
            if batch == 0:
                continue
            rho = 1.0 if em else (tau0 + it) ** (-kappa)
            state.lam = (1 - rho) * state.lam + rho * (eta + corpus / batch * sst)
            if g(self.optimizeDocConcentration):
                G_ = torch.cat(gammas) if gammas else torch.zeros((0, K), dtype=torch.float64, device=dev)
                allg = comm.all_gather_v(G_) if comm.world_size > 1 else G_
                state.alpha = CE.update_alpha(state.alpha, allg, rho)
            state.iterations = it
        if em:
            m = DistributedLDAModel._from(state.lam.cpu().numpy(), state.alpha.cpu().numpy(), eta, V)
            m._with_parent(self)
            m._train_ll, _ = m._doc_bound(df)
            m._log_prior = float(CE.topic_bound(m._state(dev)))
            return m
        m = LDAModel._from(state.lam.cpu().numpy(), state.alpha.cpu().numpy(), eta, V)
        return m._with_parent(self)


@register("org.apache.spark.ml.clustering.LocalLDAModel")
class LDAModel(Model, _LDAParams, MLWritable, MLReadable):
    """Model fitted by LDA (a local model: the topics matrix lives on every rank)."""

    def __init__(self):
        super().__init__()
        self._lam = np.zeros((0, 0))
        self._alpha = np.zeros(0)
        self._eta = 0.0
        self._V = 0

    @classmethod
    def _from(cls, lam, alpha, eta, V):
        m = cls()
        m._lam, m._alpha, m._eta, m._V = np.asarray(lam, float), np.asarray(alpha, float), float(eta), int(V)
        return m

    def isDistributed(self):
        return False

    def vocabSize(self):
        return self._V

    def topicsMatrix(self) -> DenseMatrix:
        """[vocabSize, k] matrix; column j = expected term weights of topic j."""
        beta = self._lam / self._lam.sum(1, keepdims=True)
        return DenseMatrix.from_array(beta.T)

    def estimatedDocConcentration(self) -> DenseVector:
        return DenseVector(self._alpha)

    def describeTopics(self, maxTermsPerTopic=10):
        from ..session import Session
        beta = self._lam / self._lam.sum(1, keepdims=True)
        idx = np.argsort(-beta, axis=1)[:, :maxTermsPerTopic]
        ti = np.empty(beta.shape[0], dtype=object)
        ti[:] = [list(map(int, r)) for r in idx]
        tw = np.empty(beta.shape[0], dtype=object)
        tw[:] = [[float(beta[k, j]) for j in r] for k, r in enumerate(idx)]
        s = Session.getOrCreate()
        return DataFrame(s.local_view(), OrderedDict(
            topic=C.NumericColumn(torch.arange(beta.shape[0], dtype=torch.int32)),
            termIndices=C.ArrayColumn(ti), termWeights=C.ArrayColumn(tw)))

    def _state(self, dev):
        return CE.LDAState(torch.from_numpy(self._lam).to(dev), torch.from_numpy(self._alpha).to(dev), self._eta)

    def _doc_bound(self, df):
        col = U.features_column(df, self.getOrDefault(self.featuresCol))
        dev = df.session.device if hasattr(df, "session") else torch.device("cpu")
        st = self._state(dev)
        gen = np.random.default_rng([int(self.getOrDefault(self.seed)) & 0xFFFFFFFF, 7])
        score = torch.zeros((), dtype=torch.float64, device=dev)
        tokens = torch.zeros((), dtype=torch.float64, device=dev)
        for _, rows, cols, vals, nd in _doc_chunks(col):
            s, _ = CE.lda_bound(rows.to(dev), cols.to(dev), vals.to(dev), nd, st, gen)
            score += s
            tokens += vals.sum().to(dev)
        buf = torch.stack([score, tokens])
        df.comm.all_reduce(buf)
        return float(buf[0]) + float(CE.topic_bound(st)), float(buf[1])

    def logLikelihood(self, dataset) -> float:
        return self._doc_bound(dataset)[0]

    def logPerplexity(self, dataset) -> float:
        ll, tokens = self._doc_bound(dataset)
        return -ll / max(tokens, 1e-300)

    def _transform(self, df):
        col = U.features_column(df, self.getOrDefault(self.featuresCol))
        dev = df.session.device if hasattr(df, "session") else torch.device("cpu")
        st = self._state(dev)
        Eb = torch.exp(CE._dirichlet_expectation(st.lam))
        gen = np.random.default_rng([int(self.getOrDefault(self.seed)) & 0xFFFFFFFF, 11])
        outs = []
        for _, rows, cols, vals, nd in _doc_chunks(col):
            gm, _ = CE.lda_e_step(rows.to(dev), cols.to(dev), vals.to(dev), nd, Eb, st.alpha, gen)
            theta = gm / gm.sum(1, keepdim=True)
            empty = torch.zeros(nd, dtype=torch.bool, device=dev)
            cnt = torch.zeros(nd, dtype=torch.float64, device=dev).index_add_(0, rows.to(dev), vals.to(dev))
            empty = cnt == 0
            outs.append(torch.where(empty[:, None], torch.zeros_like(theta), theta))
        T = torch.cat(outs) if outs else torch.zeros((0, st.lam.shape[0]), dtype=torch.float64)
        return df.withColumnData(self.getOrDefault(self.topicDistributionCol), U.vec_out(T))

    def _save_data(self, path):
        import pyarrow as pa
        write_data(path, {"vocabSize": pa.array([self._V], pa.int32()),
                          "topicsMatrix": mat_col([DenseMatrix.from_array(self._lam.T)]),
                          "docConcentration": vec_col([DenseVector(self._alpha)]),
                          "topicConcentration": pa.array([self._eta]),
                          "gammaShape": pa.array([100.0])})

    @classmethod
    def _load_impl(cls, path, meta):
        from .util import matrix_from_struct, vector_from_struct
        t = read_data(path).to_pylist()[0]
        lam = matrix_from_struct(t["topicsMatrix"]).toArray().T
        m = cls._from(lam, vector_from_struct(t["docConcentration"]).toArray(), t["topicConcentration"],
                      t["vocabSize"])
        apply_metadata(m, meta)
        return m


LocalLDAModel = LDAModel


@register("org.apache.spark.ml.clustering.DistributedLDAModel")
class DistributedLDAModel(LDAModel):
    """Model of ``LDA(optimizer="em")`` (Spark's DistributedLDAModel).  The topics matrix is
    small (k x vocabSize) and replicated on every rank, so "distributed" only records how it
    was trained; the extra EM diagnostics are kept and ``toLocal()`` drops them."""

    def __init__(self):
        super().__init__()
        self._train_ll = float("nan")
        self._log_prior = float("nan")

    def isDistributed(self):
        return True

    def trainingLogLikelihood(self) -> float:
        """Variational bound on the training corpus at the final iteration."""
        return self._train_ll

    def logPrior(self) -> float:
        """log p(topics | topicConcentration) + log p(docConcentration) terms of the bound."""
        return self._log_prior

    def toLocal(self) -> LDAModel:
        m = LDAModel._from(self._lam, self._alpha, self._eta, self._V)
        m._paramMap.update(self._paramMap)
        return m

    def getCheckpointFiles(self):
        return []

    def deleteCheckpointFiles(self):
        pass


# ===================================================== PowerIterationClustering
@register("org.apache.spark.ml.clustering.PowerIterationClustering")
class PowerIterationClustering(Params, MLWritable, MLReadable):
    """Power Iteration Clustering (PIC), a scalable graph clustering algorithm developed by
    Lin and Cohen. From the abstract: PIC finds a very low-dimensional embedding of a dataset
    using truncated power iteration on a normalized pair-wise similarity matrix of the data.
    Call ``assignClusters`` on a (src, dst, weight) edge DataFrame."""

    k = shared("k", "The number of clusters to create. Must be > 1.", TypeConverters.toInt)
    initMode = shared("initMode", "The initialization algorithm. This can be either 'random' to use a random "
                                  "vector as vertex properties, or 'degree' to use a normalized sum of similarities "
                                  "with other vertices.  Supported options: 'random' and 'degree'.",
                      TypeConverters.toString)
    srcCol = shared("srcCol", "Name of the input column for source vertex IDs.", TypeConverters.toString)
    dstCol = shared("dstCol", "Name of the input column for destination vertex IDs.", TypeConverters.toString)
    maxIter = shared("maxIter", "max number of iterations (>= 0).", TypeConverters.toInt)
    weightCol = shared("weightCol", "weight column name. If this is not set or empty, we treat all instance "
                                    "weights as 1.0.", TypeConverters.toString)

    @keyword_only
    def __init__(self, *, k=2, maxIter=20, initMode="random", srcCol="src", dstCol="dst", weightCol=None):
        super().__init__()
        self._setDefault(k=2, maxIter=20, initMode="random", srcCol="src", dstCol="dst")
        self._set(**self._input_kwargs)

    def assignClusters(self, dataset):
        g = self.getOrDefault
        comm = dataset.comm
        src = U.numeric_column(dataset, g(self.srcCol), torch.float64).long()
        dst = U.numeric_column(dataset, g(self.dstCol), torch.float64).long()
        if self.isDefined(self.weightCol) and g(self.weightCol):
            w = U.numeric_column(dataset, g(self.weightCol))
        else:
            w = torch.ones(src.shape[0], dtype=torch.float64, device=src.device)
        if comm.world_size > 1:
            src, dst, w = comm.all_gather_v(src), comm.all_gather_v(dst), comm.all_gather_v(w)
        ids, inv = torch.unique(torch.cat([src, dst]), return_inverse=True)
        n = ids.shape[0]
        e = src.shape[0]
        v = CE.power_iteration_embedding(inv[:e], inv[e:], w.to(torch.float64), n, g(self.maxIter),
                                         g(self.initMode), 0)
        from ..models.kmeans import fit_kmeans, predict
        from ..parallel.comm import LocalComm
        k = g(self.k)
        r = fit_kmeans(LocalComm(v.device), v[:, None].to(torch.float64), k, 20, 1e-4, 0, "k-means||", 2)
        a = predict(v[:, None].to(torch.float64), r.centers)
        from ..session import Session
        s = Session.getOrCreate()
        # every rank computes the same assignment; rank r keeps its slice of the ids
        lo, hi = (n * comm.rank) // comm.world_size, (n * (comm.rank + 1)) // comm.world_size
        cols = OrderedDict(id=C.NumericColumn(ids[lo:hi].to(torch.int64)),
                           cluster=C.NumericColumn(a[lo:hi].to(torch.int32)))
        return DataFrame(dataset.session if hasattr(dataset, "session") else s, cols)


_ = (math, HasProbabilityCol, HasTol)
