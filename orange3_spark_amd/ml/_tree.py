"""Tree estimators/models (DecisionTree*, RandomForest*, GBT*), re-exported by
``ml.classification`` and ``ml.regression`` so the reflective widgets list them."""
from __future__ import annotations

import numpy as np
import torch

from ..runtime.tracing import trace

from ..frame import column as C
from ..models import trees as TR
from . import common as U
from .base import Estimator, Model
from .linalg import DenseVector, SparseVector
from .param import (HasCheckpointInterval, HasFeaturesCol, HasLabelCol, HasMaxIter, HasPredictionCol,
                    HasProbabilityCol, HasRawPredictionCol, HasSeed, HasStepSize, HasThresholds, HasWeightCol,
                    TypeConverters, keyword_only, shared)
from .util import MLReadable, MLWritable, apply_metadata, read_data, register, write_data


class _DecisionTreeParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasSeed, HasWeightCol,
                          HasCheckpointInterval):
    maxDepth = shared("maxDepth", "Maximum depth of the tree. (>= 0) E.g., depth 0 means 1 leaf node; depth 1 "
                                  "means 1 internal node + 2 leaf nodes. Must be in range [0, 30].",
                      TypeConverters.toInt)
    maxBins = shared("maxBins", "Max number of bins for discretizing continuous features.  Must be >=2 and >= "
                                "number of categories for any categorical feature.", TypeConverters.toInt)
    minInstancesPerNode = shared("minInstancesPerNode", "Minimum number of instances each child must have after "
                                 "split. If a split causes the left or right child to have fewer than "
                                 "minInstancesPerNode, the split will be discarded as invalid. Should be >= 1.",
                                 TypeConverters.toInt)
    minWeightFractionPerNode = shared("minWeightFractionPerNode", "Minimum fraction of the weighted sample count "
                                      "that each child must have after split. Should be in [0.0, 0.5).",
                                      TypeConverters.toFloat)
    minInfoGain = shared("minInfoGain", "Minimum information gain for a split to be considered at a tree node.",
                         TypeConverters.toFloat)
    maxMemoryInMB = shared("maxMemoryInMB", "Maximum memory in MB allocated to histogram aggregation.",
                           TypeConverters.toInt)
    cacheNodeIds = shared("cacheNodeIds", "If false, the algorithm will pass trees to executors to match instances "
                                          "with nodes. If true, the algorithm will cache node IDs for each instance.",
                          TypeConverters.toBoolean)
    impurity = shared("impurity", "Criterion used for information gain calculation (case-insensitive). "
                                  "Supported options: entropy, gini, variance", TypeConverters.toString)
    leafCol = shared("leafCol", "Leaf indices column name. Predicted leaf index of each instance in each tree by "
                                "preorder.", TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(maxDepth=5, maxBins=32, minInstancesPerNode=1, minWeightFractionPerNode=0.0,
                         minInfoGain=0.0, maxMemoryInMB=256, cacheNodeIds=False, checkpointInterval=10,
                         leafCol="", seed=0)


class _EnsembleParams(_DecisionTreeParams):
    subsamplingRate = shared("subsamplingRate", "Fraction of the training data used for learning each decision "
                             "tree, in range (0, 1].", TypeConverters.toFloat)
    featureSubsetStrategy = shared("featureSubsetStrategy", "The number of features to consider for splits at "
                                   "each tree node. Supported options: 'auto' (choose automatically for task: If "
                                   "numTrees == 1, set to 'all'. If numTrees > 1 (forest), set to 'sqrt' for "
                                   "classification and to 'onethird' for regression), 'all' (use all features), "
                                   "'onethird' (use 1/3 of the features), 'sqrt' (use sqrt(number of features)), "
                                   "'log2' (use log2(number of features)), 'n' (when n is in the range (0, 1.0], "
                                   "use n * number of features. When n is in the range (1, number of features), "
                                   "use n features). default = 'auto'", TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(subsamplingRate=1.0, featureSubsetStrategy="auto")


class _RFParams(_EnsembleParams):
    numTrees = shared("numTrees", "Number of trees to train (>= 1).", TypeConverters.toInt)
    bootstrap = shared("bootstrap", "Whether bootstrap samples are used when building trees.",
                       TypeConverters.toBoolean)

    def __init__(self):
        super().__init__()
        self._setDefault(numTrees=20, bootstrap=True)


class _GBTParams(_EnsembleParams, HasMaxIter, HasStepSize):
    validationTol = shared("validationTol", "Threshold for stopping early when fit with validation is used. If the "
                           "error rate on the validation input changes by less than the validationTol, then "
                           "learning will stop early (before `maxIter`).", TypeConverters.toFloat)
    validationIndicatorCol = shared("validationIndicatorCol", "name of the column that indicates whether each row "
                                    "is for training or for validation. False indicates training; true indicates "
                                    "validation.", TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(maxIter=20, stepSize=0.1, validationTol=0.01, featureSubsetStrategy="all")


# ----------------------------------------------------------------------------- training
def _prepare(df, est, classification: bool, split_rows: torch.Tensor | None = None):
    """split_rows: optional bool mask of the rows the split candidates come from (GBT with
    a validation indicator: the training rows only, as Spark splits the dataset first)."""
    from ..frame.spill import RowBlocks, SpilledVectorColumn
    g = est.getOrDefault
    col = U.features_column(df, g(est.featuresCol))
    if isinstance(col, SpilledVectorColumn) and col.spilled_rows and split_rows is None:
        X = RowBlocks(col)                  # MEMORY_AND_DISK rows: sampled + streamed, never resident
    else:
        X = U.dense_features(df, g(est.featuresCol))
        if not X.is_cuda:
            X = X.to(torch.float64)
        elif X.dtype != torch.bfloat16:      # bf16 rows are binned as they are (no fp32 copy)
            X = X.float()
    y = U.numeric_column(df, g(est.labelCol), torch.float64)
    w = U.weights_or_none(df, est)
    comm = df.comm
    Xs = X if split_rows is None else X[split_rows.to(X.device)]
    with trace("tree.find_splits"):
        splits = TR.find_splits(comm, Xs, g(est.maxBins), g(est.seed))
    with trace("tree.bin_features"):
        bins = TR.bin_features(X, splits)
    k = U.num_classes(comm, y) if classification else 0
    rows = df._global_rows()
    return X, y.float(), None if w is None else w.float(), bins, splits, k, rows


def _min_inst(est, df, w):
    return float(est.getOrDefault(est.minInstancesPerNode))


def _min_wfrac(est) -> float:
    v = float(est.getOrDefault(est.minWeightFractionPerNode))
    if not 0.0 <= v < 0.5:
        raise ValueError(f"minWeightFractionPerNode must be in [0.0, 0.5), got {v}")
    return v


def _validation_mask(est, df):
    """Spark validationIndicatorCol (GBT): True rows validate, False rows train."""
    if not est.isDefined(est.validationIndicatorCol):
        return None
    vc = est.getOrDefault(est.validationIndicatorCol)
    if not vc:
        return None
    return U.numeric_column(df, vc, torch.float64) != 0


# ----------------------------------------------------------------------------- models
class _TreeModelMixin:
    _ens: TR.Ensemble = None
    numFeatures = 0

    @property
    def trees(self):
        return [DecisionTreeRegressionModel._of_tree(t) if self._ens.kind == "gbt" else
                (DecisionTreeClassificationModel._of_tree(t, self._ens.num_classes) if self._ens.num_classes
                 else DecisionTreeRegressionModel._of_tree(t)) for t in self._ens.trees]

    @property
    def treeWeights(self):
        return list(self._ens.weights)

    def predictLeaf(self, value):
        """Leaf index of ``value`` (a feature vector) in every tree, as a DenseVector.
        Leaves are numbered 0..numLeaves-1 in preorder (left to right), Spark's
        ``Node.predictLeaf`` / ``leafCol`` numbering."""
        x = np.asarray(value.toArray() if hasattr(value, "toArray") else value, dtype=np.float64)[None, :]
        X = torch.from_numpy(x)
        return DenseVector([float(t.leaf_index(X)[0]) for t in self._ens.trees])

    def _transform(self, df):
        out = super()._transform(df)
        lc = self.getOrDefault(self.leafCol) if self.hasParam("leafCol") and self.isDefined(self.leafCol) else ""
        if lc:                                  # Spark leafCol: per-tree preorder leaf indices
            X = self._X(df)
            out = out.withColumnData(lc, U.vec_out(torch.stack([t.leaf_index(X) for t in self._ens.trees], 1)))
        return out

    @property
    def getNumTrees(self):
        return len(self._ens.trees)

    @property
    def totalNumNodes(self):
        return int(sum(t.numNodes for t in self._ens.trees))

    @property
    def featureImportances(self):
        imp = np.zeros(self.numFeatures)
        for t in self._ens.trees:
            imp += t.feature_importance()
        s = imp.sum()
        imp = imp / s if s > 0 else imp
        nz = np.nonzero(imp)[0]
        return SparseVector(self.numFeatures, nz, imp[nz])

    @property
    def toDebugString(self):
        lines = [f"{type(self).__name__}: uid={self.uid}, numTrees={len(self._ens.trees)}, "
                 f"numFeatures={self.numFeatures}"]
        for i, t in enumerate(self._ens.trees):
            lines.append(f"  Tree {i} (weight {self._ens.weights[i]}):")
            lines += _tree_lines(t, 1, 4)
        return "\n".join(lines)

    def _X(self, df):
        X = U.dense_features(df, self.getOrDefault(self.featuresCol))
        return X.float() if X.is_cuda else X.to(torch.float64)

    # persistence, Spark's layouts: ensembles (RF / GBT) write data/ = (treeID, nodeData)
    # rows + treesMetadata/ = (treeID, metadata JSON, weights); a single decision tree
    # writes its NodeData rows flat in data/ (DecisionTreeModelReadWrite)
    def _save_data(self, path):
        import json as _json
        import pyarrow as pa
        from .util import SPARK_VERSION
        trees = self._ens.trees
        if self._ens.kind == "dt":
            write_data(path, pa.Table.from_pylist(_node_records(trees[0]), schema=pa.schema(list(_node_type()))),
                       non_null=_NODE_NON_NULL)
            return
        recs = [{"treeID": tid, "nodeData": r} for tid, t in enumerate(trees) for r in _node_records(t)]
        write_data(path, pa.Table.from_pylist(recs, schema=_ens_schema()), non_null=("treeID",))
        member = ("org.apache.spark.ml.regression.DecisionTreeRegressionModel"
                  if self._ens.kind == "gbt" or self._ens.num_classes == 0
                  else "org.apache.spark.ml.classification.DecisionTreeClassificationModel")
        tm = [{"treeID": i, "weights": float(w),
               "metadata": _json.dumps({"class": member, "timestamp": 0, "sparkVersion": SPARK_VERSION,
                                        "uid": f"{self.uid}_tree{i}", "paramMap": {}, "defaultParamMap": {}},
                                       separators=(",", ":"))}
              for i, w in enumerate(self._ens.weights)]
        tmt = pa.table({"treeID": pa.array([r["treeID"] for r in tm], pa.int32()),
                        "metadata": pa.array([r["metadata"] for r in tm], pa.string()),
                        "weights": pa.array([r["weights"] for r in tm], pa.float64())})
        write_data(path, tmt, subdir="treesMetadata", non_null=("treeID", "weights"))

    def _extra_metadata(self):
        meta = {"numFeatures": self.numFeatures}
        if self._ens.kind != "dt":
            meta["numTrees"] = len(self._ens.trees)
        if self._ens.num_classes and self._ens.kind != "gbt":
            meta["numClasses"] = self._ens.num_classes
        return meta

    @classmethod
    def _load_impl(cls, path, meta):
        table = read_data(path)
        F = meta.get("numFeatures", 0)
        name = meta["class"].rsplit(".", 1)[-1]
        kind = "gbt" if name.startswith("GBT") else ("dt" if name.startswith("DecisionTree") else "rf")
        kind = meta.get("ensembleKind", kind)
        regression = kind == "gbt" or "Regression" in name
        if "treeID" in table.column_names:
            data = table.to_pylist()
            tm = sorted(read_data(path, "treesMetadata").to_pylist(), key=lambda r: r["treeID"])
            by_tree = {}
            for r in data:
                by_tree.setdefault(r["treeID"], []).append(r["nodeData"])
            nodes = [x["nodeData"] for x in data]
            weights = [r["weights"] for r in tm]
        else:                                 # single tree: flat NodeData rows
            nodes = table.to_pylist()
            by_tree = {0: nodes}
            weights = [1.0]
        trees = [_tree_from_records(by_tree[i], F, regression) for i in sorted(by_tree)]
        if "numClasses" in meta:
            ncls = meta["numClasses"]
        elif name == "GBTClassificationModel":
            ncls = 2
        else:
            ncls = 0 if regression else max(len(x["impurityStats"]) for x in nodes)
        m = cls()
        m._ens = TR.Ensemble(trees, weights, kind, ncls)
        m.numFeatures = F
        apply_metadata(m, meta)
        return m


def _tree_lines(t: TR.Tree, nid: int, indent: int) -> list:
    pad = " " * indent
    if t.feature[nid] < 0 or 2 * nid >= len(t.feature) or t.count[2 * nid] == 0:
        v = t.value[nid]
        return [f"{pad}Predict: {float(np.argmax(v)) if len(v) > 1 else float(v[0])}"]
    f, thr = t.feature[nid], t.threshold[nid]
    return ([f"{pad}If (feature {f} <= {thr})"] + _tree_lines(t, 2 * nid, indent + 1) +
            [f"{pad}Else (feature {f} > {thr})"] + _tree_lines(t, 2 * nid + 1, indent + 1))


def _is_leaf(t, nid):
    return t.feature[nid] < 0 or 2 * nid >= len(t.feature) or t.count[2 * nid] == 0


def _node_records(t: TR.Tree) -> list:
    """Spark NodeData rows in preorder (ids 0..m-1, children -1 for leaves)."""
    recs = []

    def visit(nid):
        my = len(recs)
        v = t.value[nid]
        c = float(t.count[nid])
        if len(v) > 1:                       # classification: class counts (gini / entropy)
            stats = [float(x) for x in v * c]
        else:                                # regression (variance): [count, sum, sum of squares]
            mu = float(v[0])
            stats = [c, c * mu, c * (float(t.impurity[nid]) + mu * mu)]
        rec = {"id": my, "prediction": float(np.argmax(v)) if len(v) > 1 else float(v[0]),
               "impurity": float(t.impurity[nid]), "impurityStats": stats,
               "rawCount": int(round(t.count[nid])), "gain": float(t.gain[nid]) if not _is_leaf(t, nid) else -1.0,
               "leftChild": -1, "rightChild": -1,
               "split": {"featureIndex": -1, "leftCategoriesOrThreshold": [], "numCategories": -1}}
        recs.append(rec)
        if not _is_leaf(t, nid):
            rec["split"] = {"featureIndex": int(t.feature[nid]),
                            "leftCategoriesOrThreshold": [float(t.threshold[nid])], "numCategories": -1}
            rec["leftChild"] = visit(2 * nid)
            rec["rightChild"] = visit(2 * nid + 1)
        return my
    visit(1)
    return recs


def _tree_from_records(recs, F, regression: bool = False) -> TR.Tree:
    """Spark NodeData rows -> Tree.  ``regression``: variance trees (GBT members and the
    regressors), whose impurityStats are [count, sum, sum of squares] and whose node value is
    ``prediction``; otherwise impurityStats are class counts."""
    by_id = {r["id"]: r for r in recs}
    depth = 0

    def d(i, k):
        nonlocal depth
        depth = max(depth, k)
        r = by_id[i]
        if r["leftChild"] >= 0:
            d(r["leftChild"], k + 1)
            d(r["rightChild"], k + 1)
    d(0, 0)
    size = 2 ** (depth + 1)
    S = 1 if regression else max(1, max(len(r["impurityStats"]) for r in recs))
    feat = -np.ones(size, dtype=np.int64)
    thr = np.zeros(size)
    val = np.zeros((size, S))
    imp = np.zeros(size)
    gain = np.zeros(size)
    cnt = np.zeros(size)

    def fill(i, nid):
        r = by_id[i]
        st = np.array(r["impurityStats"], dtype=np.float64)
        if S > 1:
            tot = st.sum()
            val[nid] = st / tot if tot > 0 else st
        else:
            val[nid, 0] = r["prediction"]
        imp[nid], cnt[nid] = r["impurity"], max(r["rawCount"], 1)
        if r["leftChild"] >= 0:
            feat[nid] = r["split"]["featureIndex"]
            thr[nid] = r["split"]["leftCategoriesOrThreshold"][0]
            gain[nid] = r["gain"]
            fill(r["leftChild"], 2 * nid)
            fill(r["rightChild"], 2 * nid + 1)
    fill(0, 1)
    return TR.Tree(feat, thr, np.zeros(size, dtype=np.int64), val, imp, gain, cnt, F)


_NODE_NON_NULL = ("id", "prediction", "impurity", "rawCount", "gain", "leftChild", "rightChild")


def _node_type():
    """Spark's NodeData case class (primitive fields NOT NULL) with its SplitData struct."""
    import pyarrow as pa
    split = pa.struct([pa.field("featureIndex", pa.int32(), False),
                       ("leftCategoriesOrThreshold", pa.list_(pa.field("element", pa.float64(), False))),
                       pa.field("numCategories", pa.int32(), False)])
    return pa.struct([pa.field("id", pa.int32(), False), pa.field("prediction", pa.float64(), False),
                      pa.field("impurity", pa.float64(), False), ("impurityStats", pa.list_(pa.field("element", pa.float64(), False))),
                      pa.field("rawCount", pa.int64(), False), pa.field("gain", pa.float64(), False),
                      pa.field("leftChild", pa.int32(), False), pa.field("rightChild", pa.int32(), False),
                      ("split", split)])


def _ens_schema():
    import pyarrow as pa
    return pa.schema([pa.field("treeID", pa.int32(), False), ("nodeData", _node_type())])


class _TreeClassifierModel(_TreeModelMixin, U.ProbabilisticClassifierMixin, Model, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self.numClasses = 2
        self._ens = TR.Ensemble([], [], "rf", 2)

    def _features_for_predict(self, df, name):
        return self._X(df)

    def _raw(self, X):
        ens = self._ens
        if ens.kind == "gbt":
            F = sum(w * t.predict_value(X)[:, 0] for t, w in zip(ens.trees, ens.weights))
            return torch.stack([-F, F], 1)
        probs = [t.predict_value(X) for t in ens.trees]
        if ens.kind == "dt":
            return probs[0] * 1.0
        return torch.stack(probs).sum(0)

    def evaluate(self, df):
        """Spark >= 3.1 tree-classifier summary on ``df``: binary (ROC / PR curves, AUC)
        for two classes, multiclass metrics otherwise."""
        from . import _summary as S
        g = self.getOrDefault
        kw = dict(labelCol=g(self.labelCol), predictionCol=g(self.predictionCol),
                  weightCol=g(self.weightCol) if self.isDefined(self.weightCol) and g(self.weightCol) else None)
        pred = (lambda: self.transform(df))
        if self.numClasses == 2:
            return S.BinaryClassificationSummary(pred, scoreCol=g(self.probabilityCol), **kw)
        return S.ClassificationSummary(pred, **kw)

    def _raw2prob(self, raw):
        if self._ens.kind == "gbt":
            p = 1.0 / (1.0 + torch.exp(-2.0 * raw[:, 1]))
            return torch.stack([1 - p, p], 1)
        s = raw.sum(1, keepdim=True)
        return raw / torch.where(s > 0, s, torch.ones_like(s))


class _TreeRegressorModel(_TreeModelMixin, U.PredictionModelMixin, Model, MLWritable, MLReadable):
    def __init__(self):
        super().__init__()
        self._ens = TR.Ensemble([], [], "rf", 0)

    def _predict_tensor(self, X):
        X = X.float() if X.is_cuda else X.to(torch.float64)
        ens = self._ens
        vals = [w * t.predict_value(X)[:, 0] for t, w in zip(ens.trees, ens.weights)]
        s = sum(vals)
        return s / len(vals) if ens.kind == "rf" else s


# ----------------------------------------------------------------------------- classifiers
@register("org.apache.spark.ml.classification.DecisionTreeClassifier")
class DecisionTreeClassifier(Estimator, _DecisionTreeParams, HasProbabilityCol, HasRawPredictionCol, HasThresholds,
                             MLWritable, MLReadable):
    """Decision tree learning algorithm for classification (gini/entropy), level-wise
    with LDS histogram kernels and one histogram all-reduce per level."""
    _warm_family = "trees"          # runtime/warmup.py lazy warm-up

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction",
                 probabilityCol="probability", rawPredictionCol="rawPrediction", maxDepth=5, maxBins=32,
                 minInstancesPerNode=1, minInfoGain=0.0, maxMemoryInMB=256, cacheNodeIds=False,
                 checkpointInterval=10, impurity="gini", seed=None, weightCol=None, leafCol="",
                 minWeightFractionPerNode=0.0):
        super().__init__()
        self._setDefault(impurity="gini")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        X, y, w, bins, splits, k, rows = _prepare(df, self, True)
        tb = TR.TreeBuilder(df.comm, bins, splits, y, w, g(self.impurity).lower(), max(k, 2), g(self.maxDepth),
                            _min_inst(self, df, w), g(self.minInfoGain), 1.0, g(self.seed),
                            min_weight_fraction=_min_wfrac(self))
        tree, _ = tb.build()
        m = DecisionTreeClassificationModel._of_tree(tree, max(k, 2))
        return m._with_parent(self)


@register("org.apache.spark.ml.classification.DecisionTreeClassificationModel")
class DecisionTreeClassificationModel(_TreeClassifierModel, _DecisionTreeParams, HasProbabilityCol,
                                      HasRawPredictionCol, HasThresholds):
    @classmethod
    def _of_tree(cls, tree, k):
        m = cls()
        m._ens = TR.Ensemble([tree], [1.0], "dt", k)
        m.numClasses, m.numFeatures = k, tree.num_features
        return m

    @property
    def depth(self):
        return self._ens.trees[0].depth

    @property
    def numNodes(self):
        return self._ens.trees[0].numNodes


@register("org.apache.spark.ml.classification.RandomForestClassifier")
class RandomForestClassifier(Estimator, _RFParams, HasProbabilityCol, HasRawPredictionCol, HasThresholds,
                             MLWritable, MLReadable):
    """Random forest learning algorithm for classification (bootstrap via Poisson row
    weights keyed on (seed, global row), per-node feature subsets)."""
    _warm_family = "trees"          # runtime/warmup.py lazy warm-up

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction",
                 probabilityCol="probability", rawPredictionCol="rawPrediction", maxDepth=5, maxBins=32,
                 minInstancesPerNode=1, minInfoGain=0.0, maxMemoryInMB=256, cacheNodeIds=False,
                 checkpointInterval=10, impurity="gini", numTrees=20, featureSubsetStrategy="auto", seed=None,
                 subsamplingRate=1.0, leafCol="", minWeightFractionPerNode=0.0, weightCol=None, bootstrap=True):
        super().__init__()
        self._setDefault(impurity="gini")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        X, y, w, bins, splits, k, rows = _prepare(df, self, True)
        ff = TR.feature_fraction_for(g(self.featureSubsetStrategy), X.shape[1], True, g(self.numTrees))
        ens = TR.fit_forest(df.comm, bins, splits, y, w, g(self.numTrees), g(self.impurity).lower(), max(k, 2),
                            g(self.maxDepth), _min_inst(self, df, w), g(self.minInfoGain), g(self.subsamplingRate),
                            ff, g(self.seed), rows, g(self.bootstrap),
                            min_weight_fraction=_min_wfrac(self))
        m = RandomForestClassificationModel()
        m._ens, m.numClasses, m.numFeatures = ens, max(k, 2), X.shape[1]
        return m._with_parent(self)


@register("org.apache.spark.ml.classification.RandomForestClassificationModel")
class RandomForestClassificationModel(_TreeClassifierModel, _RFParams, HasProbabilityCol, HasRawPredictionCol,
                                      HasThresholds):
    pass


@register("org.apache.spark.ml.classification.GBTClassifier")
class GBTClassifier(Estimator, _GBTParams, HasProbabilityCol, HasRawPredictionCol, HasThresholds, MLWritable,
                    MLReadable):
    """Gradient-Boosted Trees (GBTs) learning algorithm for classification (binary, logistic
    loss; Spark semantics: tree 0 on labels, later trees on pseudo-residuals * stepSize)."""
    _warm_family = "trees"          # runtime/warmup.py lazy warm-up

    lossType = shared("lossType", "Loss function which GBT tries to minimize (case-insensitive). Supported "
                                  "options: logistic", TypeConverters.toString)

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxDepth=5,
                 maxBins=32, minInstancesPerNode=1, minInfoGain=0.0, maxMemoryInMB=256, cacheNodeIds=False,
                 checkpointInterval=10, lossType="logistic", maxIter=20, stepSize=0.1, seed=None,
                 subsamplingRate=1.0, impurity="variance", featureSubsetStrategy="all", validationTol=0.01,
                 validationIndicatorCol=None, leafCol="", minWeightFractionPerNode=0.0, weightCol=None,
                 probabilityCol="probability", rawPredictionCol="rawPrediction"):
        super().__init__()
        self._setDefault(lossType="logistic", impurity="variance")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        val = _validation_mask(self, df)
        X, y, w, bins, splits, k, rows = _prepare(df, self, True, None if val is None else ~val)
        if k > 2:
            raise ValueError(f"GBTClassifier currently only supports binary classification, got {k} classes")
        ff = TR.feature_fraction_for(g(self.featureSubsetStrategy), X.shape[1], True, 1)
        ens = TR.fit_gbt(df.comm, bins, splits, y, w, "logistic", g(self.maxIter), g(self.stepSize),
                         g(self.maxDepth), _min_inst(self, df, w), g(self.minInfoGain), g(self.subsamplingRate),
                         g(self.seed), ff, rows, True, validation=val,
                         validation_tol=g(self.validationTol), min_weight_fraction=_min_wfrac(self))
        m = GBTClassificationModel()
        m._ens, m.numClasses, m.numFeatures = ens, 2, X.shape[1]
        m.trainingLossHistory = ens.losses
        return m._with_parent(self)


@register("org.apache.spark.ml.classification.GBTClassificationModel")
class GBTClassificationModel(_TreeClassifierModel, _GBTParams, HasProbabilityCol, HasRawPredictionCol,
                             HasThresholds):
    lossType = GBTClassifier.lossType

    def __init__(self):
        super().__init__()
        self._ens = TR.Ensemble([], [], "gbt", 2)


# ----------------------------------------------------------------------------- regressors
@register("org.apache.spark.ml.regression.DecisionTreeRegressor")
class DecisionTreeRegressor(Estimator, _DecisionTreeParams, MLWritable, MLReadable):
    """Decision tree learning algorithm for regression (variance impurity)."""
    _warm_family = "trees"          # runtime/warmup.py lazy warm-up

    varianceCol = shared("varianceCol", "column name for the biased sample variance of prediction.",
                         TypeConverters.toString)

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxDepth=5,
                 maxBins=32, minInstancesPerNode=1, minInfoGain=0.0, maxMemoryInMB=256, cacheNodeIds=False,
                 checkpointInterval=10, impurity="variance", seed=None, varianceCol=None, weightCol=None,
                 leafCol="", minWeightFractionPerNode=0.0):
        super().__init__()
        self._setDefault(impurity="variance")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        X, y, w, bins, splits, _, rows = _prepare(df, self, False)
        tb = TR.TreeBuilder(df.comm, bins, splits, y, w, "variance", 1, g(self.maxDepth), _min_inst(self, df, w),
                            g(self.minInfoGain), 1.0, g(self.seed), min_weight_fraction=_min_wfrac(self))
        tree, _ = tb.build()
        return DecisionTreeRegressionModel._of_tree(tree)._with_parent(self)


@register("org.apache.spark.ml.regression.DecisionTreeRegressionModel")
class DecisionTreeRegressionModel(_TreeRegressorModel, _DecisionTreeParams):
    @classmethod
    def _of_tree(cls, tree):
        m = cls()
        m._ens = TR.Ensemble([tree], [1.0], "dt", 0)
        m.numFeatures = tree.num_features
        return m

    @property
    def depth(self):
        return self._ens.trees[0].depth

    @property
    def numNodes(self):
        return self._ens.trees[0].numNodes


@register("org.apache.spark.ml.regression.RandomForestRegressor")
class RandomForestRegressor(Estimator, _RFParams, MLWritable, MLReadable):
    """Random forest learning algorithm for regression."""
    _warm_family = "trees"          # runtime/warmup.py lazy warm-up

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxDepth=5,
                 maxBins=32, minInstancesPerNode=1, minInfoGain=0.0, maxMemoryInMB=256, cacheNodeIds=False,
                 checkpointInterval=10, impurity="variance", subsamplingRate=1.0, seed=None, numTrees=20,
                 featureSubsetStrategy="auto", leafCol="", minWeightFractionPerNode=0.0, weightCol=None,
                 bootstrap=True):
        super().__init__()
        self._setDefault(impurity="variance")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        X, y, w, bins, splits, _, rows = _prepare(df, self, False)
        ff = TR.feature_fraction_for(g(self.featureSubsetStrategy), X.shape[1], False, g(self.numTrees))
        ens = TR.fit_forest(df.comm, bins, splits, y, w, g(self.numTrees), "variance", 1, g(self.maxDepth),
                            _min_inst(self, df, w), g(self.minInfoGain), g(self.subsamplingRate), ff, g(self.seed),
                            rows, g(self.bootstrap), min_weight_fraction=_min_wfrac(self))
        ens.num_classes = 0
        m = RandomForestRegressionModel()
        m._ens, m.numFeatures = ens, X.shape[1]
        return m._with_parent(self)


@register("org.apache.spark.ml.regression.RandomForestRegressionModel")
class RandomForestRegressionModel(_TreeRegressorModel, _RFParams):
    pass


@register("org.apache.spark.ml.regression.GBTRegressor")
class GBTRegressor(Estimator, _GBTParams, MLWritable, MLReadable):
    """Gradient-Boosted Trees (GBTs) learning algorithm for regression (squared/absolute loss)."""
    _warm_family = "trees"          # runtime/warmup.py lazy warm-up

    lossType = shared("lossType", "Loss function which GBT tries to minimize (case-insensitive). Supported "
                                  "options: squared, absolute", TypeConverters.toString)

    @keyword_only
    def __init__(self, *, featuresCol="features", labelCol="label", predictionCol="prediction", maxDepth=5,
                 maxBins=32, minInstancesPerNode=1, minInfoGain=0.0, maxMemoryInMB=256, cacheNodeIds=False,
                 subsamplingRate=1.0, checkpointInterval=10, lossType="squared", maxIter=20, stepSize=0.1,
                 seed=None, impurity="variance", featureSubsetStrategy="all", validationTol=0.01,
                 validationIndicatorCol=None, leafCol="", minWeightFractionPerNode=0.0, weightCol=None):
        super().__init__()
        self._setDefault(lossType="squared", impurity="variance")
        self._set(**self._input_kwargs)

    def _fit(self, df):
        g = self.getOrDefault
        val = _validation_mask(self, df)
        X, y, w, bins, splits, _, rows = _prepare(df, self, False, None if val is None else ~val)
        ff = TR.feature_fraction_for(g(self.featureSubsetStrategy), X.shape[1], False, 1)
        ens = TR.fit_gbt(df.comm, bins, splits, y, w, g(self.lossType).lower(), g(self.maxIter), g(self.stepSize),
                         g(self.maxDepth), _min_inst(self, df, w), g(self.minInfoGain), g(self.subsamplingRate),
                         g(self.seed), ff, rows, False, validation=val,
                         validation_tol=g(self.validationTol), min_weight_fraction=_min_wfrac(self))
        m = GBTRegressionModel()
        m._ens, m.numFeatures = ens, X.shape[1]
        m.trainingLossHistory = ens.losses
        return m._with_parent(self)


@register("org.apache.spark.ml.regression.GBTRegressionModel")
class GBTRegressionModel(_TreeRegressorModel, _GBTParams):
    lossType = GBTRegressor.lossType

    def __init__(self):
        super().__init__()
        self._ens = TR.Ensemble([], [], "gbt", 0)


_ = (C, DenseVector)
