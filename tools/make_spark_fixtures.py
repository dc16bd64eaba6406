#!/usr/bin/env python
"""Write tests/fixtures/spark_models/: model directories laid out byte-for-byte the way
Spark 3.5 ``MLWriter``s write them, built by hand from Spark's documented schemas -- NOT
with this framework's writers -- so the loaders are pinned to Spark's format rather than
to their own output.

Layout per model (Spark ``DefaultParamsWriter`` + model writers):
  metadata/part-00000   one JSON line: class, timestamp, sparkVersion, uid, paramMap,
                        defaultParamMap (+ model extras: numFeatures/numTrees, rank, ...)
  data/part-*.parquet   Spark's case-class schema; vectors / matrices are the VectorUDT /
                        MatrixUDT sqlType structs; the parquet footer carries Spark's
                        ``org.apache.spark.sql.parquet.row.metadata`` schema JSON with the
                        UDT annotations (that is how Spark restores Vector columns)

Models: LogisticRegressionModel (binomial), KMeansModel, GBTClassificationModel (two
variance-impurity regression stumps + tree weights), ALSModel (user / item factor tables),
a PipelineModel (VectorAssembler -> LogisticRegressionModel), LinearSVCModel,
LinearRegressionModel, StandardScalerModel, StringIndexerModel (labelsArray),
RandomForestClassificationModel (two gini stumps, class-count impurityStats),
DecisionTreeClassificationModel (flat NodeData rows), NaiveBayesModel (multinomial: pi,
theta and a 0 x 0 sigma), MinMaxScalerModel, IDFModel, OneHotEncoderModel and
CountVectorizerModel.
"""
import json
import os
import shutil

import pyarrow as pa
import pyarrow.parquet as pq

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures", "spark_models")
TS = 1700000000000
VERSION = "3.5.1"

# ---------------------------------------------------------------- Spark SQL types (JSON)
VEC_SQL = {"type": "struct", "fields": [
    {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
    {"name": "size", "type": "integer", "nullable": True, "metadata": {}},
    {"name": "indices", "type": {"type": "array", "elementType": "integer", "containsNull": False},
     "nullable": True, "metadata": {}},
    {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
     "nullable": True, "metadata": {}}]}
MAT_SQL = {"type": "struct", "fields": [
    {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
    {"name": "numRows", "type": "integer", "nullable": False, "metadata": {}},
    {"name": "numCols", "type": "integer", "nullable": False, "metadata": {}},
    {"name": "colPtrs", "type": {"type": "array", "elementType": "integer", "containsNull": False},
     "nullable": True, "metadata": {}},
    {"name": "rowIndices", "type": {"type": "array", "elementType": "integer", "containsNull": False},
     "nullable": True, "metadata": {}},
    {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
     "nullable": True, "metadata": {}},
    {"name": "isTransposed", "type": "boolean", "nullable": False, "metadata": {}}]}
VEC_UDT = {"type": "udt", "class": "org.apache.spark.ml.linalg.VectorUDT", "pyClass": "pyspark.ml.linalg.VectorUDT",
           "sqlType": VEC_SQL}
MAT_UDT = {"type": "udt", "class": "org.apache.spark.ml.linalg.MatrixUDT", "pyClass": "pyspark.ml.linalg.MatrixUDT",
           "sqlType": MAT_SQL}

VEC_ARROW = pa.struct([pa.field("type", pa.int8(), False), ("size", pa.int32()), ("indices", pa.list_(pa.field("element", pa.int32(), False))),
                       ("values", pa.list_(pa.field("element", pa.float64(), False)))])
MAT_ARROW = pa.struct([pa.field("type", pa.int8(), False), pa.field("numRows", pa.int32(), False),
                       pa.field("numCols", pa.int32(), False), ("colPtrs", pa.list_(pa.field("element", pa.int32(), False))),
                       ("rowIndices", pa.list_(pa.field("element", pa.int32(), False))), ("values", pa.list_(pa.field("element", pa.float64(), False))),
                       pa.field("isTransposed", pa.bool_(), False)])


def field(name, typ, nullable=True):
    return {"name": name, "type": typ, "nullable": nullable, "metadata": {}}


def write_meta(path, cls, uid, params, defaults, **extra):
    d = os.path.join(path, "metadata")
    os.makedirs(d, exist_ok=True)
    meta = {"class": cls, "timestamp": TS, "sparkVersion": VERSION, "uid": uid, "paramMap": params,
            "defaultParamMap": defaults}
    meta.update(extra)
    with open(os.path.join(d, "part-00000"), "w") as f:
        f.write(json.dumps(meta, separators=(",", ":")) + "\n")
    open(os.path.join(d, "_SUCCESS"), "w").close()


def write_parquet(path, sub, table: pa.Table, spark_fields):
    d = os.path.join(path, sub)
    os.makedirs(d, exist_ok=True)
    row_meta = json.dumps({"type": "struct", "fields": spark_fields}, separators=(",", ":"))
    table = table.replace_schema_metadata({"org.apache.spark.version": VERSION,
                                           "org.apache.spark.sql.parquet.row.metadata": row_meta})
    pq.write_table(table, os.path.join(d, "part-00000-0b3a7e3c-5f1e-4c7e-9d1e-2a1b3c4d5e6f-c000.snappy.parquet"),
                   compression="snappy")
    open(os.path.join(d, "_SUCCESS"), "w").close()


LR_DEFAULTS = {"aggregationDepth": 2, "elasticNetParam": 0.0, "family": "auto", "featuresCol": "features",
               "fitIntercept": True, "labelCol": "label", "maxBlockSizeInMB": 0.0, "maxIter": 100,
               "predictionCol": "prediction", "probabilityCol": "probability", "rawPredictionCol": "rawPrediction",
               "regParam": 0.0, "standardization": True, "threshold": 0.5, "tol": 1e-06}


def logistic(path, uid="LogisticRegression_4d3a1b2c5e6f"):
    write_meta(path, "org.apache.spark.ml.classification.LogisticRegressionModel", uid,
               {"maxIter": 25, "regParam": 0.01}, LR_DEFAULTS)
    t = pa.table({
        "numClasses": pa.array([2], pa.int32()),
        "numFeatures": pa.array([3], pa.int32()),
        "interceptVector": pa.array([{"type": 1, "size": None, "indices": None, "values": [0.3]}], VEC_ARROW),
        "coefficientMatrix": pa.array([{"type": 1, "numRows": 1, "numCols": 3, "colPtrs": None, "rowIndices": None,
                                        "values": [0.5, -1.25, 2.0], "isTransposed": True}], MAT_ARROW),
        "isMultinomial": pa.array([False], pa.bool_())})
    write_parquet(path, "data", t, [field("numClasses", "integer", False), field("numFeatures", "integer", False),
                                    field("interceptVector", VEC_UDT), field("coefficientMatrix", MAT_UDT),
                                    field("isMultinomial", "boolean", False)])


def kmeans(path):
    write_meta(path, "org.apache.spark.ml.clustering.KMeansModel", "KMeans_8a7b6c5d4e3f",
               {"k": 2, "seed": 7},
               {"distanceMeasure": "euclidean", "featuresCol": "features", "initMode": "k-means||", "initSteps": 2,
                "k": 2, "maxBlockSizeInMB": 0.0, "maxIter": 20, "predictionCol": "prediction",
                "seed": -1689246527, "solver": "auto", "tol": 0.0001})
    t = pa.table({"clusterIdx": pa.array([0, 1], pa.int32()),
                  "clusterCenter": pa.array([{"type": 1, "size": None, "indices": None, "values": [0.0, 0.0]},
                                             {"type": 1, "size": None, "indices": None, "values": [5.0, 5.0]}],
                                            VEC_ARROW)})
    write_parquet(path, "data", t, [field("clusterIdx", "integer", False), field("clusterCenter", VEC_UDT)])


SPLIT = pa.struct([pa.field("featureIndex", pa.int32(), False), ("leftCategoriesOrThreshold", pa.list_(pa.field("element", pa.float64(), False))),
                   pa.field("numCategories", pa.int32(), False)])
NODE = pa.struct([pa.field("id", pa.int32(), False), pa.field("prediction", pa.float64(), False),
                  pa.field("impurity", pa.float64(), False), ("impurityStats", pa.list_(pa.field("element", pa.float64(), False))),
                  pa.field("rawCount", pa.int64(), False), pa.field("gain", pa.float64(), False),
                  pa.field("leftChild", pa.int32(), False), pa.field("rightChild", pa.int32(), False),
                  ("split", SPLIT)])
SPLIT_SQL = {"type": "struct", "fields": [
    field("featureIndex", "integer", False),
    field("leftCategoriesOrThreshold", {"type": "array", "elementType": "double", "containsNull": False}),
    field("numCategories", "integer", False)]}
NODE_SQL = {"type": "struct", "fields": [
    field("id", "integer", False), field("prediction", "double", False), field("impurity", "double", False),
    field("impurityStats", {"type": "array", "elementType": "double", "containsNull": False}),
    field("rawCount", "long", False), field("gain", "double", False), field("leftChild", "integer", False),
    field("rightChild", "integer", False), field("split", SPLIT_SQL)]}


def _stump(feature, thr, left, right, n_left, n_right):
    """Variance-impurity regression stump as Spark NodeData rows (preorder ids)."""
    def stats(n, mean, var):
        return [float(n), n * mean, n * (var + mean * mean)]
    n = n_left + n_right
    mean = (n_left * left + n_right * right) / n
    var = (n_left * left * left + n_right * right * right) / n - mean * mean
    leaf_split = {"featureIndex": -1, "leftCategoriesOrThreshold": [], "numCategories": -1}
    return [
        {"id": 0, "prediction": mean, "impurity": var, "impurityStats": stats(n, mean, var), "rawCount": n,
         "gain": var, "leftChild": 1, "rightChild": 2,
         "split": {"featureIndex": feature, "leftCategoriesOrThreshold": [thr], "numCategories": -1}},
        {"id": 1, "prediction": left, "impurity": 0.0, "impurityStats": stats(n_left, left, 0.0), "rawCount": n_left,
         "gain": -1.0, "leftChild": -1, "rightChild": -1, "split": leaf_split},
        {"id": 2, "prediction": right, "impurity": 0.0, "impurityStats": stats(n_right, right, 0.0),
         "rawCount": n_right, "gain": -1.0, "leftChild": -1, "rightChild": -1, "split": leaf_split}]


def gbt(path):
    uid = "GBTClassifier_1a2b3c4d5e6f"
    defaults = {"cacheNodeIds": False, "checkpointInterval": 10, "featureSubsetStrategy": "all",
                "featuresCol": "features", "impurity": "variance", "labelCol": "label", "leafCol": "",
                "lossType": "logistic", "maxBins": 32, "maxDepth": 5, "maxIter": 20, "maxMemoryInMB": 256,
                "minInfoGain": 0.0, "minInstancesPerNode": 1, "minWeightFractionPerNode": 0.0,
                "predictionCol": "prediction", "probabilityCol": "probability", "rawPredictionCol": "rawPrediction",
                "seed": -1287390502, "stepSize": 0.1, "subsamplingRate": 1.0, "validationTol": 0.01}
    write_meta(path, "org.apache.spark.ml.classification.GBTClassificationModel", uid, {"maxIter": 2, "maxDepth": 1},
               defaults, numFeatures=2, numTrees=2)
    rows = [{"treeID": 0, "nodeData": r} for r in _stump(0, 0.5, -0.6, 0.8, 40, 60)] + \
        [{"treeID": 1, "nodeData": r} for r in _stump(1, 1.0, 0.2, -0.3, 70, 30)]
    t = pa.Table.from_pylist(rows, schema=pa.schema([pa.field("treeID", pa.int32(), False), ("nodeData", NODE)]))
    write_parquet(path, "data", t, [field("treeID", "integer", False), field("nodeData", NODE_SQL)])
    tree_meta = [json.dumps({"class": "org.apache.spark.ml.regression.DecisionTreeRegressionModel",
                             "timestamp": TS, "sparkVersion": VERSION, "uid": f"dtr_{i}",
                             "paramMap": {"maxDepth": 1, "impurity": "variance"}, "defaultParamMap": {}},
                            separators=(",", ":")) for i in range(2)]
    tm = pa.table({"treeID": pa.array([0, 1], pa.int32()), "metadata": pa.array(tree_meta, pa.string()),
                   "weights": pa.array([1.0, 0.1], pa.float64())})
    write_parquet(path, "treesMetadata", tm, [field("treeID", "integer", False), field("metadata", "string"),
                                              field("weights", "double", False)])


def als(path):
    # ALSModel holds only ALSModelParams (Spark copies the estimator's values of those)
    write_meta(path, "org.apache.spark.ml.recommendation.ALSModel", "ALS_9f8e7d6c5b4a",
               {"userCol": "user", "itemCol": "item", "coldStartStrategy": "nan"},
               {"blockSize": 4096, "coldStartStrategy": "nan", "itemCol": "item", "predictionCol": "prediction",
                "userCol": "user"},
               rank=2)
    arr = {"type": "array", "elementType": "float", "containsNull": False}
    for name, ids, feats in (("userFactors", [10, 20], [[1.0, 0.5], [0.0, 2.0]]),
                             ("itemFactors", [1, 2, 3], [[1.0, 1.0], [2.0, -1.0], [0.5, 0.25]])):
        t = pa.table({"id": pa.array(ids, pa.int32()), "features": pa.array(feats, pa.list_(pa.field("element", pa.float32(), False)))})
        write_parquet(path, name, t, [field("id", "integer", False), field("features", arr)])


def pipeline(path):
    uids = ["VectorAssembler_5c4b3a2d1e0f", "LogisticRegression_4d3a1b2c5e6f"]
    write_meta(path, "org.apache.spark.ml.PipelineModel", "PipelineModel_0a1b2c3d4e5f", {"stageUids": uids}, {},
               language="Python")
    write_meta(os.path.join(path, "stages", f"0_{uids[0]}"), "org.apache.spark.ml.feature.VectorAssembler", uids[0],
               {"inputCols": ["a", "b", "c"], "outputCol": "features"},
               {"handleInvalid": "error", "outputCol": f"{uids[0]}__output"})
    logistic(os.path.join(path, "stages", f"1_{uids[1]}"), uids[1])


def linear_svc(path):
    write_meta(path, "org.apache.spark.ml.classification.LinearSVCModel", "LinearSVC_3c2b1a0f9e8d",
               {"regParam": 0.1, "maxIter": 50},
               {"aggregationDepth": 2, "featuresCol": "features", "fitIntercept": True, "labelCol": "label",
                "maxBlockSizeInMB": 0.0, "maxIter": 100, "predictionCol": "prediction",
                "rawPredictionCol": "rawPrediction", "regParam": 0.0, "standardization": True, "threshold": 0.0,
                "tol": 1e-06})
    t = pa.table({"coefficients": pa.array([{"type": 1, "size": None, "indices": None, "values": [1.5, -0.5]}],
                                           VEC_ARROW),
                  "intercept": pa.array([-0.25], pa.float64())})
    write_parquet(path, "data", t, [field("coefficients", VEC_UDT), field("intercept", "double", False)])


def linear_regression(path):
    write_meta(path, "org.apache.spark.ml.regression.LinearRegressionModel", "LinearRegression_7e6d5c4b3a29",
               {"regParam": 0.0},
               {"aggregationDepth": 2, "elasticNetParam": 0.0, "epsilon": 1.35, "featuresCol": "features",
                "fitIntercept": True, "labelCol": "label", "loss": "squaredError", "maxBlockSizeInMB": 0.0,
                "maxIter": 100, "predictionCol": "prediction", "regParam": 0.0, "solver": "auto",
                "standardization": True, "tol": 1e-06})
    t = pa.table({"intercept": pa.array([2.0], pa.float64()),
                  "coefficients": pa.array([{"type": 1, "size": None, "indices": None, "values": [3.0, -1.0, 0.5]}],
                                           VEC_ARROW),
                  "scale": pa.array([1.0], pa.float64())})
    write_parquet(path, "data", t, [field("intercept", "double", False), field("coefficients", VEC_UDT),
                                    field("scale", "double", False)])


def standard_scaler(path):
    write_meta(path, "org.apache.spark.ml.feature.StandardScalerModel", "StandardScaler_2a3b4c5d6e7f",
               {"inputCol": "features", "outputCol": "scaled", "withMean": True},
               {"withMean": False, "withStd": True, "outputCol": "StandardScaler_2a3b4c5d6e7f__output"})
    t = pa.table({"std": pa.array([{"type": 1, "size": None, "indices": None, "values": [2.0, 0.5]}], VEC_ARROW),
                  "mean": pa.array([{"type": 1, "size": None, "indices": None, "values": [1.0, -1.0]}], VEC_ARROW)})
    write_parquet(path, "data", t, [field("std", VEC_UDT), field("mean", VEC_UDT)])


def string_indexer(path):
    write_meta(path, "org.apache.spark.ml.feature.StringIndexerModel", "StringIndexer_6f5e4d3c2b1a",
               {"inputCol": "color", "outputCol": "color_idx"},
               {"handleInvalid": "error", "outputCol": "StringIndexer_6f5e4d3c2b1a__output",
                "stringOrderType": "frequencyDesc"})
    t = pa.table({"labelsArray": pa.array([[["red", "green", "blue"]]],
                                          pa.list_(pa.field("element", pa.list_(pa.field("element", pa.string(), True)), True)))})
    arr = {"type": "array", "elementType": {"type": "array", "elementType": "string", "containsNull": True},
           "containsNull": True}
    write_parquet(path, "data", t, [field("labelsArray", arr)])


def _cls_stump(feature, thr, n_left, n_right):
    """Gini classification stump (2 classes) as Spark NodeData rows: impurityStats are the
    per-class (weighted) counts, prediction the majority class."""
    def gini(c):
        n = sum(c)
        return 1.0 - sum((x / n) ** 2 for x in c) if n else 0.0
    tot = [n_left[0] + n_right[0], n_left[1] + n_right[1]]
    leaf_split = {"featureIndex": -1, "leftCategoriesOrThreshold": [], "numCategories": -1}

    def node(i, c, lc, rc, split, gain):
        return {"id": i, "prediction": float(c.index(max(c))), "impurity": gini(c),
                "impurityStats": [float(x) for x in c], "rawCount": int(sum(c)), "gain": gain,
                "leftChild": lc, "rightChild": rc, "split": split}
    g = gini(tot) - (sum(n_left) * gini(n_left) + sum(n_right) * gini(n_right)) / sum(tot)
    return [node(0, tot, 1, 2, {"featureIndex": feature, "leftCategoriesOrThreshold": [thr], "numCategories": -1}, g),
            node(1, n_left, -1, -1, leaf_split, -1.0), node(2, n_right, -1, -1, leaf_split, -1.0)]


RF_DEFAULTS = {"bootstrap": True, "cacheNodeIds": False, "checkpointInterval": 10, "featureSubsetStrategy": "auto",
               "featuresCol": "features", "impurity": "gini", "labelCol": "label", "leafCol": "", "maxBins": 32,
               "maxDepth": 5, "maxMemoryInMB": 256, "minInfoGain": 0.0, "minInstancesPerNode": 1,
               "minWeightFractionPerNode": 0.0, "numTrees": 20, "predictionCol": "prediction",
               "probabilityCol": "probability", "rawPredictionCol": "rawPrediction", "seed": 207336481,
               "subsamplingRate": 1.0}


def random_forest(path):
    uid = "RandomForestClassifier_0e1d2c3b4a59"
    write_meta(path, "org.apache.spark.ml.classification.RandomForestClassificationModel", uid,
               {"numTrees": 2, "maxDepth": 1}, RF_DEFAULTS, numFeatures=2, numClasses=2, numTrees=2)
    rows = [{"treeID": 0, "nodeData": r} for r in _cls_stump(0, 0.5, [30, 10], [5, 55])] + \
        [{"treeID": 1, "nodeData": r} for r in _cls_stump(1, 2.0, [8, 32], [40, 20])]
    t = pa.Table.from_pylist(rows, schema=pa.schema([pa.field("treeID", pa.int32(), False), ("nodeData", NODE)]))
    write_parquet(path, "data", t, [field("treeID", "integer", False), field("nodeData", NODE_SQL)])
    tree_meta = [json.dumps({"class": "org.apache.spark.ml.classification.DecisionTreeClassificationModel",
                             "timestamp": TS, "sparkVersion": VERSION, "uid": f"dtc_{i}",
                             "paramMap": {"maxDepth": 1, "impurity": "gini"}, "defaultParamMap": {}},
                            separators=(",", ":")) for i in range(2)]
    tm = pa.table({"treeID": pa.array([0, 1], pa.int32()), "metadata": pa.array(tree_meta, pa.string()),
                   "weights": pa.array([1.0, 1.0], pa.float64())})
    write_parquet(path, "treesMetadata", tm, [field("treeID", "integer", False), field("metadata", "string"),
                                              field("weights", "double", False)])


def decision_tree(path):
    defaults = {k: v for k, v in RF_DEFAULTS.items() if k not in ("bootstrap", "featureSubsetStrategy", "numTrees",
                                                                  "subsamplingRate")}
    write_meta(path, "org.apache.spark.ml.classification.DecisionTreeClassificationModel",
               "DecisionTreeClassifier_5a4b3c2d1e0f", {"maxDepth": 1}, defaults, numFeatures=2, numClasses=2)
    t = pa.Table.from_pylist(_cls_stump(1, -0.5, [12, 3], [4, 21]), schema=pa.schema(list(NODE)))
    write_parquet(path, "data", t, NODE_SQL["fields"])


def naive_bayes(path):
    import math as _m
    write_meta(path, "org.apache.spark.ml.classification.NaiveBayesModel", "NaiveBayes_4b5c6d7e8f90",
               {"smoothing": 1.0},
               {"featuresCol": "features", "labelCol": "label", "modelType": "multinomial",
                "predictionCol": "prediction", "probabilityCol": "probability", "rawPredictionCol": "rawPrediction",
                "smoothing": 1.0})
    pi = [_m.log(0.4), _m.log(0.6)]
    theta = [[_m.log(0.5), _m.log(0.3), _m.log(0.2)], [_m.log(0.1), _m.log(0.2), _m.log(0.7)]]
    # MatrixUDT is column-major unless isTransposed: store theta (2 x 3) column by column
    colmaj = [theta[r][c] for c in range(3) for r in range(2)]
    t = pa.table({"pi": pa.array([{"type": 1, "size": None, "indices": None, "values": pi}], VEC_ARROW),
                  "theta": pa.array([{"type": 1, "numRows": 2, "numCols": 3, "colPtrs": None, "rowIndices": None,
                                      "values": colmaj, "isTransposed": False}], MAT_ARROW),
                  "sigma": pa.array([{"type": 1, "numRows": 0, "numCols": 0, "colPtrs": None, "rowIndices": None,
                                      "values": [], "isTransposed": False}], MAT_ARROW)})
    write_parquet(path, "data", t, [field("pi", VEC_UDT), field("theta", MAT_UDT), field("sigma", MAT_UDT)])


def min_max_scaler(path):
    write_meta(path, "org.apache.spark.ml.feature.MinMaxScalerModel", "MinMaxScaler_1f2e3d4c5b6a",
               {"inputCol": "features", "outputCol": "scaled"},
               {"max": 1.0, "min": 0.0, "outputCol": "MinMaxScaler_1f2e3d4c5b6a__output"})
    t = pa.table({"originalMin": pa.array([{"type": 1, "size": None, "indices": None, "values": [0.0, -2.0]}],
                                          VEC_ARROW),
                  "originalMax": pa.array([{"type": 1, "size": None, "indices": None, "values": [4.0, 2.0]}],
                                          VEC_ARROW)})
    write_parquet(path, "data", t, [field("originalMin", VEC_UDT), field("originalMax", VEC_UDT)])


def idf(path):
    write_meta(path, "org.apache.spark.ml.feature.IDFModel", "IDF_9a8b7c6d5e4f",
               {"inputCol": "tf", "outputCol": "tfidf"}, {"minDocFreq": 0, "outputCol": "IDF_9a8b7c6d5e4f__output"})
    t = pa.table({"idf": pa.array([{"type": 1, "size": None, "indices": None, "values": [0.5, 1.25, 0.0]}],
                                  VEC_ARROW),
                  "docFreq": pa.array([[3, 1, 4]], pa.list_(pa.field("element", pa.int64(), False))),
                  "numDocs": pa.array([4], pa.int64())})
    arr = {"type": "array", "elementType": "long", "containsNull": False}
    write_parquet(path, "data", t, [field("idf", VEC_UDT), field("docFreq", arr), field("numDocs", "long", False)])


def one_hot_encoder(path):
    write_meta(path, "org.apache.spark.ml.feature.OneHotEncoderModel", "OneHotEncoder_3e4d5c6b7a81",
               {"inputCols": ["c"], "outputCols": ["c_vec"]}, {"dropLast": True, "handleInvalid": "error"})
    t = pa.table({"categorySizes": pa.array([[3]], pa.list_(pa.field("element", pa.int32(), False)))})
    write_parquet(path, "data", t, [field("categorySizes", {"type": "array", "elementType": "integer",
                                                            "containsNull": False})])


def count_vectorizer(path):
    write_meta(path, "org.apache.spark.ml.feature.CountVectorizerModel", "CountVectorizer_8e7f6a5b4c3d",
               {"inputCol": "words", "outputCol": "counts"},
               {"binary": False, "maxDF": 9.223372036854776e18, "minDF": 1.0, "minTF": 1.0,
                "outputCol": "CountVectorizer_8e7f6a5b4c3d__output", "vocabSize": 262144})
    t = pa.table({"vocabulary": pa.array([["a", "b", "c"]], pa.list_(pa.field("element", pa.string(), True)))})
    write_parquet(path, "data", t, [field("vocabulary", {"type": "array", "elementType": "string",
                                                         "containsNull": True})])


def main():
    if os.path.exists(ROOT):
        shutil.rmtree(ROOT)
    for name, fn in (("logistic_regression", logistic), ("kmeans", kmeans), ("gbt_classifier", gbt), ("als", als),
                     ("pipeline", pipeline), ("linear_svc", linear_svc), ("linear_regression", linear_regression),
                     ("standard_scaler", standard_scaler), ("string_indexer", string_indexer),
                     ("random_forest_classifier", random_forest), ("decision_tree_classifier", decision_tree),
                     ("naive_bayes", naive_bayes), ("min_max_scaler", min_max_scaler), ("idf", idf),
                     ("one_hot_encoder", one_hot_encoder), ("count_vectorizer", count_vectorizer)):
        fn(os.path.join(ROOT, name))
    print(ROOT)


if __name__ == "__main__":
    main()
