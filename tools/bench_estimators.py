"""Sweep: fit (and one transform/evaluate) time of every estimator family on one device.

Finds performance pathologies outside the headline configs.  n rows x d features of the
synthetic classification table (bf16 vectors on GPU) / blobs for clustering; prints one
JSON object {name: seconds or "error: ..."}.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from orange3_spark_amd import Session
    from orange3_spark_amd.ml import classification as C, regression as R, clustering as K, feature as F
    from orange3_spark_amd.ml import evaluation as E
    from orange3_spark_amd.sql import functions as SF
    s = Session.getOrCreate()
    sync = torch.cuda.synchronize if s.device.type == "cuda" else (lambda: None)
    n, d = a.rows, a.features
    df = s.synthetic.classification(n, d, seed=1).cache()
    df3 = df.withColumn("label3", (SF.col("label") + SF.rand(seed=2) * 2).cast("int").cast("double")).cache()
    blobs = s.synthetic.blobs(n, d, k=16, seed=3).cache()
    df.count(), df3.count(), blobs.count()
    res = {}

    def t(name, fn):
        if a.only and a.only not in name:
            return
        sync()
        t0 = time.perf_counter()
        try:
            fn()
            sync()
            res[name] = round(time.perf_counter() - t0, 3)
        except Exception as e:  # noqa: BLE001
            res[name] = f"error: {type(e).__name__}: {str(e)[:100]}"
        print(name, res[name], file=sys.stderr, flush=True)

    t("LogisticRegression(lbfgs,20)", lambda: C.LogisticRegression(maxIter=20).fit(df))
    t("LogisticRegression(multinomial,3cls,20)", lambda: C.LogisticRegression(maxIter=20, labelCol="label3").fit(df3))
    t("LinearSVC(20)", lambda: C.LinearSVC(maxIter=20).fit(df))
    t("LinearRegression(20)", lambda: R.LinearRegression(maxIter=20).fit(df))
    t("GeneralizedLinearRegression(poisson)", lambda: R.GeneralizedLinearRegression(family="poisson", maxIter=10).fit(df))
    t("NaiveBayes(gaussian)", lambda: C.NaiveBayes(modelType="gaussian").fit(df3))
    t("DecisionTreeClassifier(d5)", lambda: C.DecisionTreeClassifier(maxDepth=5).fit(df))
    t("RandomForestClassifier(10,d5)", lambda: C.RandomForestClassifier(numTrees=10, maxDepth=5).fit(df))
    t("GBTClassifier(10,d5)", lambda: C.GBTClassifier(maxIter=10, maxDepth=5).fit(df))
    t("GBTRegressor(10,d5)", lambda: R.GBTRegressor(maxIter=10, maxDepth=5).fit(df))
    t("MLP(64-16-2,10it)", lambda: C.MultilayerPerceptronClassifier(layers=[d, 16, 2], maxIter=10).fit(df))
    t("FMClassifier(10it)", lambda: C.FMClassifier(maxIter=10).fit(df))
    t("AFTSurvivalRegression", lambda: R.AFTSurvivalRegression(maxIter=10, censorCol="label").fit(
        df.withColumn("label", SF.col("label") + 1.0)))
    t("KMeans(k16,10it)", lambda: K.KMeans(k=16, maxIter=10).fit(blobs))
    t("BisectingKMeans(k8)", lambda: K.BisectingKMeans(k=8, maxIter=10).fit(blobs))
    t("GaussianMixture(k4,10it)", lambda: K.GaussianMixture(k=4, maxIter=10).fit(blobs))
    t("StandardScaler", lambda: F.StandardScaler(inputCol="features", outputCol="s").fit(df).transform(df).count())
    t("MinMaxScaler", lambda: F.MinMaxScaler(inputCol="features", outputCol="s").fit(df).transform(df).count())
    t("PCA(k8)", lambda: F.PCA(k=8, inputCol="features", outputCol="p").fit(df).transform(df).count())
    t("QuantileDiscretizer", lambda: F.QuantileDiscretizer(inputCol="label3", outputCol="q", numBuckets=4).fit(df3))
    t("StringIndexer", lambda: F.StringIndexer(inputCol="label3", outputCol="i").fit(df3).transform(df3).count())
    t("OneHotEncoder", lambda: F.OneHotEncoder(inputCols=["label3"], outputCols=["o"]).fit(df3).transform(df3).count())
    t("ChiSqSelector", lambda: F.ChiSqSelector(numTopFeatures=8, labelCol="label3").fit(
        F.QuantileDiscretizer(inputCol="label3", outputCol="q", numBuckets=2).fit(df3).transform(df3)))
    t("VarianceThresholdSelector", lambda: F.VarianceThresholdSelector(varianceThreshold=0.1).fit(df))
    lr = C.LogisticRegression(maxIter=5).fit(df).transform(df).cache()
    t("BinaryClassificationEvaluator(auc)", lambda: E.BinaryClassificationEvaluator().evaluate(lr))
    t("MulticlassClassificationEvaluator(f1)", lambda: E.MulticlassClassificationEvaluator().evaluate(lr))
    t("RegressionEvaluator(rmse)", lambda: E.RegressionEvaluator(predictionCol="prediction").evaluate(lr))
    km = K.KMeans(k=16, maxIter=3).fit(blobs).transform(blobs).cache()
    t("ClusteringEvaluator(silhouette)", lambda: E.ClusteringEvaluator().evaluate(km))
    print(json.dumps({"rows": n, "features": d, "device": str(s.device), "seconds": res}))


if __name__ == "__main__":
    main()
