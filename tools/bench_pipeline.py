#!/usr/bin/env python
"""End-to-end tutorial pipeline through the real widget path, at scale (1 GPU):

  wide columnar table (f0..f255 fp32 + label, 100M rows)
    -> Dataset Builder widget (VectorAssembler: one fused gather kernel -> padded bf16)
    -> Classification widget: LogisticRegression.fit (L-BFGS, fused gradient kernel)
    -> Model Transformer widget: model.transform (margin kernel)
    -> Evaluation widget: BinaryClassificationEvaluator areaUnderROC (score histogram kernel)

Reference chain: orangecontrib/spark/tutorials/spark_ml.ows (Hive Table -> Dataset Builder
-> Classification -> Model Transformer -> Evaluation); VectorAssembler at
widgets/ml/spark_ml_dataset.py:575-576.  Prints one JSON line with per-stage seconds and
the assembler's effective bandwidth (bytes read + written / time).
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
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--features", type=int, default=256)
    ap.add_argument("--max-iter", type=int, default=10)
    a = ap.parse_args()
    from orange3_spark_amd import Session, SessionConf
    from orangecontrib.spark_amd.widgets.ml.owclassification import OWClassification
    from orangecontrib.spark_amd.widgets.ml.owdatasetbuilder import OWDatasetBuilder
    from orangecontrib.spark_amd.widgets.ml.owevaluation import OWEvaluation
    from orangecontrib.spark_amd.widgets.ml.owmodeltransformer import OWModelTransformer
    s = Session.getOrCreate(SessionConf().setAppName("bench-pipeline"))
    gpu = s.device.type == "cuda"
    rows = a.rows if gpu else min(a.rows, 50_000)

    def sync():
        if gpu:
            torch.cuda.synchronize()
    t = time.perf_counter()
    table = s.synthetic.table(rows, a.features, seed=11)
    sync()
    res = {"rows": rows, "features": a.features, "table_gen_s": time.perf_counter() - t}
    feats = [f"f{j}" for j in range(a.features)]

    b = OWDatasetBuilder()
    b.set_data(table)
    b.set_features(feats)
    b.set_label("label")
    b.commit()                                     # warm-up (kernel load)
    sync()
    t = time.perf_counter()
    df = b.commit()
    sync()
    res["assemble_s"] = time.perf_counter() - t
    elem = table.column_data("f0").data.element_size()
    ld = df.column_data("features").data.shape[1]
    moved = rows * (a.features * elem + ld * 2 + 4 + 8)
    res["assemble_TBps"] = moved / res["assemble_s"] / 1e12
    res["features_dtype"] = str(df.column_data("features").data.dtype)

    clf = OWClassification()
    clf.get_input(df)
    clf.select_method("LogisticRegression").set_param("maxIter", str(a.max_iter))
    t = time.perf_counter()
    model = clf.apply()
    sync()
    res["fit_s"] = time.perf_counter() - t
    assert model is not None, clf.messages
    res["fit_iterations"] = model.summary.totalIterations

    mt = OWModelTransformer()
    t = time.perf_counter()
    mt.get_input_model(model)
    mt.get_input(df)
    sync()
    res["transform_s"] = time.perf_counter() - t

    ev = OWEvaluation()
    ev.get_input(mt.out_df)
    ev.select_method("BinaryClassificationEvaluator")
    t = time.perf_counter()
    vals = ev.apply()
    sync()
    res["evaluate_s"] = time.perf_counter() - t
    res["areaUnderROC"] = vals["areaUnderROC"]
    res["device"] = str(s.device)
    res["end_to_end_s"] = res["assemble_s"] + res["fit_s"] + res["transform_s"] + res["evaluate_s"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
