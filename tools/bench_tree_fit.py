"""End-to-end GBTClassifier / RandomForestClassifier .fit through the ML API (binning,
trees, model assembly) on one GPU, with traced phases."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session, SessionConf  # noqa: E402
from orange3_spark_amd.ml.classification import GBTClassifier, RandomForestClassifier  # noqa: E402
from orange3_spark_amd.runtime.tracing import TRACER  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=62_500_000)
ap.add_argument("--features", type=int, default=64)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--model", default="gbt", choices=["gbt", "rf"])
a = ap.parse_args()
s = Session(SessionConf().set("o3s.device", "cuda"))
df = s.synthetic.trees(a.rows, a.features, seed=1).cache()
est = GBTClassifier(maxIter=a.iters, maxDepth=8, seed=1) if a.model == "gbt" else \
    RandomForestClassifier(numTrees=a.iters, maxDepth=8, seed=1)
TRACER.enable(True, sync=True)
torch.cuda.synchronize()
t = time.perf_counter()
m = est.fit(df)
torch.cuda.synchronize()
dt = time.perf_counter() - t
print(json.dumps({"metric": f"{type(est).__name__}.fit seconds", "value": dt, "rows": a.rows,
                  "features": a.features, "trees": a.iters,
                  "phases_s": {k: round(v["total_s"], 4) for k, v in TRACER.summary().items()}}))
