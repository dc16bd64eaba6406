"""End-to-end KMeans.fit (k-means|| init + Lloyd) on the BASELINE shape, with phase times."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session  # noqa: E402
from orange3_spark_amd.ml.clustering import KMeans  # noqa: E402
from orange3_spark_amd.runtime.tracing import TRACER  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
s = Session.getOrCreate()
df = s.synthetic.blobs(a.rows, a.d, k=a.k, seed=3, spread=1.0)
TRACER.enable(True, sync=True)
torch.cuda.synchronize()
t = time.perf_counter()
m = KMeans(k=a.k, maxIter=a.iters, seed=1, tol=0.0).fit(df)
torch.cuda.synchronize()
dt = time.perf_counter() - t
print(json.dumps({"metric": "KMeans.fit seconds (k-means|| init + Lloyd)", "value": dt, "rows": a.rows, "d": a.d,
                  "k": a.k, "iters": m.summary.numIter, "cost": m.summary.trainingCost,
                  "phases_s": {k: round(v["total_s"], 4) for k, v in TRACER.summary().items()}}))
