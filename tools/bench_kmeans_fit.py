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
ap.add_argument("--repeat", type=int, default=1, help="fits in this process (the first is cold)")
ap.add_argument("--data", default="blobs", choices=["blobs", "uniform"])
ap.add_argument("--no-hamerly", action="store_true", help="screen every row every Lloyd iteration (A/B)")
ap.add_argument("--pair-from", type=float, default=None,
                help="ops.kmeans.PAIR_FROM: flagged fraction above which the pair screen is tried")
a = ap.parse_args()
from orange3_spark_amd.models import kmeans as _KM  # noqa: E402
_KM.HAMERLY = not a.no_hamerly
if a.pair_from is not None:
    from orange3_spark_amd.ops import kmeans as _K
    _K.PAIR_FROM = a.pair_from
SYNC = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
s = Session.getOrCreate()
if a.data == "blobs":
    df = s.synthetic.blobs(a.rows, a.d, k=a.k, seed=3, spread=1.0)
else:
    from collections import OrderedDict
    from orange3_spark_amd.frame import column as C
    from orange3_spark_amd.frame.dataframe import DataFrame
    X = torch.empty((a.rows, a.d), dtype=torch.float32, device=s.device)
    g = torch.Generator(device=s.device).manual_seed(3)
    for r0 in range(0, a.rows, 1 << 24):
        X[r0:r0 + (1 << 24)].uniform_(-1.0, 1.0, generator=g)
    df = DataFrame(s, OrderedDict(features=C.VectorColumn(X)), a.rows)
for rep in range(a.repeat):
    TRACER.reset()
    TRACER.enable(True, sync=True)
    SYNC()
    t = time.perf_counter()
    m = KMeans(k=a.k, maxIter=a.iters, seed=1, tol=0.0).fit(df)
    SYNC()
    dt = time.perf_counter() - t
    ph = {k: round(v["total_s"], 4) for k, v in TRACER.summary().items()}
    init = sum(v for k, v in ph.items() if k in ("kmeans.init.round", "kmeans.init.weights", "kmeans.init.local"))
    print(json.dumps({"metric": "KMeans.fit seconds (k-means|| init + Lloyd)", "value": dt, "fit": rep,
                      "cold": rep == 0, "data": a.data, "rows": a.rows, "d": a.d, "k": a.k, "iters": m.summary.numIter,
                      "cost": m.summary.trainingCost, "init_s": round(init, 4), "pair_from": a.pair_from,
                      "hamerly": _KM.HAMERLY, "lloyd_ms_per_iter": round(1e3 * ph.get("kmeans.iter", 0.0) /
                                                                         max(1, m.summary.numIter), 2),
                      "hamerly_stats": list(_KM.LAST_HAMERLY_STATS), "phases_s": ph}), flush=True)
