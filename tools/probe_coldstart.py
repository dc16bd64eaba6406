"""What a process's first fit pays that later fits do not (the warm-up question).

One fresh process per call: a session with the family warm-up off (or the mode given),
synthetic data, then the same fit twice; prints one JSON line with session start, data
and both fit times.  Modes:
  none      -- no warm-up at all
  preload   -- only ``ops._native.preload()`` (load every kernel code object, no fits)
  family    -- the lazy per-family warm-up (``o3s.session.warmup=lazy``)
  fits      -- the tiny warm-up fits of the fitted family at session start (round 5)
  auto      -- the default: preload, then every family warmed on a background thread
               while the data is generated (no explicit wait)
Run ``HIP_ENABLE_DEFERRED_LOADING=0`` around ``none`` to see how much of the cold cost is
code-object loading at all (every fatbin of every library loaded at HIP init).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="none", choices=("none", "preload", "family", "fits", "auto"))
    ap.add_argument("--family", default="trees", choices=("trees", "glm", "kmeans", "als"))
    ap.add_argument("--rows", type=int, default=100_000_000)
    a = ap.parse_args()
    import torch
    t0 = time.perf_counter()
    from orange3_spark_amd import Session, SessionConf
    warm = {"none": "false", "preload": "preload", "family": "lazy", "fits": a.family, "auto": "auto"}[a.mode]
    s = Session.getOrCreate(SessionConf().set("spark.master", "local[1]").set("o3s.session.warmup", warm))
    torch.cuda.synchronize()
    t_session = time.perf_counter() - t0
    t = time.perf_counter()
    if a.family == "trees":
        from orange3_spark_amd.ml.classification import GBTClassifier
        df = s.synthetic.trees(a.rows, 64, seed=3)
        fit = lambda: GBTClassifier(maxDepth=8, maxIter=3, seed=0).fit(df)  # noqa: E731
    elif a.family == "glm":
        from orange3_spark_amd.ml.classification import LogisticRegression
        df = s.synthetic.classification(a.rows, 256, seed=3)
        fit = lambda: LogisticRegression(maxIter=10, tol=0.0).fit(df)  # noqa: E731
    elif a.family == "kmeans":
        from orange3_spark_amd.ml.clustering import KMeans
        df = s.synthetic.blobs(a.rows, 128, 1024, seed=3)
        fit = lambda: KMeans(k=1024, maxIter=5, tol=0.0, seed=0).fit(df)  # noqa: E731
    else:
        from orange3_spark_amd.ml.recommendation import ALS
        df = s.synthetic.ratings(a.rows // 20, a.rows // 200, a.rows, rank=8, seed=3, implicit=True)
        fit = lambda: ALS(rank=128, maxIter=2, implicitPrefs=True, seed=0).fit(df)  # noqa: E731
    torch.cuda.synchronize()
    t_data = time.perf_counter() - t
    fits = []
    for _ in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fit()
        torch.cuda.synchronize()
        fits.append(round(time.perf_counter() - t, 4))
    print(json.dumps({"mode": a.mode, "family": a.family, "rows": a.rows,
                      "deferred_loading": os.environ.get("HIP_ENABLE_DEFERRED_LOADING", "default"),
                      "session_start_s": round(t_session, 4), "warmup_seconds": s.warmup_seconds,
                      "data_s": round(t_data, 4), "fit_s": fits, "cold_over_warm": round(fits[0] / fits[1], 4)}),
          flush=True)


if __name__ == "__main__":
    main()
