#!/usr/bin/env python
"""ALS fit through the executor pool vs in process (executor-resident model check).

Fits ``ALS(rank=128, implicitPrefs=True)`` on synthetic ratings (default 5M users x 500K
items, 100M ratings) twice on the same GPU: (1) from a driver whose executor pool holds
the data (``o3s.executor.pool=true``, 1 executor on cuda:0 -- the canvas path; the model
stays on the executor as a RemoteModel), (2) directly in this process.  Reports both fit
times and the bytes that crossed the driver pipes during fit + transform + save.
Reference call site: the Recommendation widget's ``fit`` (orangecontrib/spark/base/
spark_ml_estimator.py:22) and the Model Transformer's ``transform`` (widgets/ml/
spark_ml_model.py:53).  The driver never touches the GPU before the pool runs.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=5_000_000)
    ap.add_argument("--items", type=int, default=500_000)
    ap.add_argument("--ratings", type=int, default=100_000_000)
    ap.add_argument("--rank", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.recommendation import ALS
    from orange3_spark_amd.runtime.executors import RemoteModel
    est = ALS(rank=a.rank, implicitPrefs=True, maxIter=a.iters, regParam=0.1, seed=0)
    tmp = tempfile.mkdtemp()
    # (1) executor pool of one (the driver process never initialises HIP)
    s = Session(SessionConf().set("o3s.executor.pool", "true").set("spark.executor.instances", "1"))
    Session._active = s
    try:
        df = s.synthetic.ratings(a.users, a.items, a.ratings, rank=8, seed=1, implicit=True)
        df.count()
        pool = s.pool
        t = time.perf_counter()
        est.copy({est.maxIter: 1}).fit(df)          # first fit of the process: module / handle warm-up
        t_pool_first = time.perf_counter() - t
        b0 = pool.bytes_sent + pool.bytes_received
        t = time.perf_counter()
        model = est.fit(df)
        t_pool = time.perf_counter() - t
        resident = type(model) is RemoteModel
        n_pred = model.transform(df).count()
        model.write().overwrite().save(os.path.join(tmp, "als"))
        moved = pool.bytes_sent + pool.bytes_received - b0
        its_pool = list(model.iterationSeconds)
        print(f"[pool] fit {t_pool:.2f}s, moved {moved} B", file=sys.stderr, flush=True)
    finally:
        s.stop()
        Session._active = None
    # (2) in process
    import torch
    s2 = Session(SessionConf().set("spark.master", "local[1]").set("spark.executor.instances", "1"))
    df2 = s2.synthetic.ratings(a.users, a.items, a.ratings, rank=8, seed=1, implicit=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    est.copy({est.maxIter: 1}).fit(df2)
    torch.cuda.synchronize()
    t_direct_first = time.perf_counter() - t
    t = time.perf_counter()
    m2 = est.fit(df2)
    torch.cuda.synchronize()
    t_direct = time.perf_counter() - t
    shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps({"metric": "ALS fit through the executor pool vs in process", "unit": "s",
                      "value": t_pool, "model_resident_on_executor": resident, "direct_fit_s": t_direct,
                      "warmup_fit_1iter_s": {"pool": t_pool_first, "direct": t_direct_first}, "pool_over_direct": t_pool / t_direct,
                      "driver_pipe_bytes_fit_transform_save": moved, "predictions": n_pred,
                      "iter_seconds_pool": its_pool, "iter_seconds_direct": list(m2.iterationSeconds),
                      "config": {"users": a.users, "items": a.items, "ratings": a.ratings, "rank": a.rank,
                                 "maxIter": a.iters, "implicitPrefs": True},
                      "model_factor_bytes": (m2._U.numel() + m2._V.numel()) * 4}), flush=True)


if __name__ == "__main__":
    main()
