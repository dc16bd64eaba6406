"""Multinomial LogisticRegression: seconds per objective/gradient pass and per fit.

Synthetic n x d features (bf16 vector column, as VectorAssembler / synthetic produce) with
K classes; prints one JSON line."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--features", type=int, default=256)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    s = Session.getOrCreate()
    from orange3_spark_amd.models import glm as GLM
    from orange3_spark_amd.ml import common as U
    df = s.synthetic.classification(a.rows, a.features, seed=3)
    X = U.dense_features(df, "features")
    # K ordered classes from two features (learnable)
    z = (X[:, 0].float() + 0.5 * X[:, 1].float() + 1.5) / 3.0
    y = (z * a.classes).floor().clamp(0, a.classes - 1).to(torch.float64)
    sync = torch.cuda.synchronize if X.is_cuda else (lambda: None)
    sync()
    t = time.perf_counter()
    B, b, r = GLM.fit_multinomial(s.comm, X, y, None, a.classes, max_iter=a.iters, tol=0.0)
    sync()
    dt = time.perf_counter() - t
    print(json.dumps({"metric": "multinomial LR fit", "rows": a.rows, "features": a.features, "classes": a.classes,
                      "x_dtype": str(X.dtype), "fit_s": dt, "iters": r.iterations, "s_per_iter": dt / max(r.iterations, 1),
                      "x_shape": list(X.shape), "x_contiguous": X.is_contiguous()}))


if __name__ == "__main__":
    main()
