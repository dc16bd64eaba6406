"""Where does a process's first fit spend the time a second fit does not?

cProfile of the first and the second fit of one family in a fresh process (warm-up off),
printing the functions whose own time differs most between them -- host-side first-call
costs (imports, kernel code-object loads inside torch / HIP calls, library handles).
"""
from __future__ import annotations

import argparse
import cProfile
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="trees")
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--mode", default="false")
    a = ap.parse_args()
    import torch
    from orange3_spark_amd import Session, SessionConf
    s = Session.getOrCreate(SessionConf().set("spark.master", "local[1]").set("o3s.session.warmup", a.mode))
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
    stats, wall = [], []
    for _ in range(2):
        pr = cProfile.Profile()
        t = time.perf_counter()
        pr.enable()
        fit()
        torch.cuda.synchronize()
        pr.disable()
        wall.append(time.perf_counter() - t)
        stats.append(pstats.Stats(pr).stats)
    first, second = stats

    def own(st):
        out = {}
        for (fn, ln, name), (cc, nc, tt, ct, callers) in st.items():
            k = f"{os.path.basename(fn)}:{ln}:{name}"
            out[k] = out.get(k, 0.0) + tt
        return out
    f1, f2 = own(first), own(second)
    diff = sorted(((f1.get(k, 0) - f2.get(k, 0), f1.get(k, 0), f2.get(k, 0), k) for k in set(f1) | set(f2)),
                  reverse=True)[: a.top]
    print(json.dumps({"family": a.family, "rows": a.rows, "fit_s": [round(w, 4) for w in wall],
                      "top_own_time_delta": [{"fn": k, "first_s": round(x1, 5), "second_s": round(x2, 5),
                                              "delta_s": round(d, 5)} for d, x1, x2, k in diff]}, indent=1))


if __name__ == "__main__":
    main()
