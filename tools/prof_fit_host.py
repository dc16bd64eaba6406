#!/usr/bin/env python
"""Host-side time of the headline fit: cProfile around ``LogisticRegression(solver='sgd').fit``
on a bf16 table (default 125M x 256 = one rank's share of the N=8 bench), next to the
device time of its passes -- finds host gaps that would cap multi-GPU scaling."""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=125_000_000)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.classification import LogisticRegression
    s = Session(SessionConf().set("spark.master", "local[1]").set("spark.executor.instances", "1"))
    df = s.synthetic.classification(a.rows, 256, seed=2024)
    kw = dict(solver="sgd", stepSize=1.0, miniBatchFraction=1.0, regParam=0.0, standardization=True, tol=0.0)
    LogisticRegression(maxIter=3, **kw).fit(df)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    m = LogisticRegression(maxIter=a.steps, **kw).fit(df)
    torch.cuda.synchronize()
    pr.disable()
    wall = time.perf_counter() - t
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(35)
    print(buf.getvalue()[:12000], file=sys.stderr)
    print(json.dumps({"rows": a.rows, "steps": a.steps, "fit_wall_s": wall, "ms_per_step": wall / a.steps * 1e3,
                      "setup_s": getattr(m, "_fit_setup_seconds", None)}))


if __name__ == "__main__":
    main()
