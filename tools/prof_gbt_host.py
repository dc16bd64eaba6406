#!/usr/bin/env python
"""Host-side profile (cProfile) of the GBT BASELINE config fit (500M x 64, depth 8):
where the wall time outside the traced device phases goes."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from orange3_spark_amd import Session
    from orange3_spark_amd.ml.classification import GBTClassifier
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000_000
    s = Session.getOrCreate()
    df = s.synthetic.trees(rows, 64, seed=5)
    torch.cuda.synchronize()
    est = GBTClassifier(maxDepth=8, maxIter=3, stepSize=0.1, seed=0)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    est.fit(df)
    torch.cuda.synchronize()
    pr.disable()
    dt = time.perf_counter() - t0
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("cumulative").print_stats(35)
    print(f"fit_s {dt:.3f}")
    print(out.getvalue())


if __name__ == "__main__":
    main()
