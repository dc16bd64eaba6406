"""Run only the KMeans assign kernel a few times (for rocprofv3 --pmc runs)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session  # noqa: E402
from orange3_spark_amd.ops import kmeans as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=20_000_000)
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--mode", default="auto", choices=["auto", "screen", "split"])
ap.add_argument("--tt", type=int, default=0, help="screen kernel tiles per wave (0 = default)")
ap.add_argument("--nodist", action="store_true", help="no per-row distances (the Lloyd iterations' build)")
a = ap.parse_args()
s = Session.getOrCreate()
df = s.synthetic.blobs(a.rows, a.d, k=a.k, seed=3, spread=1.0)
X = df.column_data("features").data
C = df.true_centers.float() + 0.5
prep = K.prepare_centers(C)
if a.tt:
    K.SCREEN_TT = a.tt
import time  # noqa: E402
K.assign(X, C, prep, mode=a.mode, need_dist=not a.nodist)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.iters):
    K.assign(X, C, prep, mode=a.mode, need_dist=not a.nodist)
torch.cuda.synchronize()
print(f"done {a.mode} tt={a.tt} rows={a.rows} ms/assign={(time.perf_counter() - t) / a.iters * 1e3:.2f}")
