"""RandomForestClassifier fit time: all trees grown together (one launch per level for
the whole forest) vs one tree at a time.  Synthetic tree-structured data on one GPU."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session, SessionConf  # noqa: E402
from orange3_spark_amd.ml.classification import RandomForestClassifier  # noqa: E402
from orange3_spark_amd.models.trees import TreeBuilder  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=2_000_000)
ap.add_argument("--features", type=int, default=32)
ap.add_argument("--trees", type=int, default=20)
ap.add_argument("--depth", type=int, default=8)
a = ap.parse_args()
s = Session(SessionConf().set("o3s.device", "cuda"))
df = s.synthetic.trees(a.rows, a.features, seed=1).cache()
res = {}
for name, flag in (("batched", True), ("sequential", False)):
    TreeBuilder.batch_trees = flag
    est = RandomForestClassifier(numTrees=a.trees, maxDepth=a.depth, seed=5)
    est.fit(df)                                   # warm-up (binning cache, kernels)
    torch.cuda.synchronize()
    t = time.perf_counter()
    m = est.fit(df)
    torch.cuda.synchronize()
    res[name] = round(time.perf_counter() - t, 4)
    res[name + "_nodes"] = sum(t_.numNodes for t_ in m.trees)
TreeBuilder.batch_trees = True
print(json.dumps({"metric": "RandomForestClassifier fit seconds", "rows": a.rows, "features": a.features,
                  "trees": a.trees, "depth": a.depth, **res}))
