"""Time the KMeans assign kernel for several k (fixed rows, d) to split fixed per-row
cost (X load + conversion) from per-centroid MFMA cost."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session  # noqa: E402
from orange3_spark_amd.ops import kmeans as K  # noqa: E402

rows, d = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000, 128
s = Session.getOrCreate()
X = s.synthetic.blobs(rows, d, k=64, seed=3).column_data("features").data
out = {}
for k in (32, 128, 512, 1024, 2048):
    C = torch.randn(k, d, device=X.device)
    prep = K.prepare_centers(C)
    K.assign(X, C, prep)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        K.assign(X, C, prep)
    torch.cuda.synchronize()
    out[k] = (time.perf_counter() - t) / 3 * 1e3
print(json.dumps({"rows": rows, "d": d, "assign_ms_by_k": out}))
