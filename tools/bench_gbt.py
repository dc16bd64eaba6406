"""BASELINE config 5: GBTClassifier depth 8 on 500M x 64 (8 GPUs -> 62.5M rows per GPU).

Run on one GPU with --rows 62500000 to measure the per-GPU share; under torchrun each
rank generates its own shard.  Prints seconds per tree (after binning, excluded).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session  # noqa: E402
from orange3_spark_amd.models import trees as TR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=62_500_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--trees", type=int, default=3)
    ap.add_argument("--no-subtraction", action="store_true", help="scan every node at every level")
    a = ap.parse_args()
    TR.TreeBuilder.hist_subtraction = not a.no_subtraction
    s = Session.getOrCreate()
    df = s.synthetic.trees(a.rows, a.features, seed=5)
    X = df.column_data("features").data
    y = df.column_data("label").data
    t0 = time.perf_counter()
    splits = TR.find_splits(s.comm, X, 32, 0)
    bins = TR.bin_features(X, splits)
    torch.cuda.synchronize()
    t_bin = time.perf_counter() - t0
    rows = df._global_rows()
    TR.fit_gbt(s.comm, bins, splits, y, None, "logistic", 1, 0.1, a.depth, rows=rows)   # warmup
    torch.cuda.synchronize()
    from orange3_spark_amd.runtime.tracing import TRACER
    TRACER.reset()
    t1 = time.perf_counter()
    ens = TR.fit_gbt(s.comm, bins, splits, y, None, "logistic", a.trees, 0.1, a.depth, rows=rows)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t1) / a.trees
    from orange3_spark_amd.runtime.tracing import TRACER
    phases = {k: round(v["total_s"] / a.trees, 4) for k, v in TRACER.summary().items()} if TRACER.enabled else None
    print(json.dumps({"metric": "GBTClassifier seconds per tree (depth 8, 64 features)", "value": dt,
                      "unit": "s/tree", "rows_per_gpu": a.rows, "n_gpus": s.comm.world_size,
                      "binning_s": t_bin, "hist_subtraction": TR.TreeBuilder.hist_subtraction, "loss": ens.losses, "nodes": [t.numNodes for t in ens.trees],
                      "phase_s_per_tree": phases}))


if __name__ == "__main__":
    main()
