"""Quantile-binning kernel timing: rows x 64 bf16 features -> uint8 bins, with and without
the feature-major copy written in the same pass (models/trees.py::bin_features).

    python tools/bench_binning.py [--rows 500000000] [--features 64] [--bins 32]
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
    ap.add_argument("--rows", type=int, default=500_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--bins", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    from orange3_spark_amd.models import trees as TR
    n, F = a.rows, a.features
    dev = torch.device("cuda")
    X = torch.empty((n, F), dtype=torch.bfloat16, device=dev)
    step = 1 << 26
    g = torch.Generator(device=dev).manual_seed(1)
    for s in range(0, n, step):
        X[s:s + step].normal_(generator=g)
    qs = np.linspace(0, 1, a.bins + 1)[1:-1]
    splits = [np.quantile(np.random.default_rng(f).standard_normal(100_000), qs) for f in range(F)]
    tht, Tp = TR._thresholds(splits, F, dev)
    out = torch.empty((n, F), dtype=torch.uint8, device=dev)
    out_t = torch.empty((F, n), dtype=torch.uint8, device=dev)
    res = {}
    sig = {}
    # O3S_BIN_EYT: per-level interleaved search-tree threshold table (1, default) vs [F][Tp + 1] (0)
    for lay in ("1", "0"):
        os.environ["O3S_BIN_EYT"] = lay
        for name, ot in (("with_feature_major", out_t), ("row_major_only", None)):
            TR._bin_block_kernel(X, tht, Tp, out, ot, n)
            torch.cuda.synchronize()
            if ot is not None:
                sig[lay] = (int(out[:: 997].sum()), int(out_t[:, :: 997].sum()))
            ts = []
            for _ in range(a.reps):
                t = time.perf_counter()
                TR._bin_block_kernel(X, tht, Tp, out, ot, n)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            ms = 1e3 * min(ts)
            gb = n * F * (2 + 1 + (1 if ot is not None else 0)) / 1e9
            res[("tree_layout_" if lay == "1" else "row_layout_") + name] = {
                "ms": round(ms, 3), "GB_moved": round(gb, 1), "TBps": round(gb / ms, 2)}
    os.environ.pop("O3S_BIN_EYT")
    res["same_bins"] = sig.get("1") == sig.get("0")
    print(json.dumps({"rows": n, "features": F, "bins": a.bins, **res}), flush=True)


if __name__ == "__main__":
    main()
