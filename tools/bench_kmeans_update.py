"""Times the KMeans slab-update kernel alone (per-cluster sums + counts) over a k sweep.

Prints one JSON line: ms per update call by k, and the effective X read bandwidth.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd.ops import kmeans as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--ks", default="2,8,64,1024,4096")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--grid", type=int, default=0, help="update blocks (default 2 per CU)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    X = torch.randn(args.rows, args.d, device=dev)
    out = {"rows": args.rows, "d": args.d, "ms_by_k": {}, "tbps_by_k": {}}
    for k in [int(v) for v in args.ks.split(",")]:
        a = torch.randint(0, k, (args.rows,), device=dev, dtype=torch.int32)
        ws = K.UpdateWorkspace(dev, k, args.d, grid=args.grid or None)
        K.update(X, a, k, ws)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.iters):
            K.update(X, a, k, ws)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / args.iters
        out["ms_by_k"][k] = ms
        out["tbps_by_k"][k] = X.numel() * 4 / ms / 1e9
        print(f"k={k} {ms:.2f} ms", flush=True)
        del a, ws
    print(json.dumps(out))


if __name__ == "__main__":
    main()
