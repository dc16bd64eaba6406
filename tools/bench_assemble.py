#!/usr/bin/env python
"""VectorAssembler kernel micro-bench (1 GPU): --rows x --features plain columns of
--dtype -> padded bf16 feature matrix, timing the generic gather kernel and the
column-window kernel (64 / 128-column LDS windows).  Effective bandwidth = bytes read
(columns) + bytes written (matrix + invalid flags) over kernel time."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--features", type=int, default=256)
    ap.add_argument("--dtype", default="float32", choices=["float32", "float64"])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from orange3_spark_amd.ops import assemble as AS
    dev = torch.device("cuda", 0)
    dt = getattr(torch, a.dtype)
    n = a.rows
    cols = [torch.empty(n, dtype=dt, device=dev).uniform_(-1, 1) for _ in range(a.features)]
    srcs = [(c, None, 1) for c in cols]
    res = {"rows": n, "features": a.features, "dtype": a.dtype}
    for name, kw in (("generic", dict(path="generic")), ("cols", dict(path="cols"))):
        out = AS.assemble_bf16(srcs, n, dev, **kw)
        del out
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = AS.assemble_bf16(srcs, n, dev, **kw)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 1e3)
            ld = out[0].shape[1]
            del out
        moved = n * (a.features * cols[0].element_size() + ld * 2 + 1)
        res[name] = {"s": best, "TBps": moved / best / 1e12}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
