"""BASELINE config 4: ALS implicit rank=128, 50M users x 5M items on 8 GPUs.

Default sizes are the per-GPU share of that job (1/8 of the users, items and of 1B
ratings) so one GPU reproduces one rank's compute; under torchrun pass the full sizes.
Prints seconds per ALS iteration (both half-iterations, CG solver).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session  # noqa: E402
from orange3_spark_amd.models import als as AE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=6_250_000)
    ap.add_argument("--items", type=int, default=625_000)
    ap.add_argument("--ratings", type=int, default=125_000_000)
    ap.add_argument("--rank", type=int, default=128)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--cg", type=int, default=3)
    ap.add_argument("--dense-min-avg", type=int, default=None,
                    help="rows averaging >= this many ratings take the exact MFMA Gram + Cholesky solve (0 = CG only)")
    a = ap.parse_args()
    from orange3_spark_amd.runtime.tracing import TRACER
    s = Session.getOrCreate()
    df = s.synthetic.ratings(a.users, a.items, a.ratings, rank=8, seed=1, implicit=True)
    u = df.column_data("user").data.long()
    i = df.column_data("item").data.long()
    r = df.column_data("rating").data
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if a.dense_min_avg is not None:
        AE.DENSE_MIN_AVG = a.dense_min_avg
    res = AE.fit_als(s.comm, u, i, r, a.rank, a.iters, 0.1, True, 1.0, 0, cg_iters=a.cg, exact=False,
                     keep_full=False)
    torch.cuda.synchronize()
    print(json.dumps({"metric": "ALS implicit seconds per iteration (rank 128)", "value": min(res.iter_seconds),
                      "unit": "s/iter", "iter_seconds": res.iter_seconds, "total_s": time.perf_counter() - t0,
                      "users": a.users, "items": a.items, "ratings": a.ratings, "n_gpus": s.comm.world_size,
                      "cg_iters": a.cg,
                      "phases_s": ({k: round(v["total_s"], 4) for k, v in TRACER.summary().items()}
                                   if TRACER.enabled else None)}))


if __name__ == "__main__":
    main()
