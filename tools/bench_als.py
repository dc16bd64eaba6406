"""BASELINE config 4: ALS implicit rank=128, 50M users x 5M items on 8 GPUs.

Default sizes are the per-GPU share of that job (1/8 of the users, items and of 1B
ratings) so one GPU reproduces one rank's compute; under torchrun pass the full sizes.
Prints seconds per ALS iteration (both half-iterations).  Default ``--cg 0``: every
row's normal equations are solved exactly (als_exact kernels, Spark semantics);
``--cg K`` times the opt-in K-step conjugate-gradient approximation instead.
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
    ap.add_argument("--cg", type=int, default=0, help="0 = exact solves (default); K > 0 = K CG steps")
    ap.add_argument("--dense-min-avg", type=int, default=None,
                    help="rows averaging >= this many ratings take the exact MFMA Gram + Cholesky solve (0 = CG only)")
    ap.add_argument("--rank-of", type=int, default=None,
                    help="emulate ONE rank of a W-GPU job: --users/--items/--ratings are the full job's sizes; "
                         "this rank's user block rates items of the whole catalogue and its item block is rated "
                         "by all users, gathered from full-size factor tables (the all-gathered ones)")
    a = ap.parse_args()
    from orange3_spark_amd.runtime.tracing import TRACER
    s = Session.getOrCreate()
    if a.rank_of:
        return rank_share(s, a)
    df = s.synthetic.ratings(a.users, a.items, a.ratings, rank=8, seed=1, implicit=True)
    u = df.column_data("user").data.long()
    i = df.column_data("item").data.long()
    r = df.column_data("rating").data
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if a.dense_min_avg is not None:
        AE.DENSE_MIN_AVG = a.dense_min_avg
    res = AE.fit_als(s.comm, u, i, r, a.rank, a.iters, 0.1, True, 1.0, 0, cg_iters=a.cg, exact=None,
                     keep_full=False)
    torch.cuda.synchronize()
    print(json.dumps({"metric": "ALS implicit seconds per iteration (rank 128)", "value": min(res.iter_seconds),
                      "unit": "s/iter", "iter_seconds": res.iter_seconds, "total_s": time.perf_counter() - t0,
                      "users": a.users, "items": a.items, "ratings": a.ratings, "n_gpus": s.comm.world_size,
                      "cg_iters": a.cg, "solver": "exact" if a.cg <= 0 else f"cg{a.cg}",
                      "phases_s": ({k: round(v["total_s"], 4) for k, v in TRACER.summary().items()}
                                   if TRACER.enabled else None)}))


def rank_share(s, a):
    """Compute of one rank of the W-GPU job, faithfully sized: the rank owns users/W users
    (ratings/W of them, over all items) and items/W items (ratings/W, over all users) and
    its solves gather from the FULL factor tables (users x rank and items x rank, as after
    the per-half-iteration all-gather).  The all-gathers themselves are not run (one GPU);
    their per-rank byte counts are printed next to the time."""
    from orange3_spark_amd.ops.glm import row_keys
    W, dev, R = a.rank_of, s.device, a.rank
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    U, I, n = a.users, a.items, a.ratings // a.rank_of
    u_lo, i_lo = U // W, I // W
    rows = torch.arange(n, dtype=torch.int64, device=dev)

    def block(seed, n_own, n_other):
        own = row_keys(seed, rows) % n_own
        other = row_keys(seed ^ 0x1234567, rows) % n_other
        val = (row_keys(seed ^ 0x55, rows) % 5).to(torch.float32)     # 0 = no interaction (implicit)
        return AE.partition(s.comm, own, other, val, n_own)

    by_user, by_item = block(1, u_lo, I), block(2, i_lo, U)
    del rows
    Xf = AE.init_factors(0, U, R, 0, dev, False)           # the all-gathered tables
    Yf = AE.init_factors(0, I, R, 0x5A5A, dev, False)
    X, Y = Xf[:u_lo].clone(), Yf[:i_lo].clone()
    sync()
    its = []
    for _ in range(a.iters):
        t = time.perf_counter()
        YtY = AE.gram(Y).float()
        X = AE.solve_side(by_user, Yf, X, 0.1, True, 1.0, YtY, a.cg, False, None)
        Xf[:u_lo].copy_(X)
        XtX = AE.gram(X).float()
        Y = AE.solve_side(by_item, Xf, Y, 0.1, True, 1.0, XtX, a.cg, False, None)
        Yf[:i_lo].copy_(Y)
        sync()
        its.append(time.perf_counter() - t)
    print(json.dumps({"metric": f"ALS implicit seconds per iteration (rank {R}), compute of one rank of {W}",
                      "value": min(its), "unit": "s/iter", "iter_seconds": its, "users": U, "items": I,
                      "ratings": a.ratings, "rank_share": {"users": u_lo, "items": i_lo, "ratings_per_side": n},
                      "gathered_tables_bytes": {"users": U * R * 4, "items": I * R * 4},
                      "all_gather_bytes_received_per_rank_per_iter": (U - u_lo + I - i_lo) * R * 4,
                      "cg_iters": a.cg, "solver": "exact" if a.cg <= 0 else f"cg{a.cg}"}))
    return 0


if __name__ == "__main__":
    main()
