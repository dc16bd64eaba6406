#!/usr/bin/env python
"""Exact ALS solve kernels in isolation (rocprofv3 --pmc target; no torch bitwise ops).

Two CSRs shaped like one rank's halves of the rank-128 benchmark, scaled by --scale:
  user side: rows with 1..40 ratings (mean ~20) -> als_wood_kernel (<= 32) / als_dense_wave_kernel
  item side: rows with 100..300 ratings        -> als_dense_wave_kernel
gathering from a --other x R factor table.  Prints per-side seconds and solved rows/s."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def csr(n_rows, lo, hi, n_other, R, dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    lens = torch.randint(lo, hi + 1, (n_rows,), generator=g)
    indptr = torch.zeros(n_rows + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    cols = torch.randint(0, n_other, (nnz,), dtype=torch.int32, device=dev)
    vals = torch.randint(1, 5, (nnz,), device=dev).float()
    return indptr.to(dev), cols, vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--other", type=int, default=1_000_000, help="factor rows gathered by the user side")
    ap.add_argument("--other-item", type=int, default=None, help="factor rows gathered by the item side")
    ap.add_argument("--rank", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--explicit", action="store_true")
    a = ap.parse_args()
    from orange3_spark_amd.models import als as AE
    from orange3_spark_amd.ops import als as A
    dev = torch.device("cuda", 0)
    R, implicit = a.rank, not a.explicit
    res = {"rank": R, "implicit": implicit}
    for side, (n, lo, hi, n_other) in (("user", (a.users, 1, 40, a.other)),
                                       ("item", (a.items, 100, 300, a.other_item or a.other))):
        F = torch.randn((n_other, R), device=dev) / R ** 0.5
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        G = AE.gram(F).float() if implicit else None
        if implicit:
            torch.linalg.eigh(G.double())
        t1.record()
        torch.cuda.synchronize()
        res[side + "_gram_eigh_s"] = t0.elapsed_time(t1) / 1e3
        indptr, cols, vals = csr(n, lo, hi, n_other, R, dev, 7 if side == "user" else 8)
        w, b, pos = AE._weights(vals, implicit, 1.0)
        rows = torch.repeat_interleave(torch.arange(n, device=dev), indptr[1:] - indptr[:-1])
        lam = (0.1 * torch.zeros(n, device=dev).index_add_(0, rows, pos.float())).contiguous()
        out = torch.empty((n, R), device=dev)
        A.exact_solve(indptr, cols, w, b, F, G, lam, implicit, out)
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            A.exact_solve(indptr, cols, w, b, F, G, lam, implicit, out)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 1e3)
        small = int(((indptr[1:] - indptr[:-1]) <= 32).sum())
        res[side] = {"rows": n, "other_rows": n_other, "ratings": int(indptr[-1]), "woodbury_rows": small, "dense_rows": n - small,
                     "s": best, "rows_per_s": n / best, "finite": bool(torch.isfinite(out).all())}
        print(side, res[side], flush=True)
        del F, out, indptr, cols, vals, w, b, pos, rows, lam
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
