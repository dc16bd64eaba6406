#!/usr/bin/env python
"""Phase breakdown of the dense exact-ALS kernel (als_dense_wave_kernel, rank 128, implicit)
with its diagnostic TIM build: per-wave shader-clock cycles of the row setup, the Gram loop
(and of it, the part spent inside advance(): issuing the next DMA step and waiting for the
ring), the blocked Cholesky + forward solve, and the backward solve + store, on item rows
shaped like the ALS config's item side (~200 ratings each over a rotated user table).
Also times the production kernel on the same rows."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=625_000)
    ap.add_argument("--other", type=int, default=5_000_000)
    ap.add_argument("--mean", type=int, default=200)
    a = ap.parse_args()
    from orange3_spark_amd.models import als as AE
    from orange3_spark_amd.ops import _native as N
    from orange3_spark_amd.ops import als as AO
    dev = torch.device("cuda", 0)
    R = 128
    g = torch.Generator(device="cpu").manual_seed(11)
    lens = torch.randint(a.mean // 2, a.mean * 3 // 2 + 1, (a.items,), generator=g)
    indptr = torch.zeros(a.items + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    indptr = indptr.to(dev)
    cols = torch.randint(0, a.other, (nnz,), dtype=torch.int32, device=dev)
    vals = torch.randint(1, 5, (nnz,), device=dev).float()
    F = torch.randn((a.other, R), device=dev) / R ** 0.5
    G = torch.diag(torch.rand(R, device=dev) * a.other / R).contiguous()
    w, b, pos = AE._weights(vals, True, 1.0)
    rows = torch.repeat_interleave(torch.arange(a.items, device=dev), indptr[1:] - indptr[:-1])
    lam = (0.1 * torch.zeros(a.items, device=dev).index_add_(0, rows, pos.float())).clamp_min(0.1).contiguous()
    order = torch.argsort(lens.to(dev), descending=True).to(torch.int32)
    meta = AO.dense_meta(indptr, order, lam)
    out = torch.empty((a.items, R), device=dev)
    lib = N.kernels()
    grid = N.num_cus(dev)
    tim = torch.zeros((grid * 4, 10), dtype=torch.int64, device=dev)
    st = N.stream_of(out)

    def prod():
        N.check(lib.o3s_als_dense_wave(1, R, meta.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                       F.data_ptr(), G.data_ptr(), a.items, out.data_ptr(), grid, st), "dense")

    gd = torch.diagonal(G).contiguous()

    def prod_gd():
        N.check(lib.o3s_als_dense_wave_gd(R, meta.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                          F.data_ptr(), gd.data_ptr(), a.items, out.data_ptr(), grid, st),
                "dense_gd")

    def timed():
        N.check(lib.o3s_als_dense_wave_timed(meta.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                             F.data_ptr(), G.data_ptr(), a.items, out.data_ptr(), grid,
                                             tim.data_ptr(), st), "dense_timed")
    res = {"items": a.items, "ratings": nnz, "mean_ratings": round(nnz / a.items, 1), "grid": grid}
    runs = (("production", prod), ("production_gdiag", prod_gd))
    for name, fn in list(runs) * 3 + [("timed", timed)]:     # production A/B alternated (box noise)
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(name + "_ms", []).append(round(e0.elapsed_time(e1), 3))
    t = tim.double()
    waves = int((t.sum(1) > 0).sum())
    tot = t.sum(0)
    names = ["setup", "gram", "factor_forward", "backward_store", "gram_produce", "factor_A_diag",
             "factor_handoff", "factor_B", "factor_C", "gram_dma_wait"]
    per_row = {n: round(float(tot[i]) / a.items, 1) for i, n in enumerate(names)}
    res["cycles_per_row"] = per_row
    res["cycles_per_rating"] = {n: round(float(tot[i]) / nnz, 2) for i, n in enumerate(names)}
    res["busy_waves"] = waves
    res["max_wave_cycles"] = float(t.sum(1).max())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
