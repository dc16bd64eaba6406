#!/usr/bin/env python
"""Phase breakdown of the dense exact-ALS kernel (als_dense_mfma_kernel, rank 128,
implicit) with its diagnostic TIM build: per-block shader-clock cycles of the Gram, the
diagonal factorisations, the panel products, the trailing updates and the backward solve,
on item rows shaped like the ALS config (100..300 ratings over a 50M-row factor table).
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
    ap.add_argument("--other", type=int, default=8_000_000)
    ap.add_argument("--gl", type=int, default=1, help="phase-time the LDS-DMA ring variant")
    a = ap.parse_args()
    from orange3_spark_amd.models import als as AE
    from orange3_spark_amd.ops import _native as N
    dev = torch.device("cuda", 0)
    R = 128
    g = torch.Generator(device="cpu").manual_seed(8)
    lens = torch.randint(100, 301, (a.items,), generator=g)
    indptr = torch.zeros(a.items + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    indptr = indptr.to(dev)
    cols = torch.randint(0, a.other, (nnz,), dtype=torch.int32, device=dev)
    vals = torch.randint(1, 5, (nnz,), device=dev).float()
    F = torch.randn((a.other, R), device=dev) / R ** 0.5
    G = AE.gram(F).float().contiguous()
    w, b, pos = AE._weights(vals, True, 1.0)
    rows = torch.repeat_interleave(torch.arange(a.items, device=dev), indptr[1:] - indptr[:-1])
    lam = (0.1 * torch.zeros(a.items, device=dev).index_add_(0, rows, pos.float())).contiguous()
    dense = torch.arange(a.items, dtype=torch.int32, device=dev)
    out = torch.empty((a.items, R), device=dev)
    tim = torch.zeros((a.items, 6), dtype=torch.int64, device=dev)
    lib = N.kernels()
    st = N.stream_of(out)

    def prod_gl():
        N.check(lib.o3s_als_dense_mfma_gl(1, R, indptr.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                          F.data_ptr(), G.data_ptr(), lam.data_ptr(), dense.data_ptr(), a.items,
                                          out.data_ptr(), st), "dense_gl")

    def prod():
        N.check(lib.o3s_als_dense_mfma_blk(1, R, indptr.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                           F.data_ptr(), G.data_ptr(), lam.data_ptr(), dense.data_ptr(), a.items,
                                           out.data_ptr(), st), "dense")

    def timed():
        N.check(lib.o3s_als_dense_mfma_timed(int(a.gl), indptr.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                             F.data_ptr(), G.data_ptr(), lam.data_ptr(), dense.data_ptr(), a.items,
                                             out.data_ptr(), tim.data_ptr(), st), "dense_timed")
    res = {}
    for name, fn in (("production_blk", prod), ("production_gl", prod_gl), ("timed", timed)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        res[name + "_ms"] = e0.elapsed_time(e1)
    m = tim.double().mean(0).tolist()
    names = ["gram", "diag_factor", "panel_products", "trailing_updates_wave0", "backward", "total"]
    res["cycles_per_block_mean"] = dict(zip(names, [round(x) for x in m]))
    res["share_of_block"] = {k: round(v / m[5], 3) for k, v in zip(names[:5], m[:5])}
    res["items"], res["other_rows"], res["ratings"], res["timed_variant"] = a.items, a.other, nnz, \
        "mfma_gl" if a.gl else "mfma_blk"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
