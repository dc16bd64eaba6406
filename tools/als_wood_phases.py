#!/usr/bin/env python
"""Phase breakdown of the Woodbury exact-ALS kernel (als_wood_kernel, rank 128, implicit)
with its diagnostic TIM build: per-row shader-clock cycles of the factor-row gathers, the
S = P D P^T build (MFMA + LDS image), the n x n Cholesky, the two triangular solves and the
output, on user rows shaped like the ALS config (1..32 ratings over a 5M-row rotated item
table).  Also times the production kernel on the same rows."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=2_000_000)
    ap.add_argument("--other", type=int, default=5_000_000)
    ap.add_argument("--kn", type=int, default=32, choices=(16, 24, 32),
                    help="launch width; rows get kn/2+1..kn ratings (1..16 for kn 16)")
    a = ap.parse_args()
    from orange3_spark_amd.models import als as AE
    from orange3_spark_amd.ops import _native as N
    dev = torch.device("cuda", 0)
    R = 128
    g = torch.Generator(device="cpu").manual_seed(9)
    lo_len = 1 if a.kn == 16 else (17 if a.kn == 24 else 25)
    lens = torch.randint(lo_len, a.kn + 1, (a.users,), generator=g)
    indptr = torch.zeros(a.users + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    indptr = indptr.to(dev)
    cols = torch.randint(0, a.other, (nnz,), dtype=torch.int32, device=dev)
    vals = torch.randint(1, 5, (nnz,), device=dev).float()
    P = torch.randn((a.other, R), device=dev) / R ** 0.5
    eig = (torch.rand(R, device=dev) * a.other / R).contiguous()
    w, b, pos = AE._weights(vals, True, 1.0)
    rows = torch.repeat_interleave(torch.arange(a.users, device=dev), indptr[1:] - indptr[:-1])
    lam = (0.1 * torch.zeros(a.users, device=dev).index_add_(0, rows, pos.float())).clamp_min(0.1).contiguous()
    small = torch.arange(a.users, dtype=torch.int32, device=dev)
    out = torch.empty((a.users, R), device=dev)
    tim = torch.zeros((a.users, 5), dtype=torch.int64, device=dev)
    lib = N.kernels()
    st = N.stream_of(out)

    def prod():
        N.check(lib.o3s_als_wood_kn(R, a.kn, indptr.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                    P.data_ptr(), eig.data_ptr(), lam.data_ptr(), small.data_ptr(), a.users,
                                    out.data_ptr(), st), "wood")

    def timed():
        N.check(lib.o3s_als_wood_timed(a.kn, indptr.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(), P.data_ptr(),
                                       eig.data_ptr(), lam.data_ptr(), small.data_ptr(), a.users, out.data_ptr(),
                                       tim.data_ptr(), st), "wood_timed")
    res = {}
    # A/B of the build switches (csrc/als_exact.hip), alternated, 5 rounds: min / median ms
    variants = {"s16": "1", "s32": "0"} if a.kn != 16 else {"s16": "1"}
    ab = {k: [] for k in variants}
    for rep in range(5):
        for k, s16 in variants.items():
            os.environ["O3S_ALS_WOOD24_16"] = s16
            prod()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            prod()
            e1.record()
            torch.cuda.synchronize()
            ab[k].append(e0.elapsed_time(e1))
    os.environ.pop("O3S_ALS_WOOD24_16")
    res["ab_ms"] = {k: {"min": round(min(v), 3), "median": round(sorted(v)[len(v) // 2], 3)} for k, v in ab.items()}
    for name, fn in (("production", prod), ("timed", timed)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        res[name + "_ms"] = e0.elapsed_time(e1)
    m = tim.double().mean(0).tolist()
    names = ["gathers", "s_build", "cholesky", "solves", "output"]
    tot = sum(m)
    res["cycles_per_row_mean"] = dict(zip(names, [round(x) for x in m]))
    res["share_of_row"] = {k: round(v / tot, 3) for k, v in zip(names, m)}
    res["kn"] = a.kn
    res["users"], res["other_rows"], res["ratings"], res["mean_len"] = a.users, a.other, nnz, nnz / a.users
    res["ns_per_row_production"] = res["production_ms"] * 1e6 / a.users
    print(json.dumps(res))


if __name__ == "__main__":
    main()
