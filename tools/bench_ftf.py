#!/usr/bin/env python
"""F^T F of an ALS factor table: ftf_kernel vs the chunked hipBLASLt fp32 GEMMs it replaced."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from orange3_spark_amd.ops import als as A
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    R = 128
    F = torch.randn((n, R), device="cuda") / R ** 0.5

    def gemm_chunks(chunk=1 << 20):
        out = torch.zeros((R, R), dtype=torch.float64, device=F.device)
        for a in range(0, n, chunk):
            Fc = F[a:a + chunk]
            out += (Fc.T @ Fc).double()
        return out

    res = {"rows": n, "rank": R}
    for name, fn in (("ftf_kernel", lambda: A.ftf(F)), ("hipblaslt_chunks", gemm_chunks)):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            out = fn()
        torch.cuda.synchronize()
        res[name + "_ms"] = (time.perf_counter() - t) / 3 * 1e3
        res[name + "_sample"] = float(out[5, 7])
    ref = A.ftf(F[: 1_000_000]) - (F[: 1_000_000].double().T @ F[: 1_000_000].double())
    res["ftf_max_abs_err_1M_rows"] = float(ref.abs().max())
    res["GB_per_s_ftf"] = n * R * 4 / res["ftf_kernel_ms"] / 1e6
    print(json.dumps(res))


if __name__ == "__main__":
    main()
