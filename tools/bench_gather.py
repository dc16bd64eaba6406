"""Random-row gather rate (the floor of an exact ALS iteration).

Gathers ``--rows`` random rows (uniform indices, like the ratings of the ALS config) of
an [n, R] fp32 table with ``o3s_gather_probe`` (csrc/probe.hip) for several table sizes and
grids, and reports GB/s of row bytes.  Compare with the ALS kernels: one ALS iteration of
the 50M x 5M x 1B config gathers 1B rows from each side (1.02 TB at rank 128)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd.ops import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200_000_000)
    ap.add_argument("--rank", type=int, default=128)
    ap.add_argument("--tables", default="1000000,6250000,50000000")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    R = a.rank
    lib = N.kernels()
    res = {"rank": R, "rows_gathered": a.rows, "row_bytes": R * 4, "runs": []}
    ncu = N.num_cus(dev)
    for n in (int(x) for x in a.tables.split(",")):
        F = torch.randn((n, R), device=dev)
        idx = torch.randint(0, n, (a.rows,), device=dev, dtype=torch.int32)
        for per_cu in (4, 16, 64):
            grid = ncu * per_cu
            out = torch.empty((grid * 4 * 64 * 4,), device=dev)
            N.check(lib.o3s_gather_probe(F.data_ptr(), R, idx.data_ptr(), a.rows, grid, out.data_ptr(),
                                         N.stream_of(F)), "gather_probe")
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                N.check(lib.o3s_gather_probe(F.data_ptr(), R, idx.data_ptr(), a.rows, grid, out.data_ptr(),
                                             N.stream_of(F)), "gather_probe")
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / 3
            res["runs"].append({"table_rows": n, "table_GB": round(n * R * 4 / 1e9, 2), "grid": grid,
                                "seconds": round(dt, 5), "GBps": round(a.rows * R * 4 / dt / 1e9, 1)})
            print(json.dumps(res["runs"][-1]), flush=True)
        del F, idx
        torch.cuda.empty_cache()
    best = max(r["GBps"] for r in res["runs"])
    res["best_GBps"] = best
    res["als_iteration_floor_s"] = round(2 * 1_000_000_000 * R * 4 / (best * 1e9), 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
