"""Phase split of kmeanspp_kernel (one workgroup, all k greedy k-means++ steps) on a
k-means||-sized candidate set: m = 4097 candidates x D = 128, k = 1024, 8 trials.  Prints
thread 0's shader-clock totals per phase (scan, draw, candidate rows, distances +
potentials, pick, d2 update) and the kernel wall time."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd.models import kmeans as KM  # noqa: E402


def main():
    m, D, k = int(os.environ.get("M", 4097)), 128, 1024
    g = torch.Generator(device="cpu").manual_seed(1)
    P = (torch.randn(m, D, generator=g, dtype=torch.float64) * 3).cuda()
    w = torch.randint(1, 5000, (m,), generator=g).to(torch.float64).cuda()
    KM._local_kmeanspp(P, w, k, seed=3, iters=0)              # warm
    tim = torch.zeros(6, dtype=torch.int64, device="cuda")
    KM.KPP_TIMING = tim
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    KM._local_kmeanspp(P, w, k, seed=3, iters=0)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    KM.KPP_TIMING = None
    cyc = tim.cpu().tolist()
    tot = sum(cyc)
    names = ["scan", "draw", "candidate_rows", "distances_potentials", "pick", "d2_update"]
    print(json.dumps({"m": m, "D": D, "k": k, "wall_s": wall, "cycles_total": tot,
                      "share": {n: round(c / max(tot, 1), 3) for n, c in zip(names, cyc)},
                      "cycles_per_step": {n: round(c / (k - 1)) for n, c in zip(names, cyc)}}))


if __name__ == "__main__":
    main()
