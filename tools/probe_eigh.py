#!/usr/bin/env python
"""Times the rank x rank eigendecomposition of the ALS Woodbury path (G = Y^T Y, fp64):
torch.linalg.eigh on the GPU (first call in the process and steady state) vs on the host
(D2H of G, LAPACK, H2D of Q and e)."""
import json
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for R in (128, 64):
        Y = torch.randn(100000, R, device=dev, dtype=torch.float64)
        G = Y.T @ Y
        torch.cuda.synchronize()
        for name, fn in (("gpu", lambda: torch.linalg.eigh(G)),
                         ("host", lambda: [t.to(dev) for t in torch.linalg.eigh(G.cpu())])):
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            first = time.perf_counter() - t
            t = time.perf_counter()
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            res[f"{name}_R{R}"] = {"first_ms": first * 1e3, "steady_ms": (time.perf_counter() - t) * 100}
            print(name, R, res[f"{name}_R{R}"], flush=True)
        ev_g, V_g = torch.linalg.eigh(G)
        ev_h, V_h = torch.linalg.eigh(G.cpu())
        res[f"eig_max_rel_diff_R{R}"] = float(((ev_g.cpu() - ev_h).abs() / ev_h.abs().max()).max())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
