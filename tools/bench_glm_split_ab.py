"""A/B of the mixed GLM pass as one launch vs K launches over row slices, alternating
the two several times (same data, same grid): is the split gain above run-to-run noise?

  python tools/bench_glm_split_ab.py [--rows 480000000] [--k 16] [--rounds 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from orange3_spark_amd.ops import glm as G


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=480_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--grid", type=int, default=3072)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, d, seed = a.rows, a.d, 5
    wt, bt = G.synth_truth(seed, d)
    X, y = G.synth_glm(n, d, seed, device=dev, wtrue=wt, btrue=bt)
    coef = (torch.randn(d, generator=torch.Generator().manual_seed(1)) * 0.02).to(dev)
    ws = G.GlmWorkspace(dev, d, grid=a.grid)
    plans = {}
    for K in (1, a.k):
        k = (n + K - 1) // K
        sl = [(i * k, min(n, (i + 1) * k)) for i in range(K)]
        plans[K] = [(lo, hi, torch.cat([y[lo:hi], y[lo:hi]])) for lo, hi in sl]

    def run(K):
        for lo, hi, yy in plans[K]:
            G.glm_grad_mixed(X[lo:hi], yy, None, hi - lo, d, seed, n + lo, coef, 0.0, 0, ws)

    res = {1: [], a.k: []}
    for K in (1, a.k):
        run(K)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for K in (1, a.k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                run(K)
            e1.record()
            torch.cuda.synchronize()
            res[K].append(e0.elapsed_time(e1) / 3)
        print(json.dumps({f"K{K}": round(v[-1], 3) for K, v in res.items()}), flush=True)
    print(json.dumps({"rows": n, "grid": a.grid, "K1_ms": res[1], f"K{a.k}_ms": res[a.k],
                      "K1_min": min(res[1]), f"K{a.k}_min": min(res[a.k])}))


if __name__ == "__main__":
    main()
