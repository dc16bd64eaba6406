"""Footprint experiment for the mixed GLM pass: one launch over all resident rows vs K
launches over 1/K row slices (same kernel, same grid).  Static grid-stride tile walks
drift apart over a long launch, widening the address window the waves touch; splitting
the pass restarts the waves in lockstep every 1/K of the table.

  python tools/bench_glm_split.py [--rows 480000000] [--grid 3072]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from orange3_spark_amd.ops import glm as G


def timed(fn, reps=4):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=480_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--grid", type=int, default=3072)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, d, seed = a.rows, a.d, 5
    wt, bt = G.synth_truth(seed, d)
    X, y = G.synth_glm(n, d, seed, device=dev, wtrue=wt, btrue=bt)
    y2 = torch.cat([y, y])
    coef = (torch.randn(d, generator=torch.Generator().manual_seed(1)) * 0.02).to(dev)
    ws = G.GlmWorkspace(dev, d, grid=a.grid)
    r = {"rows": n, "d": d, "grid": a.grid}
    for K in (1, 2, 4, 8, 16):
        k = (n + K - 1) // K
        sl = [(i * k, min(n, (i + 1) * k)) for i in range(K)]

        def res_only():
            for lo, hi in sl:
                G.glm_grad_mixed(X[lo:hi], y[lo:hi], None, 0, d, seed, n, coef, 0.0, 0, ws)

        def both():
            for lo, hi in sl:
                yy = torch.cat([y[lo:hi], y[lo:hi]]) if K > 1 else y2
                G.glm_grad_mixed(X[lo:hi], yy, None, hi - lo, d, seed, n + lo, coef, 0.0, 0, ws)
        ys = [torch.cat([y[lo:hi], y[lo:hi]]) for lo, hi in sl]

        def both_pre():
            for (lo, hi), yy in zip(sl, ys):
                G.glm_grad_mixed(X[lo:hi], yy, None, hi - lo, d, seed, n + lo, coef, 0.0, 0, ws)
        r[f"K{K}_res_only_ms"] = timed(res_only)
        r[f"K{K}_res_only_TBps"] = n * d * 2 / 1e9 / r[f"K{K}_res_only_ms"]
        r[f"K{K}_both_ms"] = timed(both_pre)
        del ys
        print(json.dumps({k2: v for k2, v in r.items() if k2.startswith(f"K{K}_")}), flush=True)
    print(json.dumps(r, indent=1))


if __name__ == "__main__":
    main()
