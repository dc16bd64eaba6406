"""Micro-benchmark of the fused GLM gradient pass (bf16 stream) on one GPU.

Prints achieved HBM bandwidth of the materialised pass and rows/s of the
synthetic-lineage (regenerate-in-kernel) pass.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd.ops import glm as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=125_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    X, y = G.synth_glm(a.rows, a.d, seed=1, device=dev)
    torch.cuda.synchronize()
    gen_s = time.time() - t0
    ws = G.GlmWorkspace(dev, X.shape[1])
    coef = torch.full((X.shape[1],), 0.01, device=dev)
    res = {"rows": a.rows, "d": a.d, "gen_s": gen_s}
    for name, fn in (("mem", lambda: G.glm_grad(X, y, None, coef, 0.0, 0, ws)),
                     ("synth", lambda: G.glm_grad_synth(a.rows, X.shape[1], a.d, 1, 0,
                                                       *G.synth_truth(1, a.d), coef, 0.0, 0, ws))):
        fn(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters
        bytes_ = a.rows * (X.shape[1] * 2 + 4)
        res[name] = {"ms": dt * 1e3, "rows_per_s": a.rows / dt,
                     "GBps": bytes_ / dt / 1e9 if name == "mem" else None}
    gm = G.glm_grad(X, y, None, coef, 0.0, 0, ws).clone()
    gs = G.glm_grad_synth(a.rows, X.shape[1], a.d, 1, 0, *G.synth_truth(1, a.d), coef, 0.0, 0, ws).clone()
    res["mem_vs_synth_max_rel"] = float(((gm - gs).abs() / gm.abs().clamp_min(1e-3 * a.rows)).max())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
