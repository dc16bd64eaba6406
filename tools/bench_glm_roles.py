"""Per-role timing of the one-launch mixed GLM pass (csrc/glm.hip glm_grad_mixed_kernel):
resident-only, lineage-only and mixed, plus the single-role kernels, on one GPU.

  python tools/bench_glm_roles.py [--rows 125000000] [--d 256] [--grid 8192] [--waves 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from orange3_spark_amd.ops import glm as G


def timed(fn, reps=5):
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
    ap.add_argument("--rows", type=int, default=125_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--grid", type=int, default=8192)
    ap.add_argument("--waves", type=int, default=3)
    ap.add_argument("--mode", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    G.MIX_WAVES = a.waves
    G.MIX_MODE = a.mode
    n, d, seed = a.rows, a.d, 5
    wt, bt = G.synth_truth(seed, d)
    X, y = G.synth_glm(n, d, seed, device=dev, wtrue=wt, btrue=bt)
    y2 = torch.cat([y, y])
    coef = (torch.randn(d, generator=torch.Generator().manual_seed(1)) * 0.02).to(dev)
    ws = G.GlmWorkspace(dev, d, grid=a.grid)
    ws8 = G.GlmWorkspace(dev, d)
    empty = X[:0]
    r = {"rows": n, "d": d, "grid": a.grid, "waves": a.waves, "mode": a.mode}
    r["mixed_res_only_ms"] = timed(lambda: G.glm_grad_mixed(X, y, None, 0, d, seed, n, coef, 0.0, 0, ws))
    r["mixed_lin_only_ms"] = timed(lambda: G.glm_grad_mixed(empty, y, None, n, d, seed, 0, coef, 0.0, 0, ws))
    r["mixed_both_ms"] = timed(lambda: G.glm_grad_mixed(X, y2, None, n, d, seed, n, coef, 0.0, 0, ws))
    if a.mode != 0:
        print(json.dumps(r, indent=1))
        return
    r["res_kernel_ms"] = timed(lambda: G.glm_grad(X, y, None, coef, 0.0, 0, ws8))
    r["lin_kernel_ms"] = timed(lambda: G.glm_grad_synth(n, d, d, seed, 0, wt, bt, coef, 0.0, 0, ws8))
    gb = n * d * 2 / 1e9
    r["mixed_res_only_TBps"] = gb / r["mixed_res_only_ms"]
    r["res_kernel_TBps"] = gb / r["res_kernel_ms"]
    r["mixed_lin_only_Grows_s"] = n / r["mixed_lin_only_ms"] / 1e6
    r["lin_kernel_Grows_s"] = n / r["lin_kernel_ms"] / 1e6
    print(json.dumps(r, indent=1))


if __name__ == "__main__":
    main()
