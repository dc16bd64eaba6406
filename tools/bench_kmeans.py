"""BASELINE config 2: KMeans k=1024 on 100M x 128 fp32, 1 MI355X.

Times Lloyd iterations (assign MFMA kernel + slab update kernel + all-reduce + centre
update); prints one JSON line (samples/s per iteration).

``--data blobs`` (well-separated Gaussian clusters) vs ``--data uniform`` (U[-1,1]^d: no
cluster structure, so many rows sit near a Voronoi boundary); ``--init offset`` (true
centres + 0.5, blobs only) vs ``--init kmeans||`` (Spark's default k-means|| init, timed
separately).  The JSON reports ``flagged_fraction`` -- the share of rows whose one-MFMA
fp16 screen could not certify the argmin and were re-solved by the split-precision kernel
-- and the assign rate as ``fp16_screen_tflops`` (screen mode: 2 N K D / t with ONE fp16
MFMA per k-step, not an fp32 rate) or ``split_fp32_equiv_tflops`` (split mode: three bf16
MFMAs emulate fp32).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session  # noqa: E402
from orange3_spark_amd.ops import kmeans as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--torch-baseline", action="store_true", help="also time a torch (rocBLAS GEMM) assign")
    ap.add_argument("--mode", default="auto", choices=["auto", "screen", "split"],
                    help="assign path: one-MFMA screen + near-tie re-solve, or split precision everywhere")
    ap.add_argument("--data", default="blobs", choices=["blobs", "uniform"])
    ap.add_argument("--init", default=None, choices=["offset", "kmeans||"],
                    help="default: offset for blobs, kmeans|| for uniform")
    ap.add_argument("--presplit", default="auto", choices=["auto", "on", "off"],
                    help="screen kernel over pre-split fp16 rows (ops.kmeans.PRESPLIT)")
    ap.add_argument("--cost", default="sums", choices=["sums", "rows"],
                    help="iteration cost from the cluster sums (the fit's path: no per-row distance in the "
                         "assign pass) or from per-row distances")
    a = ap.parse_args()
    K.PRESPLIT = {"auto": None, "on": True, "off": False}[a.presplit]
    init = a.init or ("offset" if a.data == "blobs" else "kmeans||")
    if init == "offset" and a.data != "blobs":
        raise SystemExit("--init offset needs --data blobs (true centres)")
    s = Session.getOrCreate()
    comm = s.comm
    if a.data == "blobs":
        df = s.synthetic.blobs(a.rows, a.d, k=a.k, seed=3, spread=1.0)
        X = df.column_data("features").data
    else:
        X = torch.empty((a.rows, a.d), dtype=torch.float32, device=s.device)
        g = torch.Generator(device=s.device).manual_seed(3)
        for r0 in range(0, a.rows, 1 << 24):
            r1 = min(a.rows, r0 + (1 << 24))
            X[r0:r1].uniform_(-1.0, 1.0, generator=g)
    t_init = None
    if init == "offset":
        C = df.true_centers.float() + 0.5
    else:
        from orange3_spark_amd.models.kmeans import kmeans_parallel_init
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        C = kmeans_parallel_init(comm, X, a.k, 2, 7).float()
        torch.cuda.synchronize()
        t_init = time.perf_counter() - t1
    ws = K.UpdateWorkspace(X.device, (a.k + 31) // 32 * 32, a.d)
    need = a.cost == "rows"
    sumsq = K.moments(X, torch.zeros(a.d, device=X.device))[1]
    torch.cuda.synchronize()

    def it(C):
        prep = K.prepare_centers(C)
        asg, d = K.assign(X, C, prep, mode=a.mode, need_dist=need)
        sums, cnt = K.update(X, asg, ws.K, ws)
        if need:
            cost = d.double().sum()
        else:
            Cd = C.double()
            cost = sumsq - (2.0 * (Cd * sums[: a.k]).sum() - (cnt[: a.k] * (Cd * Cd).sum(1)).sum())
        buf = torch.cat([sums[: a.k].reshape(-1), cnt[: a.k], cost.reshape(1)])
        comm.all_reduce(buf)
        cnt = buf[a.k * a.d: a.k * a.d + a.k]
        sums = buf[: a.k * a.d].reshape(a.k, a.d)
        return torch.where(cnt[:, None] > 0, sums / cnt.clamp_min(1)[:, None], C.double()).float(), float(buf[-1])

    C, _ = it(C)
    torch.cuda.synchronize()
    t_assign = time.perf_counter()
    prep = K.prepare_centers(C)
    st = {}
    for _ in range(a.iters):
        asg, d = K.assign(X, C, prep, mode=a.mode, stats=st, need_dist=need)
    torch.cuda.synchronize()
    t_assign = (time.perf_counter() - t_assign) / a.iters
    t_upd = time.perf_counter()
    for _ in range(a.iters):
        K.update(X, asg, ws.K, ws)
    torch.cuda.synchronize()
    t_upd = (time.perf_counter() - t_upd) / a.iters
    t0 = time.perf_counter()
    cost = None
    for _ in range(a.iters):
        C, cost = it(C)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    flop = 2.0 * a.rows * a.k * a.d
    flagged = st.get("flagged")
    rate_key = "split_fp32_equiv_tflops" if (a.mode == "split" or flagged == a.rows) else "fp16_screen_tflops"
    out = {"metric": "KMeans Lloyd iteration samples/s (k=1024, 100M x 128 fp32)", "value": a.rows / dt,
           "unit": "samples/s", "ms_per_iter": dt * 1e3, "assign_ms": t_assign * 1e3, "update_ms": t_upd * 1e3,
           rate_key: flop / t_assign / 1e12, "rows": a.rows, "d": a.d, "k": a.k, "cost": cost,
           "data": a.data, "cost_from": a.cost, "init": init, "init_s": t_init, "assign_mode": a.mode,
           "near_tie_rows_resolved": flagged, "flagged_fraction": None if flagged is None else flagged / a.rows}
    if a.torch_baseline:
        t1 = time.perf_counter()
        K.assign_torch(X[: 10_000_000], C, chunk=1 << 20)
        torch.cuda.synchronize()
        out["torch_fp64_assign_ms_per_10M"] = (time.perf_counter() - t1) * 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
