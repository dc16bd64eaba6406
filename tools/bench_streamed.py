#!/usr/bin/env python
"""MEMORY_AND_DISK streaming rate of the GLM pass (frame/spill.py): a bf16 N x 256 table
whose rows beyond an HBM budget live in pinned host memory.  Reports, per fit iteration,
the rows/s over resident rows, over streamed rows, and the PCIe bound (a raw pinned
host -> device copy of the same chunk size on the same GPU).  Also checks the streamed
fit's coefficients against the all-resident fit.  One JSON line.

Reference call sites: ``df.cache()`` (orangecontrib/spark/widgets/data/spark_df_cache.py:39)
then the Classification widget's ``fit`` (orangecontrib/spark/base/spark_ml_estimator.py:22).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=120_000_000)
    ap.add_argument("--features", type=int, default=256)
    ap.add_argument("--resident", type=float, default=0.25, help="share of rows kept in HBM")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--chunk-mb", type=int, default=512)
    a = ap.parse_args()
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.frame import spill
    from orange3_spark_amd.frame.dataframe import StorageLevel
    from orange3_spark_amd.ml.classification import LogisticRegression
    spill.CHUNK_BYTES = a.chunk_mb << 20
    s = Session(SessionConf().set("spark.master", "local[1]").set("spark.executor.instances", "1"))
    df = s.synthetic.classification(a.rows, a.features, seed=11, resident_fraction=1.0).cache()
    kw = dict(solver="sgd", maxIter=a.iters, stepSize=1.0, tol=0.0, regParam=0.0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    ref = LogisticRegression(**kw).fit(df)
    torch.cuda.synchronize()
    t_res = time.perf_counter() - t
    ld = df.column_data("features").ld
    keep = int(a.rows * a.resident)
    s.conf.set("o3s.storage.hbmBudget", str(keep * ld * 2))
    t = time.perf_counter()
    sp = df.select("features", "label").persist(StorageLevel.MEMORY_AND_DISK)
    del df
    torch.cuda.synchronize()
    t_spill = time.perf_counter() - t
    col = sp.column_data("features")
    print(f"[bench_streamed] spilled {col.spilled_rows} rows ({col.host.numel() * 2 / 2**30:.1f} GiB pinned) "
          f"in {t_spill:.1f}s", file=sys.stderr, flush=True)
    LogisticRegression(**dict(kw, maxIter=1)).fit(sp)           # warm the streamer buffers
    torch.cuda.synchronize()
    t = time.perf_counter()
    m = LogisticRegression(**kw).fit(sp)
    torch.cuda.synchronize()
    t_str = time.perf_counter() - t
    # PCIe bound: raw pinned H2D of one chunk, repeated
    st = col.streamer()
    rows = st.chunk_rows
    dst = torch.empty((rows, ld), dtype=torch.bfloat16, device="cuda")
    src = col.host[:rows]
    for _ in range(3):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    reps = 20
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    h2d = reps * src.numel() * 2 / (time.perf_counter() - t)
    passes = a.iters                                   # the stats pass is fused with iteration 1
    res_rate = a.rows * passes / t_res
    # streamed-pass time minus the resident rows' share at the resident rate
    t_stream_only = t_str - col.resident_rows * passes / res_rate
    out = {"metric": "GLM pass over host-streamed rows (MEMORY_AND_DISK)", "unit": "rows/s",
           "value": col.spilled_rows * passes / max(t_stream_only, 1e-9), "mode": "resident+streamed",
           "rows": a.rows, "features": a.features, "resident_rows": col.resident_rows,
           "streamed_rows": col.spilled_rows, "iters": a.iters, "chunk_mb": a.chunk_mb,
           "fit_s_all_resident": round(t_res, 4), "fit_s_streamed": round(t_str, 4),
           "resident_rows_per_s": res_rate, "streamed_rows_per_s_total": a.rows * passes / t_str,
           "pcie_h2d_bytes_per_s": h2d, "pcie_bound_rows_per_s": h2d / (ld * 2),
           "streamed_share_of_pcie_bound": (col.spilled_rows * passes / max(t_stream_only, 1e-9)) / (h2d / (ld * 2)),
           "coef_max_abs_diff": float(np.abs(m.coefficients.toArray() - ref.coefficients.toArray()).max()),
           "spill_seconds_untimed": round(t_spill, 2), "dtype": "bf16", "data": "synthetic"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
