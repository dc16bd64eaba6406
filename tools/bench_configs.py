#!/usr/bin/env python
"""Full BASELINE configs through the public estimator API on ONE process (N = 1 point of
the curves; under torchrun each rank holds 1/N of the rows).

* ``--config als``: ``ALS(rank=128, implicitPrefs=True).fit`` on 50M users x 5M items with
  1B ratings (BASELINE "ALS implicit rank=128, 50M users x 5M items").
* ``--config gbt``: ``GBTClassifier(maxDepth=8).fit`` on 500M x 64 (BASELINE "GBTClassifier
  depth=8, 500M x 64").

Data generation (on device, synthetic) is untimed; the ``fit`` is timed end to end
(setup: id maps / rating partitions / binning, then every iteration / tree).  One JSON line
per run in the bench.py key schema.  Reference call site of both fits: the Recommendation /
Classification widgets' ``method().fit(in_df, params=...)``
(orangecontrib/spark/base/spark_ml_estimator.py:19-25).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _mem_gb():
    return round(torch.cuda.max_memory_allocated() / 2**30, 1) if torch.cuda.is_available() else None


def _alloc_stats():
    """Caching-allocator events of the run: retries (an allocation that first failed and
    flushed the cache) and device mallocs / frees (each a synchronising hipMalloc/hipFree)."""
    if not torch.cuda.is_available():
        return None
    st = torch.cuda.memory_stats()
    return {"num_alloc_retries": st.get("num_alloc_retries"), "num_device_alloc": st.get("num_device_alloc"),
            "num_device_free": st.get("num_device_free"), "reserved_gb": round(torch.cuda.memory_reserved() / 2**30, 1)}


def run_als(s, a):
    from orange3_spark_amd.ml.recommendation import ALS
    from orange3_spark_amd.runtime.tracing import TRACER
    t0 = time.perf_counter()
    df = s.synthetic.ratings(a.users, a.items, a.ratings, rank=8, seed=1, implicit=True)
    _sync()
    t_gen = time.perf_counter() - t0
    print(f"[bench_configs] ratings generated in {t_gen:.1f}s", file=sys.stderr, flush=True)
    est = ALS(rank=a.rank, implicitPrefs=True, maxIter=a.iters, regParam=0.1, alpha=1.0, seed=0)
    TRACER.reset()
    s.comm.barrier()
    _sync()
    t1 = time.perf_counter()
    model = est.fit(df)
    _sync()
    s.comm.barrier()
    fit_s = time.perf_counter() - t1
    its = list(model.iterationSeconds)
    per_iter = sorted(its)[len(its) // 2]
    setup_s = fit_s - sum(its)
    out = {"metric": "ALS implicit seconds per iteration (rank 128, 50M x 5M, 1B ratings)",
           "value": per_iter, "unit": "s/iter", "higher_is_better": False, "n_gpus": s.comm.world_size,
           "dtype": "fp32", "data": "synthetic", "mode": "resident",
           "config": {"model": "ALS implicitPrefs=True rank=128", "users": a.users, "items": a.items,
                      "ratings": a.ratings, "maxIter": a.iters, "parallelism": f"dp{s.comm.world_size}"},
           "fit_seconds": round(fit_s, 3), "setup_seconds": round(setup_s, 3), "iter_seconds": its,
           "datagen_seconds_untimed": round(t_gen, 2), "max_mem_gb": _mem_gb(),
           "phases_s": ({k: round(v["total_s"], 4) for k, v in TRACER.summary().items()}
                        if TRACER.enabled else None)}
    if TRACER.enabled:   # the fit's spans in order (iteration 1 vs the steady state)
        out["events_ms"] = [[n, round(dt * 1e3, 2)] for n, _t, dt, _a, _tid in TRACER._events
                            if n.startswith("als.") and not n.startswith("als.gather")][:400]
    return out


def run_gbt(s, a):
    from orange3_spark_amd.ml.classification import GBTClassifier
    from orange3_spark_amd.runtime.tracing import TRACER
    t0 = time.perf_counter()
    df = s.synthetic.trees(a.rows, a.features, seed=5)
    _sync()
    t_gen = time.perf_counter() - t0
    print(f"[bench_configs] rows generated in {t_gen:.1f}s", file=sys.stderr, flush=True)
    est = GBTClassifier(maxDepth=a.depth, maxIter=a.trees, stepSize=0.1, seed=0)
    if a.prewarm:                       # a tiny fit first: code-object loading, first-use setup
        t_w = time.perf_counter()
        GBTClassifier(maxDepth=a.depth, maxIter=2, stepSize=0.1, seed=0).fit(s.synthetic.trees(100_000, a.features, seed=6))
        _sync()
        print(f"[bench_configs] prewarm fit {time.perf_counter() - t_w:.2f}s", file=sys.stderr, flush=True)
    # the fit is timed --repeat times in this process: the first (cold) fit's fresh device
    # allocations (the 32 GB feature-major copy) are cleared by the driver before first use
    # (~1.6 s on a box whose memory a previous process used); later fits reuse the caching
    # allocator's blocks, as in a long-running session.  value = the last (warm) fit.
    fits, phases_each = [], []
    for _ in range(max(1, a.repeat)):
        TRACER.reset()
        s.comm.barrier()
        _sync()
        t1 = time.perf_counter()
        model = est.fit(df)
        _sync()
        s.comm.barrier()
        fits.append(time.perf_counter() - t1)
        if TRACER.enabled:
            phases_each.append({k: round(v["total_s"], 4) for k, v in TRACER.summary().items()})
    fit_s = fits[-1]
    ph = {k: round(v["total_s"], 4) for k, v in TRACER.summary().items()} if TRACER.enabled else None
    prep = None
    if ph:
        prep = sum(v for k, v in ph.items() if k in ("tree.find_splits", "tree.bin_features"))
    out = {"metric": "GBTClassifier seconds per tree (depth 8, 500M x 64)",
           "value": fit_s / a.trees, "unit": "s/tree", "higher_is_better": False, "n_gpus": s.comm.world_size,
           "dtype": "fp32", "data": "synthetic", "mode": "resident",
           "config": {"model": f"GBTClassifier maxDepth={a.depth} maxBins=32", "rows": a.rows,
                      "features": a.features, "maxIter": a.trees, "parallelism": f"dp{s.comm.world_size}"},
           "fit_seconds": round(fit_s, 3), "fit_seconds_each": [round(x, 3) for x in fits], "binning_seconds": prep,
           "per_tree_excl_binning_s": (round((fit_s - prep) / a.trees, 4) if prep is not None else None),
           "train_loss": [round(x, 5) for x in model.trainingLossHistory][-3:],
           "datagen_seconds_untimed": round(t_gen, 2), "max_mem_gb": _mem_gb(), "alloc": _alloc_stats(),
           "phases_s": ph, "phases_each_fit_s": phases_each or None}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("als", "gbt"), required=True)
    ap.add_argument("--users", type=int, default=50_000_000)
    ap.add_argument("--items", type=int, default=5_000_000)
    ap.add_argument("--ratings", type=int, default=1_000_000_000)
    ap.add_argument("--rank", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--rows", type=int, default=500_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--trees", type=int, default=5)
    ap.add_argument("--repeat", type=int, default=2, help="GBT: fits timed in one process (value = the last)")
    ap.add_argument("--trace", action="store_true", help="per-phase timings (synchronising tracer)")
    ap.add_argument("--prewarm", action="store_true", help="GBT: one tiny untimed fit before the timed ones")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from orange3_spark_amd import Session
    from orange3_spark_amd.conf import SessionConf
    conf = SessionConf()
    if a.trace:
        conf.set("o3s.trace", "true").set("o3s.trace.sync", "true")
    s = Session.getOrCreate(conf)
    out = run_als(s, a) if a.config == "als" else run_gbt(s, a)
    out["session_warmup_s_untimed"] = getattr(s, "warmup_seconds", None)
    if s.comm.rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
