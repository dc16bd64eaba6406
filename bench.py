#!/usr/bin/env python
"""Headline benchmark: samples/sec of LogisticRegression.fit on 1B x 256 synthetic data.

BASELINE.json metric: "samples/sec LogisticRegression.fit on 1Bx256 synthetic at
1/2/4/8 MI355X" (config: "LogisticRegression SGD bf16 on 1B x 256 synthetic, row-sharded
DP 8xMI355X").

What is timed: ``LogisticRegression(solver='sgd', maxIter=K, miniBatchFraction=1.0).fit(df)``
end to end -- the summarizer (standardization moments) pass, K gradient-descent
iterations (each one fused bf16 gradient pass over ALL 1B rows sharded over the ranks,
one RCCL all-reduce of the (D+3)-vector, an on-device update), and the model
construction.  The summarizer pass is fused with iteration 1's gradient (both are
functions of the same rows at the all-zero initial iterate), so a K-iteration fit reads
the data K times.  W untimed warm-up fits (maxIter=W) run first.  value = 1B * K / (max
over ranks of the timed fit's wall time).

Strong scaling: the dataset is always 1B x 256 whatever N is.  1B x 256 bf16 = 512 GB:
at N >= 2 every row is resident in HBM; at N = 1 the rows that do not fit in one GPU's
HBM budget are recomputed in-kernel from their generating lineage on every pass (Spark
MEMORY_ONLY semantics; see synthetic.py) -- every sample is still processed every
iteration.  ``hbm_only_rows_per_s`` reports the rate over HBM-resident rows alone (what a
real, fully resident table gets), measured by separate passes after the timed region.

Launch: ``python bench.py --gpus N`` starts N ranks itself (a child
``torch.distributed.run --nproc-per-node N`` process, before anything touches the GPU);
under an existing launcher (WORLD_SIZE set) it runs as one rank.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

METRIC = "samples/sec LogisticRegression.fit on 1Bx256 synthetic at 1/2/4/8 MI355X"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _self_launch(a, argv) -> int:
    """Run this script on ``a.gpus`` ranks through torch.distributed.run as a child
    process (never exec: the parent has not touched the GPU and just relays the exit
    code; rank 0 of the child prints the JSON line straight to our stdout)."""
    args = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *args]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.run(cmd, env=env).returncode


def _hbm_only_rate(df, comm, on_gpu, passes=3):
    """Rows/s of the gradient pass over the HBM-resident rows alone (all ranks)."""
    from orange3_spark_amd.frame import column as C
    from orange3_spark_amd.models import glm as GLM
    feat = df.column_data("features")
    X = feat.data
    y = df.column_data("label").data[: X.shape[0]].to(torch.float32)
    data = GLM.GlmData(comm, C.VectorColumn(X, feat.size), y)
    coef = torch.zeros(data.ws.dpad + 1 if data.kernel else data.ld + 1, dtype=torch.float32, device=X.device)
    run = (lambda: data.pass_device(coef, None, 0)) if data.kernel else (lambda: data.pass_torch(coef[:-1], 0.0, 0))
    comm.all_reduce(run())
    comm.barrier()
    t = time.perf_counter()
    for _ in range(passes):
        comm.all_reduce(run())
    if on_gpu:
        torch.cuda.synchronize()
    comm.barrier()
    el = comm.max_scalar(time.perf_counter() - t)
    return comm.sum_scalar(int(X.shape[0])) * passes / el


def _allreduce_us(comm, n, on_gpu, reps=50):
    """Median wall time (us, max over ranks) of one all-reduce of the step's gradient
    vector (n fp32: coefficients + intercept + loss + count), synchronised per call."""
    import statistics
    buf = torch.zeros(n, dtype=torch.float32, device=comm.device)
    for _ in range(5):
        comm.all_reduce(buf)
    ts = []
    for _ in range(reps):
        if on_gpu:
            torch.cuda.synchronize()
        t = time.perf_counter()
        comm.all_reduce(buf)
        if on_gpu:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return comm.max_scalar(statistics.median(ts)) * 1e6


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001
        return None


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--features", type=int, default=256)
    ap.add_argument("--resident-fraction", type=float, default=None,
                    help="share of free HBM the feature cache may use (default: session conf, 0.85)")
    ap.add_argument("--no-hbm-only", action="store_true", help="skip the resident-rows-only rate")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow N > 1 GPU ranks on a non-RCCL backend (O3S_DIST_BACKEND=gloo, ranks sharing a GPU); "
                         "the JSON is then marked rehearsal and is not a headline")
    a = ap.parse_args(argv)

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _self_launch(a, argv)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.classification import LogisticRegression
    from orange3_spark_amd.synthetic import LineageVectorColumn

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)", file=sys.stderr)
    # one rank = one in-process GPU session (never an executor pool, whatever the node has)
    conf = SessionConf().set("spark.master", "spmd" if world > 1 else "local[1]").setAppName("bench-lr")
    conf.set("spark.executor.instances", str(world))
    s = Session(conf)
    comm = s.comm
    on_gpu = s.device.type == "cuda"
    rows = a.rows if on_gpu else min(a.rows, 200_000)
    rehearsal = comm.world_size > 1 and on_gpu and comm.backend != "nccl"
    if rehearsal and not a.rehearsal:
        # a multi-GPU headline must have run its gradient all-reduce on RCCL over xGMI
        print(f"bench.py: refusing to report n_gpus={comm.world_size} over backend {comm.backend!r} "
              "(RCCL expected; pass --rehearsal for a gloo rehearsal run)", file=sys.stderr)
        return 3

    t0 = time.time()
    df = s.synthetic.classification(rows, a.features, seed=2024, resident_fraction=a.resident_fraction)
    feat = df.column_data("features")
    resident = feat.resident_rows if isinstance(feat, LineageVectorColumn) else len(df)
    lineage = feat.lineage_rows if isinstance(feat, LineageVectorColumn) else 0
    kw = dict(solver="sgd", stepSize=1.0, miniBatchFraction=1.0, regParam=0.0, standardization=True, tol=0.0)
    if a.warmup > 0:
        LogisticRegression(maxIter=a.warmup, **kw).fit(df)
    comm.barrier()
    if on_gpu:
        torch.cuda.synchronize()
    data_s = time.time() - t0

    from orange3_spark_amd.parallel.comm import COMM_STATS
    ar0 = tuple(COMM_STATS.get("all_reduce", (0, 0)))
    t = time.perf_counter()
    model = LogisticRegression(maxIter=a.steps, **kw).fit(df)
    if on_gpu:
        torch.cuda.synchronize()
    comm.barrier()
    elapsed = comm.max_scalar(time.perf_counter() - t)
    ar1 = tuple(COMM_STATS.get("all_reduce", (0, 0)))
    ar_us = _allreduce_us(comm, a.features + 3, on_gpu) if comm.world_size > 1 else None

    hist = model.summary.objectiveHistory
    setup = comm.max_scalar(float(getattr(model, "_fit_setup_seconds", 0.0)))
    hbm_rate = None
    if not a.no_hbm_only and resident > 0:
        hbm_rate = _hbm_only_rate(df, comm, on_gpu)
    tot_resident = comm.sum_scalar(int(resident))
    tot_lineage = comm.sum_scalar(int(lineage))
    value = rows * a.steps / elapsed
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "samples/s",
        "n_gpus": comm.world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (counter-hash generated 1B x 256, random-init weights); rows beyond the HBM "
                "cache budget are regenerated in-kernel each pass",
        "config": {
            "model": "LogisticRegression binomial, solver=sgd (full-batch gradient descent, miniBatchFraction=1), "
                     "standardization=true; timed = whole fit() incl. summarizer pass",
            "global_batch": rows,
            "seq_len": a.features,
            "features": a.features,
            "parallelism": f"dp{comm.world_size}",
            "resident_rows": int(tot_resident),
            "lineage_rows": int(tot_lineage),
            "device": str(s.device) if on_gpu else "cpu",
        },
        # how the rows reach each pass: HBM-resident, plus (N = 1) rows regenerated in-kernel
        # from their lineage; "streamed" (pinned host -> HBM) is tools/bench_streamed.py
        "mode": "resident" if tot_lineage == 0 else "resident+lineage",
        "fit_setup_ms": setup * 1e3,
        "fit_setup_share": setup / elapsed if elapsed > 0 else None,
        "hbm_only_rows_per_s": hbm_rate,
        "data_gen_and_warmup_s": data_s,
        "first_loss": hist[0] if hist else None,
        "final_loss": hist[-1] if hist else None,
        # the collective layer this number was measured on (MULTICHIP self-verification):
        # backend "nccl" is RCCL on ROCm; "local" is one rank with no collective at all
        "backend": comm.backend,
        "collective_world": comm.world_size,
        "rccl_version": _rccl_version() if comm.backend == "nccl" else None,
        "rehearsal": rehearsal,
        # all-reduces issued inside the timed fit (this rank) and their payload, plus the
        # latency of one gradient-sized all-reduce measured after the timed region
        "allreduce_calls_timed": ar1[0] - ar0[0],
        "allreduce_bytes_timed": ar1[1] - ar0[1],
        "allreduce_us_per_call": ar_us,
    }
    if comm.rank == 0:
        print(json.dumps(out), flush=True)
    if comm.world_size > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
