#!/usr/bin/env python
"""Collective micro-benchmark at the payload sizes the estimators issue.

  all_reduce   2 KB      LogisticRegression / LinearSVC gradient (D+3 fp64) -- latency bound
  all_reduce   528 KB    KMeans k=1024 x 129 fp32 sums + counts per Lloyd iteration
  all_reduce   2 MB      GBT depth-8 level histogram (bins 32)
  all_reduce   16 MB     GBT level histogram (bins 256)
  all_gather   2.56 GB   ALS item factors 5M x 128 fp32 gathered every half-iteration
                         (each rank contributes 1/N); once with RCCL's all_gather (rings)
                         and once as the full-mesh grouped isend/irecv (O3S_ALLGATHER=mesh)

``python tools/bench_comm.py --gpus N`` launches N ranks itself (child torch.distributed.run,
like bench.py); under an existing launcher it runs as one rank.  RCCL over xGMI on GPUs,
gloo on CPU (sizes scaled down with --scale).  Prints one JSON line: per op and size the
median time, algorithm bandwidth (payload / time) and ring bus bandwidth
(2 (N-1)/N x payload / time for all_reduce, (N-1)/N x payload / time for all_gather).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

import torch

SIZES = [("all_reduce", 2 << 10, "lr_grad"), ("all_reduce", 528 << 10, "kmeans_sums"),
         ("all_reduce", 2 << 20, "gbt_level_32bins"), ("all_reduce", 16 << 20, "gbt_level_256bins"),
         ("all_gather", 2_560_000_000, "als_item_factors"),
         ("all_gather_mesh", 2_560_000_000, "als_item_factors (peer-to-peer full mesh)")]


def _self_launch(n, argv):
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    return subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--scale", type=float, default=None, help="payload scale (default 1 on GPU, 1/64 on CPU)")
    a = ap.parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _self_launch(a.gpus, argv)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from orange3_spark_amd import Session, SessionConf
    world = int(os.environ.get("WORLD_SIZE", "1"))
    s = Session(SessionConf().set("spark.master", "spmd" if world > 1 else "local").setAppName("bench-comm"))
    comm = s.comm
    dev = s.device
    gpu = dev.type == "cuda"
    scale = a.scale if a.scale is not None else (1.0 if gpu else 1 / 64)
    n = comm.world_size
    res = []
    for op, nbytes, what in SIZES:
        nb = max(1024, int(nbytes * scale)) if op.startswith("all_gather") else max(256, int(nbytes * min(scale * 64, 1.0)))
        elems = nb // 4
        iters = a.iters if nb < (256 << 20) else max(3, a.iters // 5)
        if op == "all_reduce":
            t = torch.ones(elems, dtype=torch.float32, device=dev)
            fn = (lambda t=t: comm.all_reduce(t))
            bus = 2.0 * (n - 1) / n if n > 1 else 0.0
        else:
            shard = max(1, elems // n)
            src = torch.ones(shard, dtype=torch.float32, device=dev)
            out = torch.empty(shard * n, dtype=torch.float32, device=dev)
            if op == "all_gather_mesh" and n > 1:
                fn = (lambda o=out, x=src: comm._all_gather_mesh(o, x, False))
            else:
                fn = (lambda o=out, x=src: comm.all_gather_into(o, x))
            nb = shard * n * 4
            bus = (n - 1) / n if n > 1 else 0.0
        for _ in range(3):
            fn()
        comm.barrier()
        times = []
        for _ in range(iters):
            if gpu:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            if gpu:
                torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        med = comm.max_scalar(statistics.median(times))
        res.append({"op": op, "what": what, "bytes": nb, "median_us": med * 1e6,
                    "algbw_GBps": nb / med / 1e9, "busbw_GBps": bus * nb / med / 1e9})
        del fn
        if gpu:
            torch.cuda.empty_cache()
    if comm.rank == 0:
        print(json.dumps({"n_ranks": n, "backend": comm.backend, "device": str(dev), "results": res}), flush=True)
    if n > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
