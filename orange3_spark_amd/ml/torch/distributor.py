"""TorchDistributor: run a PyTorch training function or script on the node's GPUs, one
process per GPU, ``torch.distributed`` over RCCL (``nccl`` backend name on ROCm) / gloo.

Spark's ``pyspark.ml.torch.distributor.TorchDistributor`` (Spark >= 3.4, beyond the
reference's Spark 1.6 surface) launches ``torchrun`` on barrier-mode executors.  Here the
"cluster" is the single MI355X node, so ``run`` launches the processes directly:

* a **function** is serialised with cloudpickle (closures and lambdas work, as in Spark)
  and executed by ``num_processes`` fresh interpreters (``spawn``: no process inherits GPU
  state) with ``MASTER_ADDR=127.0.0.1``, ``MASTER_PORT``, ``RANK``, ``LOCAL_RANK``,
  ``WORLD_SIZE`` set -- the function calls ``torch.distributed.init_process_group`` itself,
  exactly as under ``torchrun``; rank 0's return value is returned;
* a **script path** runs under ``python -m torch.distributed.run --nproc-per-node N
  --master-addr 127.0.0.1`` as a child process (its exit status is checked).

A failing rank raises ``RuntimeError`` carrying that rank's traceback; the other ranks
are terminated.  ``use_gpu=True`` requires ``num_processes`` visible GPUs (counted without
initialising HIP in this process).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import traceback


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(payload: bytes, rank: int, world: int, port: int, use_gpu: bool, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world))
    if not use_gpu:
        os.environ["HIP_VISIBLE_DEVICES"] = ""
    try:
        import cloudpickle
        fn, args, kwargs = cloudpickle.loads(payload)
        out = fn(*args, **kwargs)
        q.put((rank, "ok", cloudpickle.dumps(out) if rank == 0 else None))
    except BaseException:  # noqa: BLE001 - reported to the driver with the traceback
        q.put((rank, "error", traceback.format_exc()))


class TorchDistributor:
    """Distributed PyTorch training on the local MI355X GPUs (or CPU processes with gloo)."""

    def __init__(self, num_processes: int = 1, local_mode: bool = True, use_gpu: bool = True, _ssl_conf=None,
                 timeout: float | None = None):
        """``timeout`` (seconds, None = no deadline): like Spark's barrier-task timeout, a
        run whose ranks have not all reported by then is torn down -- every rank is
        terminated, survivors are killed -- and RuntimeError names the silent ranks."""
        self.timeout = None if timeout is None else float(timeout)
        if int(num_processes) < 1:
            raise ValueError("num_processes must be >= 1")
        if not local_mode:
            raise ValueError("local_mode=False needs a multi-node cluster; this engine drives one node "
                             "(all of its GPUs are local)")
        self.num_processes = int(num_processes)
        self.local_mode = True
        self.use_gpu = bool(use_gpu)
        if self.use_gpu:
            import torch
            n = torch.cuda.device_count()          # does not initialise HIP on this image
            if n < self.num_processes:
                raise RuntimeError(f"use_gpu=True needs {self.num_processes} GPUs, {n} visible")

    # ------------------------------------------------------------------ run
    def run(self, train_object, *args, **kwargs):
        if isinstance(train_object, str):
            return self._run_script(train_object, *args)
        if not callable(train_object):
            raise TypeError("train_object must be a function or a path to a Python script")
        return self._run_function(train_object, *args, **kwargs)

    def _run_function(self, fn, *args, **kwargs):
        import multiprocessing as mp

        import cloudpickle
        payload = cloudpickle.dumps((fn, args, kwargs))
        port = _free_port()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_worker, args=(payload, r, self.num_processes, port, self.use_gpu, q))
                 for r in range(self.num_processes)]
        for p in procs:
            p.start()
        import time
        results, error = {}, None
        deadline = None if self.timeout is None else time.monotonic() + self.timeout
        try:
            while len(results) < len(procs) and error is None:
                if deadline is not None and time.monotonic() > deadline:
                    silent = [r for r in range(len(procs)) if r not in results]
                    error = f"timed out after {self.timeout:g} s; ranks {silent} never reported"
                    break
                wait = 5.0 if deadline is None else max(0.05, min(5.0, deadline - time.monotonic()))
                try:
                    rank, status, data = q.get(timeout=wait)
                except Exception:  # noqa: BLE001 - queue.Empty: check for ranks that died silently
                    dead = [r for r, p in enumerate(procs) if p.exitcode not in (None, 0) and r not in results]
                    if dead:
                        error = f"rank {dead[0]} exited with code {procs[dead[0]].exitcode}"
                    continue
                if status == "error":
                    error = f"rank {rank} failed:\n{data}"
                results[rank] = data
        finally:
            for p in procs:
                if error is not None and p.is_alive():
                    p.terminate()
            for p in procs:
                p.join(10 if error is not None else 60)
                if p.is_alive():                 # ignored SIGTERM / still stuck in a collective
                    p.kill()
                    p.join(10)
        if error is not None:
            raise RuntimeError(f"TorchDistributor: {error}")
        return cloudpickle.loads(results[0])

    def _run_script(self, path: str, *args):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={self.num_processes}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), path, *[str(a) for a in args]]
        env = dict(os.environ)
        if not self.use_gpu:
            env["HIP_VISIBLE_DEVICES"] = ""
        res = subprocess.run(cmd, env=env)
        if res.returncode != 0:
            raise RuntimeError(f"TorchDistributor: {path} exited with code {res.returncode}")
        return None
