"""RCCL (backend "nccl") on the real device: a one-rank process group created the way
``parallel/comm.py::init_process_group`` creates it (``device_id`` bound, eager init), then
every collective the estimators issue, on device tensors, through RCCL's own kernels.

A one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks per device), so this
checks the part of the multi-GPU path a single MI355X can run: communicator creation on
this image, RCCL kernels for all_reduce / all_gather_into_tensor / reduce_scatter_tensor /
broadcast / all_to_all_single, the device barrier, and a CUDA-graph-free async handle.
The rank-count logic itself is covered by the gloo tests (tests/test_distributed*.py)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _work(port, q):
    try:
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        os.environ.pop("O3S_DIST_BACKEND", None)
        import torch.distributed as dist
        from orange3_spark_amd.parallel.comm import TorchComm, init_process_group
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        init_process_group(dev, None, 120)
        comm = TorchComm(dev)
        out = {"backend": comm.backend, "cpu_group": comm._cpu_group is not None}
        x = torch.arange(1024, dtype=torch.float64, device=dev)
        dist.all_reduce(x)
        out["all_reduce"] = bool(torch.equal(x, torch.arange(1024, dtype=torch.float64, device=dev)))
        g = torch.empty(1024, dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(g, x)
        out["all_gather"] = bool(torch.equal(g, x))
        r = torch.empty(1024, dtype=torch.float64, device=dev)
        dist.reduce_scatter_tensor(r, x)
        out["reduce_scatter"] = bool(torch.equal(r, x))
        b = torch.full((7,), 3.0, device=dev)
        dist.broadcast(b, 0)
        out["broadcast"] = bool((b == 3).all())
        a2a = torch.empty(1024, dtype=torch.float64, device=dev)
        dist.all_to_all_single(a2a, x, [1024], [1024])
        out["all_to_all"] = bool(torch.equal(a2a, x))
        big = torch.ones(16 << 20, dtype=torch.bfloat16, device=dev)          # 32 MB payload, async handle
        w = dist.all_reduce(big, async_op=True)
        w.wait()
        torch.cuda.synchronize()
        out["async_big"] = bool((big == 1).all())
        dist.barrier(device_ids=[0])
        out["objects"] = comm.all_gather_object({"rank": 0}) == [{"rank": 0}]
        dist.destroy_process_group()
        q.put(out)
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put({"error": repr(e)})


@pytest.mark.timeout(180)
def test_rccl_one_rank_collectives():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_work, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=150)
    p.join(30)
    assert "error" not in out, out
    assert out["backend"] == "nccl"
    for k in ("all_reduce", "all_gather", "reduce_scatter", "broadcast", "all_to_all", "async_big", "objects"):
        assert out[k], (k, out)
    assert p.exitcode == 0
