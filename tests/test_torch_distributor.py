"""TorchDistributor (pyspark.ml.torch): a closure trained over 2 gloo processes returns
rank 0's value; failures carry the rank's traceback; script mode runs under torchrun."""
import pytest

from orange3_spark_amd.ml.torch import TorchDistributor


def test_function_two_processes_allreduce():
    scale = 3.0                                            # captured: cloudpickle ships closures

    def train(n):
        import os

        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        r = int(os.environ["RANK"])
        t = torch.tensor([float(r + 1) * scale] * n)
        dist.all_reduce(t)
        w = int(os.environ["WORLD_SIZE"])
        dist.destroy_process_group()
        return {"sum": t.tolist(), "world": w, "rank": r}

    out = TorchDistributor(num_processes=2, local_mode=True, use_gpu=False).run(train, 4)
    assert out == {"sum": [9.0] * 4, "world": 2, "rank": 0}


def test_failure_reports_rank_traceback():
    def bad():
        import os
        if os.environ["RANK"] == "1":
            raise ValueError("boom on rank 1")
        return 1

    with pytest.raises(RuntimeError, match="boom on rank 1"):
        TorchDistributor(num_processes=2, use_gpu=False).run(bad)


def test_timeout_tears_down_hung_rank():
    """A rank that never reports (sleeping, as if stuck in a collective) hits the deadline:
    every rank is terminated and the error names the silent rank."""
    import time

    def hang():
        import os
        import time as _t
        if os.environ["RANK"] == "1":
            _t.sleep(600)
        return 0

    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match=r"timed out .*ranks \[(0, )?1\]"):
        TorchDistributor(num_processes=2, use_gpu=False, timeout=30).run(hang)
    assert time.monotonic() - t0 < 120


def test_script_mode(tmp_path):
    out = tmp_path / "done"
    script = tmp_path / "train.py"
    script.write_text(
        "import os, sys\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "open(sys.argv[1] + os.environ['RANK'], 'w').write(os.environ['WORLD_SIZE'])\n"
        "dist.destroy_process_group()\n")
    assert TorchDistributor(num_processes=2, use_gpu=False).run(str(script), str(out)) is None
    assert (tmp_path / "done0").read_text() == "2" and (tmp_path / "done1").read_text() == "2"


def test_argument_checks():
    with pytest.raises(ValueError):
        TorchDistributor(num_processes=0, use_gpu=False)
    with pytest.raises(ValueError):
        TorchDistributor(local_mode=False, use_gpu=False)
    with pytest.raises(TypeError):
        TorchDistributor(use_gpu=False).run(42)


@pytest.mark.gpu
def test_gpu_distributor_runs_framework_fit_over_rccl():
    """One process per GPU (the box has one): RCCL process group + this framework's LR fit
    on cuda inside the distributed function."""
    def train():
        import torch
        import torch.distributed as dist
        dist.init_process_group("nccl")
        t = torch.ones(4, device="cuda:0")
        dist.all_reduce(t)
        from orange3_spark_amd import Session
        from orange3_spark_amd.ml.classification import LogisticRegression
        s = Session.getOrCreate()
        m = LogisticRegression(maxIter=5).fit(s.synthetic.classification(100_000, 32, seed=3))
        out = (float(t.sum()), s.device.type, float(m.summary.objectiveHistory[-1]))
        dist.destroy_process_group()
        return out

    total, dev, loss = TorchDistributor(num_processes=1, use_gpu=True).run(train)
    assert total == 4.0 and dev == "cuda" and 0 < loss < 0.7
