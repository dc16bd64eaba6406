"""bench.py driver contract: one JSON line with the required keys, and the multi-rank
(torchrun, gloo on CPU, world_size 4) run reports the same losses as one rank -- the
row-sharded DP step must not change the optimisation (strong scaling, same data)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _env():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    return env


@pytest.mark.timeout(300)
def test_bench_single_and_four_ranks_agree():
    args = ["--steps", "3", "--warmup", "1", "--rows", "24000", "--features", "32"]
    one = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=_env(), capture_output=True, text=True,
                         timeout=240)
    assert one.returncode == 0, one.stderr[-2000:]
    r1 = _json_line(one.stdout)
    assert KEYS <= set(r1) and r1["n_gpus"] == 1 and r1["steps"] == 3 and r1["warmup"] == 1
    assert r1["higher_is_better"] is True and r1["config"]["global_batch"] == 24000 and r1["value"] > 0
    four = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "4",
                           *args], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert four.returncode == 0, four.stderr[-3000:]
    r4 = _json_line(four.stdout)
    assert r4["n_gpus"] == 4 and r4["config"]["parallelism"] == "dp4" and r4["config"]["global_batch"] == 24000
    # the record names its collective layer: gloo over 4 CPU ranks (RCCL on a GPU node),
    # one gradient all-reduce per iteration inside the timed fit, and its measured latency
    assert r4["backend"] == "gloo" and r4["collective_world"] == 4 and r4["rehearsal"] is False
    assert r4["allreduce_calls_timed"] >= 3 and r4["allreduce_bytes_timed"] > 0 and r4["allreduce_us_per_call"] > 0
    assert r1["backend"] == "local" and r1["allreduce_us_per_call"] is None
    assert abs(r4["first_loss"] - r1["first_loss"]) < 1e-9
    assert abs(r4["final_loss"] - r1["final_loss"]) < 1e-7 * abs(r1["final_loss"])
    assert r1["hbm_only_rows_per_s"] > 0 and 0 <= r1["fit_setup_share"] <= 1


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_bench_refuses_a_gloo_headline():
    """Two GPU ranks on gloo (not RCCL) must not print a headline JSON without --rehearsal."""
    env = dict(os.environ, OMP_NUM_THREADS="4", O3S_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                          "--steps", "1", "--warmup", "0", "--rows", "100000", "--no-hbm-only"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=240)
    assert two.returncode != 0 and "refusing" in two.stderr
    assert not [ln for ln in two.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(300)
def test_bench_self_launches_n_ranks():
    """The plain driver command ``python bench.py --gpus 4`` (no launcher around it)
    starts 4 ranks itself and reports n_gpus 4 with the 1-rank losses."""
    args = ["--steps", "2", "--warmup", "1", "--rows", "16000", "--features", "16", "--no-hbm-only"]
    one = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=_env(), capture_output=True, text=True,
                         timeout=240)
    assert one.returncode == 0, one.stderr[-2000:]
    r1 = _json_line(one.stdout)
    four = subprocess.run([sys.executable, "bench.py", "--gpus", "4", *args], cwd=ROOT, env=_env(),
                          capture_output=True, text=True, timeout=240)
    assert four.returncode == 0, four.stderr[-3000:]
    r4 = _json_line(four.stdout)
    assert r4["n_gpus"] == 4 and r4["config"]["parallelism"] == "dp4"
    assert abs(r4["final_loss"] - r1["final_loss"]) < 1e-7 * abs(r1["final_loss"])


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_bench_two_ranks_match_one_rank():
    """The GPU bench path (mixed resident + lineage kernel, device SGD update, HIP graph at
    one rank / eager at two) on one MI355X: two ranks share cuda:0 over gloo (RCCL needs a
    GPU per rank) and must report the one-rank losses."""
    args = ["--steps", "3", "--warmup", "1", "--rows", "6000000", "--features", "256", "--resident-fraction", "0.002"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    one = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=240)
    assert one.returncode == 0, one.stderr[-2000:]
    r1 = _json_line(one.stdout)
    assert r1["config"]["device"].startswith("cuda") and r1["config"]["lineage_rows"] > 0
    assert r1["config"]["resident_rows"] > 0
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                          *args, "--rehearsal"], cwd=ROOT, env=dict(env, O3S_DIST_BACKEND="gloo"),
                         capture_output=True, text=True, timeout=240)
    assert two.returncode == 0, two.stderr[-3000:]
    r2 = _json_line(two.stdout)
    assert r2["backend"] == "gloo" and r2["rehearsal"] is True and r2["collective_world"] == 2
    assert r1["backend"] == "local" and r1["rehearsal"] is False and r1["collective_world"] == 1
    assert r2["n_gpus"] == 2 and r2["config"]["global_batch"] == 6000000
    assert r2["config"]["resident_rows"] + r2["config"]["lineage_rows"] == 6000000
    assert abs(r2["first_loss"] - r1["first_loss"]) < 1e-6
    assert abs(r2["final_loss"] - r1["final_loss"]) < 1e-5 * abs(r1["final_loss"])
