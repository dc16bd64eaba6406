"""Two ranks on ONE MI355X (gloo process group, both on cuda:0): the GPU kernels of the
sharded estimators (GLM gradient, KMeans screen/update, tree histograms + partition,
batched forests, ALS passes) must give the single-rank answer.  RCCL needs one GPU per
rank, so the 8-GPU RCCL run itself is the round driver's; this rehearses every
collective call site of those estimators on device tensors."""
import os
import socket

import numpy as np
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


def _work(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), O3S_DIST_BACKEND="gloo")
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.classification import GBTClassifier, LogisticRegression, RandomForestClassifier
    from orange3_spark_amd.ml.clustering import KMeans
    from orange3_spark_amd.ml.recommendation import ALS
    conf = SessionConf().set("o3s.device", "cuda").set("spark.master", "spmd" if world > 1 else "local")
    s = Session(conf)
    res = {}
    df = s.synthetic.classification(20_001, 16, seed=5)
    res["lr"] = LogisticRegression(maxIter=20, regParam=0.01).fit(df).coefficients.toArray()
    km = KMeans(k=8, seed=2, maxIter=8).fit(s.synthetic.blobs(40_000, 32, k=8, seed=1))
    res["km_cost"] = km.summary.trainingCost
    res["km_centers"] = np.stack([np.asarray(c) for c in km.clusterCenters()])
    tdf = s.synthetic.trees(30_000, 12, seed=2)
    g = GBTClassifier(maxIter=4, maxDepth=4, seed=1).fit(tdf)
    res["gbt_loss"] = np.array(g.trainingLossHistory)
    rf = RandomForestClassifier(numTrees=5, maxDepth=5, seed=3).fit(tdf)
    res["rf_nodes"] = [t.numNodes for t in rf.trees]
    res["rf_imp"] = rf.featureImportances.toArray()
    rng = np.random.default_rng(0)
    pdf = pd.DataFrame({"user": rng.integers(0, 300, 5000), "item": rng.integers(0, 120, 5000),
                        "rating": rng.normal(size=5000)})
    res["als_U"] = ALS(rank=8, maxIter=3, seed=1).fit(s.createDataFrame(pdf))._U.cpu().numpy()
    # opt-in CG path (this shape is below the size gate: the unchunked all_gather_v path)
    from orange3_spark_amd.models import als as ALSE
    from orange3_spark_amd.models.als import fit_als
    lo, hi = (5000 * rank) // world, (5000 * (rank + 1)) // world
    t = torch.tensor(pdf.to_numpy()[lo:hi], device=s.device)
    cg = fit_als(s.comm, t[:, 0].long(), t[:, 1].long(), t[:, 2].float(), rank=32, max_iter=3, implicit=True,
                 alpha=2.0, exact=False, cg_iters=3)
    res["als_cg"] = np.concatenate([cg.U.cpu().numpy().ravel(), cg.V.cpu().numpy().ravel()])
    # the DEFAULT exact solver above the size gate (per-rank nnz * R^2 > 2^26): the chunked
    # slot-layout path -- HIP Woodbury + dense kernels with row_range, writing in place into
    # factor tables that the async all-gathers fill (counted, so the path provably ran)
    calls = [0]
    real = ALSE._gather_slots

    def counted(*a, **k):
        calls[0] += 1
        return real(*a, **k)
    ALSE._gather_slots = counted
    g2 = np.random.default_rng(7)
    nr = 240_000
    uu = g2.integers(0, 20_000, nr)
    ii = np.minimum((g2.pareto(1.2, nr) * 40).astype(np.int64), 2_999)
    rr = g2.integers(1, 6, nr).astype(np.float32)
    lo, hi = (nr * rank) // world, (nr * (rank + 1)) // world
    dev = s.device
    from orange3_spark_amd.parallel.comm import COMM_STATS
    bc0 = COMM_STATS.get("broadcast", [0, 0])[0]
    for implicit in (True, False):
        if not implicit:
            # implicit exact fits keep the tables in the Gram eigenbasis: at world 2 every
            # half-iteration's (eig, Q) comes from rank 0, so both ranks' rows
            # live in one basis -- counted here, the equality below checks the result
            res["eig_broadcasts"] = COMM_STATS.get("broadcast", [0, 0])[0] - bc0
        ex = fit_als(s.comm, torch.from_numpy(uu[lo:hi]).to(dev), torch.from_numpy(ii[lo:hi]).to(dev),
                     torch.from_numpy(rr[lo:hi]).to(dev), rank=32, max_iter=3, reg=0.05, implicit=implicit,
                     alpha=2.0, seed=3)
        res[f"als_exact_{int(implicit)}"] = (ex.U.cpu().numpy(), ex.V.cpu().numpy())
    res["gather_calls"] = calls[0]
    if rank == 0:
        torch.save(res, os.path.join(out_dir, f"g{world}.pt"))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_gpu_world2_matches_world1(tmp_path):
    ctx = mp.get_context("spawn")
    for world in (1, 2):
        port = _free_port()
        procs = [ctx.Process(target=_work, args=(r, world, port, str(tmp_path))) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
    a = torch.load(tmp_path / "g1.pt", weights_only=False)
    b = torch.load(tmp_path / "g2.pt", weights_only=False)
    assert np.allclose(a["lr"], b["lr"], atol=1e-5)
    # per-block fp32 slab partials are summed over different row blocks per shard layout
    assert a["km_cost"] == pytest.approx(b["km_cost"], rel=1e-4)
    assert np.allclose(a["km_centers"], b["km_centers"], atol=1e-3)
    assert np.allclose(a["gbt_loss"], b["gbt_loss"], rtol=1e-5)
    assert a["rf_nodes"] == b["rf_nodes"]
    assert np.allclose(a["rf_imp"], b["rf_imp"], atol=1e-6)
    assert np.allclose(a["als_U"], b["als_U"], atol=1e-3)
    assert np.allclose(a["als_cg"], b["als_cg"], atol=1e-4)
    assert a["gather_calls"] == 0 and b["gather_calls"] == 2 * (1 + 2 * 3)
    assert a["eig_broadcasts"] == 0 and b["eig_broadcasts"] >= 3        # one per user half-iteration
    for imp in (0, 1):
        for x, y in zip(a[f"als_exact_{imp}"], b[f"als_exact_{imp}"]):
            assert x.shape == y.shape
            # fp32 kernels on the same factor rows; only YtY's fp64 partial sums differ by shard
            assert np.abs(x - y).max() <= 1e-4 * max(1.0, np.abs(x).max()), (imp, float(np.abs(x - y).max()))


def _host_tensor_work(rank, world, port, out_dir, strict):
    """Every tensor collective of a GPU session's TorchComm fed HOST tensors: RCCL takes
    device tensors only, so the comm stages them through the device and hands the result
    back on the host (gloo here, which would accept either, runs the same staging code)."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), O3S_DIST_BACKEND="gloo")
    import json
    import torch.distributed as dist
    from orange3_spark_amd.parallel import comm as C
    C.COMM_STRICT = strict
    comm = C.TorchComm(torch.device("cuda:0"))
    res = {}
    if strict:
        try:
            comm.all_reduce(torch.ones(2))
            res["raised"] = False
        except Exception as e:                                   # noqa: BLE001 -- the comm wraps it
            res["raised"] = "host tensor" in str(e)
    else:
        t = torch.full((3,), float(rank + 1))
        comm.all_reduce(t)
        res["all_reduce"] = (t.device.type, t.tolist())
        g = comm.all_gather(torch.tensor([rank]))
        res["all_gather"] = (g.device.type, g.tolist())
        gv = comm.all_gather_v(torch.arange(rank + 1))
        res["all_gather_v"] = (gv.device.type, gv.tolist())
        b = torch.tensor([rank + 5.0])
        comm.broadcast(b, 0)
        res["broadcast"] = (b.device.type, b.tolist())
        rs = comm.reduce_scatter(torch.ones(4) * (rank + 1))
        res["reduce_scatter"] = (rs.device.type, rs.tolist())
        recv, cnt = comm.all_to_all_v(torch.tensor([10 * rank, 10 * rank + 1]), [1, 1])
        res["all_to_all_v"] = (recv.device.type, recv.tolist(), cnt)
        out = torch.empty(2, dtype=torch.int64)
        comm.all_gather_into(out, torch.tensor([rank]))
        res["all_gather_into"] = (out.device.type, out.tolist())
        d = torch.full((2,), float(rank), device="cuda:0")         # device tensors: unchanged path
        comm.all_reduce(d)
        res["device"] = (d.device.type, d.tolist())
    with open(os.path.join(out_dir, f"host{int(strict)}_{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("strict", [False, True])
def test_gpu_collectives_stage_host_tensors(tmp_path, strict):
    import json
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_host_tensor_work, args=(r, 2, port, str(tmp_path), strict)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
        assert p.exitcode == 0
    for r in range(2):
        res = json.load(open(tmp_path / f"host{int(strict)}_{r}.json"))
        if strict:
            assert res["raised"] is True
            continue
        assert res["all_reduce"] == ["cpu", [3.0, 3.0, 3.0]]
        assert res["all_gather"] == ["cpu", [0, 1]]
        assert res["all_gather_v"] == ["cpu", [0, 0, 1]]
        assert res["broadcast"] == ["cpu", [5.0]]
        assert res["reduce_scatter"] == ["cpu", [3.0, 3.0]]
        assert res["all_to_all_v"] == ["cpu", [r, 10 + r], [1, 1]]
        assert res["all_gather_into"] == ["cpu", [0, 1]]
        assert res["device"] == ["cuda", [1.0, 1.0]]
