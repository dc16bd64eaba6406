"""Multi-process (gloo, world_size=2) runs of the distributed code paths; results must
match the single-process run (row sharding must not change the answer)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _work(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.classification import GBTClassifier, LogisticRegression
    from orange3_spark_amd.ml.clustering import KMeans
    from orange3_spark_amd.ml.evaluation import BinaryClassificationEvaluator, MulticlassClassificationEvaluator
    from orange3_spark_amd.ml.recommendation import ALS
    conf = SessionConf().set("o3s.device", "cpu").set("spark.master", "spmd" if world > 1 else "local")
    s = Session(conf)
    res = {}
    df = s.synthetic.classification(3001, 12, seed=5)
    res["count"] = df.count()
    m = LogisticRegression(maxIter=30, regParam=0.01).fit(df)
    res["lr_coef"] = m.coefficients.toArray()
    out = m.transform(df)
    res["auc"] = BinaryClassificationEvaluator().evaluate(out)
    res["acc"] = MulticlassClassificationEvaluator(metricName="accuracy").evaluate(out)
    km = KMeans(k=4, seed=2, maxIter=10).fit(s.synthetic.blobs(2000, 5, k=4, seed=1))
    res["km_cost"] = km.summary.trainingCost
    res["sample_n"] = df.sample(False, 0.3, seed=9).count()
    g = GBTClassifier(maxIter=3, maxDepth=3, seed=1).fit(s.synthetic.trees(2000, 6, seed=2))
    res["gbt_loss"] = g.trainingLossHistory
    from orange3_spark_amd.ml.classification import RandomForestClassifier
    rf = RandomForestClassifier(numTrees=4, maxDepth=4, seed=3).fit(s.synthetic.trees(2000, 6, seed=2))
    res["rf_nodes"] = [t.numNodes for t in rf.trees]
    res["rf_imp"] = rf.featureImportances.toArray()
    rng = np.random.default_rng(0)
    u = rng.integers(0, 50, 600)
    i = rng.integers(0, 30, 600)
    r = rng.normal(size=600)
    rows = np.stack([u, i, r], 1)
    lo, hi = (600 * rank) // world, (600 * (rank + 1)) // world
    pdf = pd.DataFrame({"user": u, "item": i, "rating": r})
    als = ALS(rank=3, maxIter=3, seed=1).fit(s.createDataFrame(pdf))
    res["als_U"] = als._U.numpy()
    from orange3_spark_amd.models.als import fit_als     # opt-in CG path (below the size gate: unchunked;
    # the chunked slot-layout path is covered by tests/test_distributed_gates.py)
    t = torch.from_numpy(rows[lo:hi])
    cg = fit_als(s.comm, t[:, 0].long(), t[:, 1].long(), t[:, 2].float(), rank=4, max_iter=3, implicit=True,
                 alpha=2.0, exact=False, cg_iters=3)
    res["als_cg"] = np.concatenate([cg.U.numpy().ravel(), cg.V.numpy().ravel()])
    from orange3_spark_amd.ml.classification import NaiveBayes
    from orange3_spark_amd.ml.feature import VectorAssembler
    from orange3_spark_amd.ml.regression import GeneralizedLinearRegression, IsotonicRegression
    xi = np.round(rng.uniform(0, 10, 400), 1)
    yi = xi + rng.normal(0, 1, 400)
    dfi = VectorAssembler(inputCols=["x"], outputCol="features").transform(
        s.createDataFrame(pd.DataFrame({"x": xi, "label": yi})))
    iso = IsotonicRegression().fit(dfi)
    res["iso"] = np.concatenate([iso.boundaries.toArray(), iso.predictions.toArray()])
    res["nb_theta"] = NaiveBayes(modelType="gaussian").fit(df).theta.toArray()
    res["glr"] = GeneralizedLinearRegression(family="binomial").fit(df).coefficients.toArray()
    from orange3_spark_amd.ml.clustering import BisectingKMeans, GaussianMixture
    blobs = s.synthetic.blobs(1200, 4, k=3, seed=4)
    res["bkm_cost"] = BisectingKMeans(k=3, seed=1).fit(blobs).summary.trainingCost
    res["gmm_ll"] = GaussianMixture(k=3, seed=1, maxIter=20).fit(blobs).summary.logLikelihood
    res["groupby"] = sorted((row.g, row.n) for row in s.createDataFrame(
        pd.DataFrame({"g": list("abcab" * 20)})).groupBy("g").count().withColumnRenamed("count", "n").collect())
    if rank == 0:
        torch.save(res, os.path.join(out_dir, f"w{world}.pt"))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    del rows, lo, hi


@pytest.mark.timeout(600)
def test_world2_matches_world1(tmp_path):
    _work(0, 1, _free_port(), str(tmp_path))
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_work, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
        assert p.exitcode == 0
    a = torch.load(tmp_path / "w1.pt", weights_only=False)
    b = torch.load(tmp_path / "w2.pt", weights_only=False)
    assert a["count"] == b["count"] == 3001
    assert np.allclose(a["lr_coef"], b["lr_coef"], atol=1e-6)
    assert abs(a["auc"] - b["auc"]) < 1e-9 and abs(a["acc"] - b["acc"]) < 1e-9
    assert a["km_cost"] == pytest.approx(b["km_cost"], rel=1e-9)
    assert a["sample_n"] == b["sample_n"]
    assert np.allclose(a["gbt_loss"], b["gbt_loss"], rtol=1e-6)
    assert a["rf_nodes"] == b["rf_nodes"] and np.allclose(a["rf_imp"], b["rf_imp"], atol=1e-9)
    assert np.allclose(a["als_U"], b["als_U"], atol=1e-4)
    assert np.allclose(a["als_cg"], b["als_cg"], atol=1e-5)
    assert a["groupby"] == b["groupby"]
    assert a["iso"].shape == b["iso"].shape and np.allclose(a["iso"], b["iso"], atol=1e-9)
    assert np.allclose(a["nb_theta"], b["nb_theta"], atol=1e-9)
    assert np.allclose(a["glr"], b["glr"], atol=1e-8)
    assert a["bkm_cost"] == pytest.approx(b["bkm_cost"], rel=1e-9)
    assert a["gmm_ll"] == pytest.approx(b["gmm_ll"], rel=1e-9)


def _mesh_work(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.parallel import comm as CM
    s = Session(SessionConf().set("o3s.device", "cpu").set("spark.master", "spmd"))
    c = s.comm
    t = torch.arange(5 * 3, dtype=torch.float32).reshape(5, 3) + 100 * rank
    ring = torch.empty((5 * world, 3))
    c.all_gather_into(ring, t)
    CM.ALLGATHER_ALGO = "mesh"
    mesh = torch.full((5 * world, 3), -1.0)
    w = c.all_gather_into(mesh, t, async_op=True)
    w.wait()
    mesh2 = torch.full((5 * world, 3), -1.0)
    c.all_gather_into(mesh2, t)
    ok = torch.equal(ring, mesh) and torch.equal(ring, mesh2)
    # the ALS chunked factor gathers go through the same entry point
    from orange3_spark_amd.models.als import fit_als
    rng = np.random.default_rng(0)
    u, i, r = rng.integers(0, 40, 500), rng.integers(0, 25, 500), rng.normal(size=500)
    lo, hi = (500 * rank) // world, (500 * (rank + 1)) // world
    res = fit_als(c, torch.from_numpy(u[lo:hi]), torch.from_numpy(i[lo:hi]), torch.from_numpy(r[lo:hi]).float(),
                  rank=4, max_iter=3, implicit=True, alpha=2.0, exact=False, cg_iters=3)
    CM.ALLGATHER_ALGO = "ring"
    ref = fit_als(c, torch.from_numpy(u[lo:hi]), torch.from_numpy(i[lo:hi]), torch.from_numpy(r[lo:hi]).float(),
                  rank=4, max_iter=3, implicit=True, alpha=2.0, exact=False, cg_iters=3)
    ok = ok and torch.equal(res.U, ref.U) and torch.equal(res.V, ref.V)
    torch.save({"ok": ok, "ring": ring}, os.path.join(out_dir, f"mesh{rank}.pt"))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_mesh_all_gather_matches_ring(tmp_path):
    """The full-mesh all-gather (grouped isend/irecv to every peer) fills the output
    exactly like all_gather_into_tensor, sync and async, and the ALS factor gathers
    give bit-identical factors under either algorithm (gloo, 3 ranks)."""
    world = 3
    mp.spawn(_mesh_work, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        got = torch.load(tmp_path / f"mesh{r}.pt", weights_only=True)
        assert got["ok"], r
        assert torch.equal(got["ring"][5:10], torch.arange(15, dtype=torch.float32).reshape(5, 3) + 100)
