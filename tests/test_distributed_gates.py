"""Every BASELINE config's DEFAULT multi-rank path, at world 2 and 4 (gloo, CPU), with
shapes ABOVE the size gates that pick the single-rank / small-problem paths.

The 8-GPU configs (ALS implicit rank 128, GBT depth 8, LR SGD, KMeans) run these exact
code paths on RCCL; no 8-GPU node is available to the build, so these runs are the
evidence that row sharding does not change the answer:

* ALS (implicit and explicit, exact per-row solves -- the Recommendation widget's
  default, orangecontrib/spark/widgets/ml/spark_ml_recommendation.py:15 ->
  base/spark_ml_estimator.py:22): ``nnz_rank * R^2 > 2^26`` on every rank, so fit_als
  takes the CHUNKED slot-layout path (models/als.py ``_slot_pos`` / ``_gather_slots``,
  all-gathers landing in place in the factor tables); a call counter proves it ran;
* GBTClassifier / KMeans (k-means||) / LogisticRegression(solver="sgd").

Each world's result must equal world 1 (ALS factors 1e-6 relative).
"""
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


N_RATINGS, N_USERS, N_ITEMS, RANK = 320_000, 12_000, 1_500, 32


def _ratings(seed=0):
    rng = np.random.default_rng(seed)
    # skewed item popularity: some items have thousands of ratings (dense-kernel rows),
    # most users have a handful (Woodbury rows)
    u = rng.integers(0, N_USERS, N_RATINGS)
    i = np.minimum((rng.pareto(1.2, N_RATINGS) * 40).astype(np.int64), N_ITEMS - 1)
    r = rng.integers(1, 6, N_RATINGS).astype(np.float64)
    r[rng.random(N_RATINGS) < 0.1] *= -1          # a few negative (implicit: b = 0) entries
    return u, i, r


def _work(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(max(1, 8 // max(world, 2)))
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.classification import GBTClassifier, LogisticRegression
    from orange3_spark_amd.ml.clustering import KMeans
    from orange3_spark_amd.ml.recommendation import ALS
    from orange3_spark_amd.models import als as ALSE
    calls = {"gather_slots": 0, "slot_pos": 0}
    real_gs, real_sp = ALSE._gather_slots, ALSE._slot_pos

    def gs(*a, **k):
        calls["gather_slots"] += 1
        return real_gs(*a, **k)

    def sp(*a, **k):
        calls["slot_pos"] += 1
        return real_sp(*a, **k)
    ALSE._gather_slots, ALSE._slot_pos = gs, sp
    conf = SessionConf().set("o3s.device", "cpu").set("spark.master", "spmd" if world > 1 else "local")
    s = Session(conf)
    res = {}
    u, i, r = _ratings()
    pdf = pd.DataFrame({"user": u, "item": i, "rating": r})
    df = s.createDataFrame(pdf)
    for name, implicit in (("als_imp", True), ("als_exp", False)):
        m = ALS(rank=RANK, maxIter=3, regParam=0.05, alpha=2.0, implicitPrefs=implicit, seed=3).fit(df)
        order_u = np.argsort(m._uid_t.numpy())
        order_i = np.argsort(m._iid_t.numpy())
        res[name] = (m._uid_t.numpy()[order_u], m._U.numpy()[order_u], m._iid_t.numpy()[order_i],
                     m._V.numpy()[order_i])
    res["calls"] = dict(calls)
    tdf = s.synthetic.trees(24_000, 10, seed=2)
    g = GBTClassifier(maxIter=4, maxDepth=5, seed=1).fit(tdf)
    res["gbt_loss"] = np.array(g.trainingLossHistory)
    res["gbt_pred"] = np.array([row.prediction for row in g.transform(tdf).select("prediction").collect()])
    km = KMeans(k=24, seed=2, maxIter=8).fit(s.synthetic.blobs(30_000, 16, k=24, seed=1))
    res["km_cost"] = km.summary.trainingCost
    res["km_centers"] = np.stack([np.asarray(c) for c in km.clusterCenters()])
    cdf = s.synthetic.classification(40_001, 24, seed=5)
    sgd = LogisticRegression(solver="sgd", maxIter=15, tol=0.0, miniBatchFraction=0.5, regParam=0.01).fit(cdf)
    res["sgd_coef"] = sgd.coefficients.toArray()
    res["sgd_hist"] = np.array(sgd.summary.objectiveHistory)
    torch.save(res, os.path.join(out_dir, f"w{world}_r{rank}.pt"))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


def _run(world, tmp_path):
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_work, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(900)
        assert p.exitcode == 0, (world, p.exitcode)
    return [torch.load(tmp_path / f"w{world}_r{r}.pt", weights_only=False) for r in range(world)]


def _close_rel(a, b, rel):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max()) <= rel * max(1.0, float(np.abs(a).max()))


@pytest.mark.timeout(1800)
def test_default_multirank_paths_above_size_gates_match_world1(tmp_path):
    from orange3_spark_amd.models.als import gather_chunks
    # the gate of models/als.py (small = max per-rank nnz * R^2 <= 2^26) must be FALSE on
    # every rank at world 4, or this test would not reach the chunked path (the call
    # counters below check that it did)
    assert (N_RATINGS // 4) * RANK * RANK > (1 << 26)
    ref = _run(1, tmp_path)[0]
    assert ref["calls"]["gather_slots"] == 0                 # world 1: no all-gathers
    for world in (2, 4):
        got = _run(world, tmp_path)
        for r, res in enumerate(got):
            # chunked path: initial item gather + per iteration (user + item) -> 1 + 2 * 3 per fit
            assert res["calls"]["gather_slots"] == 2 * (1 + 2 * 3), (world, r, res["calls"])
            assert res["calls"]["slot_pos"] == 2 * 2
        res = got[0]
        for name in ("als_imp", "als_exp"):
            uid0, U0, iid0, V0 = ref[name]
            uid1, U1, iid1, V1 = res[name]
            assert np.array_equal(uid0, uid1) and np.array_equal(iid0, iid1)
            assert _close_rel(U0, U1, 1e-6), (name, world, float(np.abs(U0 - U1).max()))
            assert _close_rel(V0, V1, 1e-6), (name, world, float(np.abs(V0 - V1).max()))
        assert np.allclose(ref["gbt_loss"], res["gbt_loss"], rtol=1e-6)
        assert np.array_equal(ref["gbt_pred"], res["gbt_pred"])
        assert ref["km_cost"] == pytest.approx(res["km_cost"], rel=1e-9)
        assert np.allclose(ref["km_centers"], res["km_centers"], atol=1e-9)
        assert np.allclose(ref["sgd_coef"], res["sgd_coef"], atol=1e-6)
        assert np.allclose(ref["sgd_hist"], res["sgd_hist"], rtol=1e-6)
    # the comm model: 2 chunks for small tables, more as the transfer grows, capped
    assert gather_chunks(12_000, 32, 2) == 2
    assert gather_chunks(50_000_000, 128, 8) == 16 and 2 < gather_chunks(5_000_000, 128, 8) <= 16


def _empty_rank_work(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from orange3_spark_amd.models.als import fit_als, global_ids
    from orange3_spark_amd.parallel.comm import make_comm
    c = make_comm("cpu")
    rng = np.random.default_rng(1)
    u, i, r = rng.integers(0, 900, 1200), rng.integers(0, 60, 1200), rng.normal(size=1200)
    if rank == 1:                                   # an empty partition (e.g. df.limit(n))
        u, i, r = u[:0], i[:0], r[:0]
    ids = global_ids(c, torch.from_numpy(u))
    res = fit_als(c, torch.from_numpy(u), torch.from_numpy(i), torch.from_numpy(r).float(), rank=4, max_iter=2)
    torch.save({"ids": ids, "U": res.U, "V": res.V}, os.path.join(out_dir, f"e{rank}.pt"))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_global_ids_with_an_empty_rank(tmp_path):
    """A rank holding no rows over a dense id range takes the same collective path as the
    others (the bitmap/sort choice used the rank-local count)."""
    mp.spawn(_empty_rank_work, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    a = torch.load(tmp_path / "e0.pt", weights_only=True)
    b = torch.load(tmp_path / "e1.pt", weights_only=True)
    assert torch.equal(a["ids"], b["ids"]) and torch.equal(a["U"], b["U"]) and torch.equal(a["V"], b["V"])
    rng = np.random.default_rng(1)
    assert torch.equal(a["ids"], torch.from_numpy(np.unique(rng.integers(0, 900, 1200))))
