"""MEMORY_AND_DISK storage (frame/spill.py): rows of vector columns beyond the HBM budget
live in pinned host memory and stream through the GLM / KMeans passes in double-buffered
chunks.  The fitted model must equal the all-resident fit (reference: ``df.cache()``,
orangecontrib/spark/widgets/data/spark_df_cache.py:39, then ``fit``,
orangecontrib/spark/base/spark_ml_estimator.py:22)."""
import numpy as np
import pandas as pd
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.frame.dataframe import StorageLevel
from orange3_spark_amd.frame.spill import HostStreamer, SpilledVectorColumn
from orange3_spark_amd.ml.classification import LogisticRegression
from orange3_spark_amd.ml.clustering import KMeans
from orange3_spark_amd.ml.feature import VectorAssembler


def _session(device="cpu", budget=None):
    conf = SessionConf().set("o3s.device", device)
    if budget is not None:
        conf.set("o3s.storage.hbmBudget", str(budget))
    return Session(conf)


def _budgeted_frame(budget, **kw):
    """An all-resident assembled frame, then an HBM budget set on its session (persist
    below applies it; assembling UNDER a budget streams straight into spilled rows)."""
    s = _session()
    df = _lr_frame(s, **kw)
    s.conf.set("o3s.storage.hbmBudget", str(budget))
    return df


def _lr_frame(s, n=3000, d=7, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)) * rng.uniform(0.5, 2, size=d)
    y = (X @ rng.normal(size=d) + rng.normal(scale=0.5, size=n) > 0).astype(float)
    pdf = pd.DataFrame(X, columns=[f"f{i}" for i in range(d)])
    pdf["label"] = y
    return VectorAssembler(inputCols=[f"f{i}" for i in range(d)], outputCol="features").transform(
        s.createDataFrame(pdf))


def test_persist_memory_and_disk_spills_beyond_budget():
    df = _budgeted_frame(1000 * 7 * 8).persist(StorageLevel.MEMORY_AND_DISK)   # room for 1000 rows
    col = df.column_data("features")
    assert isinstance(col, SpilledVectorColumn) and len(col) == 3000
    assert col.resident_rows == 1000 and col.spilled_rows == 2000
    assert df.storageLevel == "MEMORY_AND_DISK" and df.count() == 3000
    ref = _lr_frame(_session())
    assert np.allclose(col.to_numpy(), ref.column_data("features").to_numpy())
    # row ops on the spilled column
    assert np.allclose(col.take(torch.tensor([5, 1500, 2999])).to_numpy(),
                       ref.column_data("features").to_numpy()[[5, 1500, 2999]])
    assert df.filter(df.label > 0).count() == ref.filter(ref.label > 0).count()
    assert len(df.limit(10).toPandas()) == 10
    d2 = _budgeted_frame(1 << 40).persist(StorageLevel.DISK_ONLY)
    c2 = d2.column_data("features")
    assert isinstance(c2, SpilledVectorColumn) and c2.resident_rows == 0


def test_spill_when_prefix_does_not_fit_next_to_the_column(monkeypatch):
    """The auto budget counts the column's own bytes as available, so the new resident
    prefix may not fit beside the old column: the prefix is staged through
    host memory and re-allocated after the old column is dropped; with less free memory
    than the budget, the resident part shrinks to what fits instead of raising OOM."""
    from orange3_spark_amd.frame import spill
    free = iter([0, 500 * 7 * 8 + (64 << 20)])           # before / after dropping the column
    monkeypatch.setattr(spill, "device_free_bytes", lambda dev: next(free))
    df = _budgeted_frame(1000 * 7 * 8).persist(StorageLevel.MEMORY_AND_DISK)
    col = df.column_data("features")
    assert isinstance(col, SpilledVectorColumn) and len(col) == 3000
    assert col.resident_rows == 500 and col.spilled_rows == 2500
    ref = _lr_frame(_session())
    assert np.allclose(col.to_numpy(), ref.column_data("features").to_numpy())


def test_host_streamer_covers_every_row_in_order():
    host = torch.arange(1000 * 4, dtype=torch.float32).reshape(1000, 4)
    st = HostStreamer(host, "cpu", chunk_bytes=4 * 4 * 96)
    seen = []
    st.run(lambda X, off: seen.append((off, X.clone())))
    assert [o for o, _ in seen] == list(range(0, 1000, 96))
    assert torch.equal(torch.cat([x for _, x in seen]), host)


@pytest.mark.parametrize("solver", ["l-bfgs", "sgd"])
def test_lr_on_streamed_rows_equals_resident(solver, monkeypatch):
    from orange3_spark_amd.frame import spill
    monkeypatch.setattr(spill, "CHUNK_BYTES", 8 * 8 * 300)   # many chunks
    kw = dict(maxIter=25, regParam=0.01, solver=solver, tol=0.0)
    ref = LogisticRegression(**kw).fit(_lr_frame(_session()))
    df = _budgeted_frame(700 * 7 * 8).persist(StorageLevel.MEMORY_AND_DISK)
    assert df.column_data("features").spilled_rows == 2300
    m = LogisticRegression(**kw).fit(df)
    assert np.allclose(m.coefficients.toArray(), ref.coefficients.toArray(), rtol=1e-9, atol=1e-12)
    assert m.intercept == pytest.approx(ref.intercept, rel=1e-9, abs=1e-12)
    p1 = m.transform(df).select("probability").toPandas()
    assert len(p1) == 3000


def test_kmeans_on_streamed_rows_equals_resident(monkeypatch):
    from orange3_spark_amd.frame import spill
    monkeypatch.setattr(spill, "CHUNK_BYTES", 8 * 8 * 500)
    s0 = _session()
    base = s0.synthetic.blobs(4000, 8, k=6, seed=3, spread=0.5)
    ref = KMeans(k=6, seed=2, maxIter=15).fit(base)
    s1 = _session(budget=900 * 8 * 8)
    df = s1.synthetic.blobs(4000, 8, k=6, seed=3, spread=0.5).select("features").persist(StorageLevel.MEMORY_AND_DISK)
    assert df.column_data("features").spilled_rows > 0
    m = KMeans(k=6, seed=2, maxIter=15).fit(df)
    assert np.allclose(np.array(m.clusterCenters()), np.array(ref.clusterCenters()), rtol=1e-9, atol=1e-9)
    assert m.summary.trainingCost == pytest.approx(ref.summary.trainingCost, rel=1e-9)


@pytest.mark.gpu
def test_gpu_streamed_lr_and_kmeans_match_resident(monkeypatch):
    """Tiny HBM budget on the MI355X: the bf16 GLM pass and the fp32 KMeans pass stream the
    host rows through double-buffered H2D copies; coefficients / centres match the
    all-resident fit."""
    from orange3_spark_amd.frame import spill
    monkeypatch.setattr(spill, "CHUNK_BYTES", 4 << 20)
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.classification(600_000, 64, seed=9, resident_fraction=1.0).cache()
    ref = LogisticRegression(maxIter=20, regParam=0.0).fit(df)
    ref_sgd = LogisticRegression(maxIter=8, solver="sgd", tol=0.0, miniBatchFraction=0.5, seed=3).fit(df)
    s.conf.set("o3s.storage.hbmBudget", str(150_000 * 64 * 2))
    sp = df.select("features", "label").persist(StorageLevel.MEMORY_AND_DISK)
    col = sp.column_data("features")
    assert isinstance(col, SpilledVectorColumn) and col.resident_rows == 150_000 and col.host.is_pinned()
    m = LogisticRegression(maxIter=20, regParam=0.0).fit(sp)
    assert np.allclose(m.coefficients.toArray(), ref.coefficients.toArray(), rtol=2e-4, atol=2e-5)
    m2 = LogisticRegression(maxIter=8, solver="sgd", tol=0.0, miniBatchFraction=0.5, seed=3).fit(sp)
    assert np.allclose(m2.coefficients.toArray(), ref_sgd.coefficients.toArray(), rtol=2e-4, atol=2e-5)
    from orange3_spark_amd.ml.evaluation import BinaryClassificationEvaluator
    a1 = BinaryClassificationEvaluator().evaluate(m.transform(sp))
    a0 = BinaryClassificationEvaluator().evaluate(ref.transform(df))
    assert abs(a1 - a0) < 1e-4
    blobs = s.synthetic.blobs(400_000, 32, k=16, seed=4, spread=0.4)
    kref = KMeans(k=16, seed=1, maxIter=10).fit(blobs)
    s.conf.set("o3s.storage.hbmBudget", str(100_000 * 32 * 4))
    kb = blobs.select("features").persist(StorageLevel.MEMORY_AND_DISK)
    assert kb.column_data("features").spilled_rows == 300_000
    km = KMeans(k=16, seed=1, maxIter=10).fit(kb)
    A, B = np.array(km.clusterCenters()), np.array(kref.clusterCenters())
    # the init's distance kernels differ (split-precision for streamed chunks): compare the
    # centre SETS (each reference centre has a streamed-fit centre within 1e-3)
    dist = np.sqrt(((A[:, None] - B[None]) ** 2).sum(-1))
    assert dist.min(0).max() < 1e-3 and km.summary.trainingCost == pytest.approx(kref.summary.trainingCost, rel=1e-4)


def test_cache_widget_storage_level():
    from orangecontrib.spark_amd.widgets.data.owcache import OWCacheDataFrame
    s = _session(budget=500 * 7 * 8)
    w = OWCacheDataFrame(storageLevel="MEMORY_AND_DISK")
    df = _lr_frame(s)
    w.get_input(df)
    out = w.sent["DataFrame"]
    assert isinstance(out.column_data("features"), SpilledVectorColumn) and out.storageLevel == "MEMORY_AND_DISK"
    w2 = OWCacheDataFrame()
    w2.get_input(_lr_frame(s))
    assert w2.sent["DataFrame"].is_cached and w2.sent["DataFrame"].storageLevel == "MEMORY_ONLY"


def _write_parquet(tmp_path, n=3000, d=7, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)) * rng.uniform(0.5, 2, size=d)
    y = (X @ rng.normal(size=d) + rng.normal(scale=0.5, size=n) > 0).astype(float)
    pdf = pd.DataFrame(X, columns=[f"f{i}" for i in range(d)])
    pdf["label"] = y
    path = str(tmp_path / "t.parquet")
    pdf.to_parquet(path)
    return path, [f"f{i}" for i in range(d)]


def _ooc_fits(s, path, names):
    from orange3_spark_amd.ml.classification import GBTClassifier
    df = VectorAssembler(inputCols=names, outputCol="features").transform(s.read.parquet(path))
    lr = LogisticRegression(maxIter=30, regParam=0.01).fit(df)
    km = KMeans(k=4, seed=2, maxIter=8).fit(df)
    gbt = GBTClassifier(maxIter=3, maxDepth=3, seed=1).fit(df)
    return df, lr.coefficients.toArray(), km.summary.trainingCost, np.array(gbt.trainingLossHistory)


def test_out_of_core_parquet_assembles_into_spilled_rows_and_fits(tmp_path):
    """Out-of-core table (reference spark_table.py:80 + spark_df_cache.py:39):
    with the HBM budget below the table, VectorAssembler streams the rows into a
    SpilledVectorColumn (resident prefix = the budget) and LR, KMeans and GBT (tree
    binning over streamed chunks) give the all-resident results."""
    path, names = _write_parquet(tmp_path)
    s = _session(budget=1000 * 7 * 8)
    df, lr, km, gbt = _ooc_fits(s, path, names)
    col = df.column_data("features")
    assert isinstance(col, SpilledVectorColumn) and col.resident_rows == 1000 and col.spilled_rows == 2000
    ref_df, lr0, km0, gbt0 = _ooc_fits(_session(), path, names)
    assert not isinstance(ref_df.column_data("features"), SpilledVectorColumn)
    assert np.allclose(col.to_numpy(), ref_df.column_data("features").to_numpy())
    assert np.allclose(lr, lr0, atol=1e-7)
    assert km == pytest.approx(km0, rel=1e-9)
    assert np.allclose(gbt, gbt0, rtol=1e-9)


@pytest.mark.gpu
def test_gpu_out_of_core_parquet_ingest_stays_under_budget(tmp_path):
    """GPU: a parquet table 4x the HBM budget is read into pinned host columns (no device
    bytes), assembled chunk by chunk into a SpilledVectorColumn with the device peak under
    the budget plus two chunks, and LR / KMeans / GBT match the all-resident fits."""
    n, d = 400_000, 32
    path, names = _write_parquet(tmp_path, n=n, d=d, seed=3)
    budget = n * 64 * 2 // 4                       # a quarter of the assembled bf16 rows
    s = _session("cuda", budget=budget)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    raw = s.read.parquet(path)
    assert raw.column_data("f0").data.device.type == "cpu"          # zero copy over the Arrow buffer
    df = VectorAssembler(inputCols=names, outputCol="features").transform(raw)
    torch.cuda.synchronize()
    col = df.column_data("features")
    assert isinstance(col, SpilledVectorColumn) and col.spilled_rows > 0
    from orange3_spark_amd.frame.spill import CHUNK_BYTES
    assert torch.cuda.max_memory_allocated() - base <= budget + 3 * CHUNK_BYTES
    from orange3_spark_amd.ml.classification import GBTClassifier
    lr = LogisticRegression(maxIter=20, regParam=0.01).fit(df).coefficients.toArray()
    km = KMeans(k=8, seed=2, maxIter=6).fit(df).summary.trainingCost
    gbt = np.array(GBTClassifier(maxIter=3, maxDepth=4, seed=1).fit(df).trainingLossHistory)
    r = _session("cuda")
    rdf = VectorAssembler(inputCols=names, outputCol="features").transform(r.read.parquet(path))
    assert not isinstance(rdf.column_data("features"), SpilledVectorColumn)
    assert torch.equal(torch.cat([col.data.cpu(), col.host]), rdf.column_data("features").data.cpu())
    assert np.allclose(lr, LogisticRegression(maxIter=20, regParam=0.01).fit(rdf).coefficients.toArray(), atol=1e-5)
    assert km == pytest.approx(KMeans(k=8, seed=2, maxIter=6).fit(rdf).summary.trainingCost, rel=1e-4)
    assert np.allclose(gbt, np.array(GBTClassifier(maxIter=3, maxDepth=4, seed=1).fit(rdf).trainingLossHistory),
                       rtol=1e-5)


def test_scalers_and_union_on_spilled_rows_match_resident(tmp_path):
    """Feature stages and ``union`` on an out-of-core frame (spilled columns
    broke most consumers): StandardScaler / MinMaxScaler / MaxAbsScaler fit block by block
    and transform into a spilled output of the same split; union keeps the first frame's
    resident rows and moves the rest to host memory -- nothing materialises the column."""
    from orange3_spark_amd.ml.feature import MaxAbsScaler, MinMaxScaler, StandardScaler
    path, names = _write_parquet(tmp_path)
    s = _session(budget=1000 * 7 * 8)
    df = VectorAssembler(inputCols=names, outputCol="features").transform(s.read.parquet(path))
    ref = VectorAssembler(inputCols=names, outputCol="features").transform(_session().read.parquet(path))
    assert isinstance(df.column_data("features"), SpilledVectorColumn)

    def boom(self):
        raise AssertionError("materialised a spilled column")
    orig_full = SpilledVectorColumn.full
    SpilledVectorColumn.full = boom
    try:
        outs = []
        for est in (StandardScaler(withMean=True, inputCol="features", outputCol="s"),
                    MinMaxScaler(min=-1.0, max=2.0, inputCol="features", outputCol="s"),
                    MaxAbsScaler(inputCol="features", outputCol="s")):
            m = est.fit(df)
            o = m.transform(df).column_data("s")
            assert isinstance(o, SpilledVectorColumn) and o.resident_rows == 1000 and o.spilled_rows == 2000
            outs.append((m, o))
        u = df.union(df)
        uc = u.column_data("features")
        assert isinstance(uc, SpilledVectorColumn) and uc.resident_rows == 1000 and len(uc) == 6000
    finally:
        SpilledVectorColumn.full = orig_full
    for (m, o), est in zip(outs, (StandardScaler(withMean=True, inputCol="features", outputCol="s"),
                                  MinMaxScaler(min=-1.0, max=2.0, inputCol="features", outputCol="s"),
                                  MaxAbsScaler(inputCol="features", outputCol="s"))):
        r = est.fit(ref).transform(ref).column_data("s").to_numpy()
        assert np.allclose(o.to_numpy(), r, atol=1e-12)
    a = ref.column_data("features").to_numpy()
    assert np.array_equal(uc.to_numpy(), np.concatenate([a, a]))
    assert u.count() == 6000


def _write_parquet_with_nulls(tmp_path, n=3000, d=5, seed=1):
    rng = np.random.default_rng(seed)
    pdf = pd.DataFrame(rng.normal(size=(n, d)), columns=[f"f{i}" for i in range(d)])
    for i in range(d):                        # ~4% of rows get a null somewhere, on both sides of the split
        pdf.loc[rng.random(n) < 0.01, f"f{i}"] = np.nan
    pdf["label"] = (rng.random(n) > 0.5).astype(float)
    path = str(tmp_path / "nulls.parquet")
    pdf.to_parquet(path)
    return path, [f"f{i}" for i in range(d)], pdf


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_out_of_core_assembly_skips_invalid_rows_like_resident(tmp_path, device):
    """handleInvalid="skip" on a table beyond the HBM budget (it raised before,
    so behaviour depended on the table's size): the flagged rows are dropped from every
    column, the output keeps the resident-prefix + host layout, and the rows equal the
    resident run's."""
    path, names, pdf = _write_parquet_with_nulls(tmp_path)
    from orange3_spark_amd.ops.glm import padded_width
    row = padded_width(len(names)) * 2 if device == "cuda" else len(names) * 8
    s = _session(device, budget=1000 * row)
    va = VectorAssembler(inputCols=names, outputCol="features", handleInvalid="skip")
    out = va.transform(s.read.parquet(path))
    col = out.column_data("features")
    assert isinstance(col, SpilledVectorColumn) and col.resident_rows < 1000 and col.spilled_rows > 0
    ref = va.transform(_session(device).read.parquet(path))
    keep = ~pdf[names].isna().any(axis=1).to_numpy()
    assert out.count() == ref.count() == int(keep.sum()) < len(pdf)
    assert np.array_equal(col.to_numpy(), ref.column_data("features").to_numpy())
    assert np.array_equal(out.select("label").toPandas()["label"].to_numpy(), pdf["label"].to_numpy()[keep])


def test_map_blocks_output_prefix_respects_the_budget(tmp_path):
    """a map over an out-of-core column must not allocate a second device
    prefix as large as the input's; with a budget below the input's resident prefix, the
    output's extra rows go to the host part, in row order, with the same values."""
    from orange3_spark_amd.frame.spill import map_blocks
    path, names = _write_parquet(tmp_path)
    s = _session(budget=1000 * 7 * 8)
    col = VectorAssembler(inputCols=names, outputCol="features").transform(s.read.parquet(path)).column_data("features")
    assert isinstance(col, SpilledVectorColumn) and col.resident_rows == 1000
    row_bytes = col.ld * col.data.element_size()
    full = map_blocks(col, lambda x: 2.0 * x + 1.0)
    part = map_blocks(col, lambda x: 2.0 * x + 1.0, chunk_bytes=300 * 8 * col.ld, budget=300 * row_bytes)
    assert full.resident_rows == 1000 and part.resident_rows == 300 and len(part) == len(col) == 3000
    assert part.spilled_rows == 2700
    assert np.array_equal(part.to_numpy(), full.to_numpy())
    assert np.allclose(full.to_numpy(), 2.0 * col.to_numpy() + 1.0)


@pytest.mark.gpu
def test_gpu_scalers_and_union_on_spilled_rows(tmp_path):
    """GPU: StandardScaler fit/transform and union over a host-resident parquet table
    assembled into spilled bf16 rows equal the all-resident results (bf16 storage)."""
    from orange3_spark_amd.ml.feature import StandardScaler
    n, d = 200_000, 16
    path, names = _write_parquet(tmp_path, n=n, d=d, seed=4)
    from orange3_spark_amd.ops.glm import padded_width
    s = _session("cuda", budget=n * padded_width(d) * 2 // 4)     # a quarter of the bf16 rows
    df = VectorAssembler(inputCols=names, outputCol="features").transform(s.read.parquet(path))
    r = _session("cuda")
    rdf = VectorAssembler(inputCols=names, outputCol="features").transform(r.read.parquet(path))
    assert isinstance(df.column_data("features"), SpilledVectorColumn)
    est = StandardScaler(withMean=True, inputCol="features", outputCol="s")
    m, m0 = est.fit(df), est.fit(rdf)
    assert np.allclose(m.mean.toArray(), m0.mean.toArray(), atol=1e-9)
    assert np.allclose(m.std.toArray(), m0.std.toArray(), rtol=1e-9)
    o = m.transform(df).column_data("s")
    assert isinstance(o, SpilledVectorColumn)
    ref = m0.transform(rdf).column_data("s").to_numpy()
    assert np.allclose(o.to_numpy(), ref, atol=2e-2 * np.abs(ref).max())      # bf16 output storage
    u = df.union(df).column_data("features")
    assert isinstance(u, SpilledVectorColumn) and len(u) == 2 * n
    a = rdf.column_data("features").to_numpy()
    assert np.array_equal(u.to_numpy(), np.concatenate([a, a]))
