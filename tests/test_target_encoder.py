"""TargetEncoder (Spark 4.0): encodings == a pandas groupby oracle of Spark's blend formula
enc = w*mean_c + (1-w)*mean_global, w = n_c/(n_c+smoothing); null category, unseen
handling, validation, save/load, world_size-independent fit (gloo, 2 ranks)."""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml.feature import TargetEncoder, TargetEncoderModel


@pytest.fixture(scope="module")
def s():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _pdf(n=400, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 6, n).astype(float)
    a[::17] = np.nan                                    # nulls form their own category
    b = rng.integers(0, 3, n).astype(float)
    y = (rng.random(n) < 0.2 + 0.1 * np.nan_to_num(a, nan=2.0)).astype(float)
    return pd.DataFrame({"a": a, "b": b, "label": y, "cont": rng.normal(size=n) + b})


def _oracle(pdf, col, lab, smoothing):
    g = pdf[lab].mean()
    key = pdf[col].fillna(-1)
    st = pdf.groupby(key)[lab].agg(["count", "mean"])
    w = st["count"] / (st["count"] + smoothing)
    return (w * st["mean"] + (1 - w) * g).to_dict(), g


@pytest.mark.parametrize("tt,lab", [("binary", "label"), ("continuous", "cont")])
@pytest.mark.parametrize("smoothing", [0.0, 5.0])
def test_encodings_match_oracle(s, tt, lab, smoothing):
    pdf = _pdf()
    df = s.createDataFrame(pdf)
    m = TargetEncoder(inputCols=["a", "b"], outputCols=["a_te", "b_te"], labelCol=lab, targetType=tt,
                      smoothing=smoothing).fit(df)
    out = m.transform(df).select("a", "b", "a_te", "b_te").toPandas()
    for c in ("a", "b"):
        enc, g = _oracle(pdf, c, lab, smoothing)
        want = pdf[c].fillna(-1).map(enc).to_numpy()
        assert np.allclose(out[c + "_te"].to_numpy(), want, atol=1e-12)
        got = m.encodings[c]
        assert got[2147483647] == pytest.approx(g)
        assert {k: v for k, v in got.items() if k != 2147483647} == pytest.approx(enc)


def test_unseen_and_invalid(s):
    pdf = _pdf()
    m = TargetEncoder(inputCol="b", outputCol="b_te").fit(s.createDataFrame(pdf))
    new = s.createDataFrame(pd.DataFrame({"b": [0.0, 7.0, np.nan]}))
    with pytest.raises(ValueError, match="Unseen"):
        m.transform(new).collect()
    m.setHandleInvalid("keep")
    got = m.transform(new).select("b_te").toPandas()["b_te"].to_numpy()
    g = pdf["label"].mean()
    assert got[1] == pytest.approx(g) and got[2] == pytest.approx(g)   # no null category in fit -> global
    with pytest.raises(ValueError, match="indices"):
        TargetEncoder(inputCol="x", outputCol="o").fit(s.createDataFrame(pd.DataFrame({"x": [0.5, 1.0],
                                                                                      "label": [0.0, 1.0]})))
    with pytest.raises(ValueError, match="0 or 1"):
        TargetEncoder(inputCol="x", outputCol="o").fit(s.createDataFrame(pd.DataFrame({"x": [0.0, 1.0],
                                                                                      "label": [0.0, 2.0]})))


def test_save_load(s, tmp_path):
    pdf = _pdf()
    df = s.createDataFrame(pdf)
    m = TargetEncoder(inputCols=["a", "b"], outputCols=["a_te", "b_te"], smoothing=2.0).fit(df)
    m.write().overwrite().save(str(tmp_path / "te"))
    m2 = TargetEncoderModel.load(str(tmp_path / "te"))
    assert m2.getOrDefault(m2.smoothing) == 2.0
    a = m.transform(df).select("a_te", "b_te").toPandas().to_numpy()
    b = m2.transform(df).select("a_te", "b_te").toPandas().to_numpy()
    assert np.array_equal(a, b)


def _work(rank, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE="2")
    sess = Session(SessionConf().set("o3s.device", "cpu").set("spark.master", "spmd"))
    m = TargetEncoder(inputCols=["a", "b"], outputCols=["a_te", "b_te"], smoothing=3.0).fit(
        sess.createDataFrame(_pdf()))
    q.put((rank, m.encodings))


def test_world2_matches_world1(s):
    import multiprocessing as mp
    import socket
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_work, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    want = TargetEncoder(inputCols=["a", "b"], outputCols=["a_te", "b_te"], smoothing=3.0).fit(
        s.createDataFrame(_pdf())).encodings
    for r in (0, 1):
        for c in ("a", "b"):
            assert got[r][c] == pytest.approx(want[c], abs=1e-12)


@pytest.mark.gpu
def test_gpu_target_encoder_matches_cpu():
    pdf = _pdf(20000, seed=4)
    res = []
    for dev in ("cpu", "cuda"):
        d = Session(SessionConf().set("o3s.device", dev)).createDataFrame(pdf)
        m = TargetEncoder(inputCols=["a", "b"], outputCols=["a_te", "b_te"], smoothing=4.0).fit(d)
        res.append(m.transform(d).select("a_te", "b_te").toPandas().to_numpy())
    assert np.allclose(res[0], res[1], atol=1e-12)
