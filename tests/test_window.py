"""Window functions (DataFrame API and SQL OVER) against pandas oracles."""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.sql import Window
from orange3_spark_amd.sql import functions as F


@pytest.fixture(scope="module")
def s():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _pdf(n=300, seed=0):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({"g": rng.choice(["a", "b", "c"], n), "v": rng.integers(0, 15, n).astype(float),
                         "id": np.arange(n)})


def _window_frame(df):
    w = Window.partitionBy("g").orderBy("v", "id")
    wt = Window.partitionBy("g").orderBy("v")                    # ties -> RANGE frame peers
    return df.select(
        "g", "v", "id",
        F.row_number().over(w).alias("rn"), F.rank().over(wt).alias("rk"), F.dense_rank().over(wt).alias("dr"),
        F.percent_rank().over(wt).alias("pr"), F.cume_dist().over(wt).alias("cd"), F.ntile(4).over(w).alias("nt"),
        F.lag("v", 2).over(w).alias("lag2"), F.lead("v", 1, -1.0).over(w).alias("lead1"),
        F.sum("v").over(wt).alias("run_range"), F.sum("v").over(w.rowsBetween(-2, 0)).alias("sum3"),
        F.max("v").over(w.rowsBetween(-3, 1)).alias("mx"), F.min("v").over(w.rowsBetween(Window.unboundedPreceding,
                                                                                         Window.currentRow)).alias("cmin"),
        F.avg("v").over(Window.partitionBy("g")).alias("gavg"), F.count("v").over(w).alias("cnt"))


def test_window_functions_match_pandas(s):
    p = _pdf()
    r = _window_frame(s.createDataFrame(p)).toPandas().sort_values("id").reset_index(drop=True)
    q = p.sort_values(["g", "v", "id"])
    grp = q.groupby("g")
    q = q.assign(rn=grp.cumcount() + 1,
                 rk=grp.v.rank(method="min").astype(int), dr=grp.v.rank(method="dense").astype(int),
                 lag2=grp.v.shift(2), lead1=grp.v.shift(-1).fillna(-1.0),
                 sum3=grp.v.rolling(3, min_periods=1).sum().reset_index(level=0, drop=True),
                 mx=grp.v.apply(lambda x: x[::-1].rolling(2, min_periods=1).max()[::-1]).reset_index(level=0, drop=True),
                 cmin=grp.v.cummin(), gavg=grp.v.transform("mean"), cnt=grp.cumcount() + 1)
    n = grp.v.transform("size")
    q["pr"] = (q.rk - 1) / (n - 1)
    q["cd"] = grp.v.rank(method="max") / n
    q["run_range"] = _range_sum(q)
    q["nt"] = _ntile(q, 4)
    q = q.sort_values("id").reset_index(drop=True)
    for c in ("rn", "rk", "dr", "nt", "cnt"):
        assert r[c].astype(int).tolist() == q[c].astype(int).tolist(), c
    for c in ("pr", "cd", "lead1", "sum3", "cmin", "gavg", "run_range"):
        assert np.allclose(r[c].astype(float), q[c].astype(float)), c
    lag = r["lag2"].astype(float)
    assert np.allclose(lag.fillna(-99), q["lag2"].fillna(-99))
    # max over ROWS BETWEEN 3 PRECEDING AND 1 FOLLOWING
    exp_mx = []
    for _, d in p.sort_values(["g", "v", "id"]).groupby("g"):
        vals = d.v.values
        for i in range(len(vals)):
            exp_mx.append((d.id.values[i], vals[max(0, i - 3): i + 2].max()))
    exp_mx = dict(exp_mx)
    assert np.allclose(r.mx.values, [exp_mx[i] for i in r.id.values])


def _range_sum(q):
    out = []
    for _, d in q.groupby("g", sort=False):
        tot = d.groupby("v").v.sum().cumsum()
        out.append(pd.Series(tot.reindex(d.v).values, index=d.index))
    return pd.concat(out).reindex(q.index)


def _ntile(q, k):
    out = []
    for _, d in q.groupby("g", sort=False):
        n = len(d)
        base, extra = divmod(n, k)
        tiles = []
        for t in range(k):
            tiles += [t + 1] * (base + (1 if t < extra else 0))
        out.append(pd.Series(tiles, index=d.index))
    return pd.concat(out).reindex(q.index)


def test_sql_over_clause(s):
    p = _pdf(60, seed=3)
    s.createDataFrame(p).createOrReplaceTempView("wt")
    r = s.sql("SELECT id, g, ROW_NUMBER() OVER (PARTITION BY g ORDER BY v DESC, id) AS rn, "
              "SUM(v) OVER (PARTITION BY g) AS tot, LAG(v, 1, 0) OVER (PARTITION BY g ORDER BY id) AS prev, "
              "AVG(v) OVER (ORDER BY id ROWS BETWEEN 2 PRECEDING AND CURRENT ROW) AS ma FROM wt ORDER BY id").toPandas()
    assert r.id.tolist() == list(range(60))
    q = p.sort_values(["g", "v", "id"], ascending=[True, False, True])
    q["rn"] = q.groupby("g").cumcount() + 1
    q = q.sort_values("id")
    assert r.rn.tolist() == q.rn.tolist()
    assert np.allclose(r.tot, p.groupby("g").v.transform("sum"))
    assert np.allclose(r.prev.astype(float), p.groupby("g").v.shift(1).fillna(0))
    assert np.allclose(r.ma, p.v.rolling(3, min_periods=1).mean())


def test_window_with_column_and_global_order(s):
    df = s.createDataFrame(pd.DataFrame({"x": [5.0, 1.0, 3.0, 3.0]}))
    out = df.withColumn("r", F.dense_rank().over(Window.orderBy(F.col("x").desc()))).toPandas()
    assert out.x.tolist() == [5.0, 3.0, 3.0, 1.0] and out.r.tolist() == [1, 2, 2, 3]
    assert not any(c.startswith("__win") for c in out.columns)


def _range_oracle(pdf, a, b, desc, fn):
    """Brute-force Spark RangeFrame: rows of the same g whose value lies in [v+a, v+b]
    (DESC: s = -v)."""
    out = []
    for _, r in pdf.iterrows():
        part = pdf[pdf.g == r.g]
        if pd.isna(r.v):
            fr = part[part.v.isna()]
        else:
            s = -part.v if desc else part.v
            si = -r.v if desc else r.v
            fr = part[part.v.notna() & (s >= si + a) & (s <= si + b)]
        vals = fr.v.dropna()
        out.append(None if fn != "count" and vals.empty else
                   {"sum": vals.sum(), "count": len(fr), "max": vals.max() if len(vals) else None,
                    "avg": vals.mean() if len(vals) else None}[fn])
    return out


@pytest.mark.parametrize("a,b,desc", [(-3, 0, False), (-2, 2, False), (1, 4, False), (-2.5, 1.5, False),
                                      (-3, 1, True)])
def test_range_frame_value_offsets(s, a, b, desc):
    rng = np.random.default_rng(3)
    n = 240
    pdf = pd.DataFrame({"g": rng.choice(["a", "b", "c"], n), "v": rng.integers(0, 30, n).astype(float),
                        "id": np.arange(n)})
    df = s.createDataFrame(pdf)
    o = F.col("v").desc() if desc else F.col("v")
    w = Window.partitionBy("g").orderBy(o).rangeBetween(a, b)
    got = df.select("id", F.sum("v").over(w).alias("s"), F.count("*").over(w).alias("c"),
                    F.max("v").over(w).alias("m"), F.avg("v").over(w).alias("av")).toPandas().sort_values("id")
    for col, fn in (("s", "sum"), ("c", "count"), ("m", "max"), ("av", "avg")):
        exp = _range_oracle(pdf, a, b, desc, fn)
        g = got[col].tolist()
        for x, y in zip(g, exp):
            if y is None:
                assert x is None or (isinstance(x, float) and np.isnan(x))
            else:
                assert x == pytest.approx(y)


def test_range_frame_offsets_nulls_and_sql(s):
    rows = [("a", v, i) for i, v in enumerate([1.0, 2.0, None, 4.0, 7.0, None, 8.0])]
    df = s.createDataFrame(rows, ["g", "v", "id"])            # float None -> NaN: sorts last, NaNs are peers
    w = Window.partitionBy("g").orderBy("v").rangeBetween(-3, 0)
    got = df.select("id", F.sum("v").over(w).alias("s"), F.count("*").over(w).alias("c")) \
        .toPandas().sort_values("id")
    # a NaN row's frame = the NaN rows (its peers)
    assert got.s.tolist()[:2] == [1.0, 3.0] and got.s.tolist()[3:5] == [7.0, 11.0] and got.s.tolist()[6] == 15.0
    assert got.c.tolist() == [1, 2, 2, 3, 2, 2, 2]
    w2 = Window.partitionBy("g").orderBy("v").rangeBetween(Window.unboundedPreceding, 1)
    got2 = df.select("id", F.count("*").over(w2).alias("c")).toPandas().sort_values("id")
    assert got2.c.tolist() == [2, 2, 7, 3, 5, 7, 5]      # NaN rows: partition start .. last NaN peer
    df.createOrReplaceTempView("rt")
    q = s.sql("SELECT id, SUM(v) OVER (PARTITION BY g ORDER BY v RANGE BETWEEN 3 PRECEDING AND CURRENT ROW) AS s "
              "FROM rt").toPandas().sort_values("id")
    assert q.s.tolist()[3:5] == [7.0, 11.0]
    with pytest.raises(ValueError):
        df.select(F.sum("v").over(Window.orderBy("v", "id").rangeBetween(-1, 1))).toPandas()


def test_window_moment_and_host_aggregates(s):
    rng = np.random.default_rng(5)
    n = 90
    pdf = pd.DataFrame({"g": rng.choice(["a", "b"], n), "v": rng.integers(0, 9, n).astype(float),
                        "id": np.arange(n)})
    df = s.createDataFrame(pdf)
    w = Window.partitionBy("g").orderBy("id").rowsBetween(-4, 0)
    got = df.select("id", F.var_pop("v").over(w).alias("vp"), F.skewness("v").over(w).alias("sk"),
                    F.kurtosis("v").over(w).alias("ku"), F.collect_set("v").over(w).alias("cs"),
                    F.median("v").over(w).alias("md"), F.product("v").over(w).alias("pr")) \
        .toPandas().sort_values("id").reset_index(drop=True)
    for i, r in pdf.iterrows():
        part = pdf[(pdf.g == r.g) & (pdf.id <= r.id)].tail(5).v.to_numpy()
        mu = part.mean()
        m2 = ((part - mu) ** 2).mean()
        assert got.vp[i] == pytest.approx(m2, abs=1e-9)
        if m2 > 0:
            assert got.sk[i] == pytest.approx(((part - mu) ** 3).mean() / m2 ** 1.5, abs=1e-7)
            assert got.ku[i] == pytest.approx(((part - mu) ** 4).mean() / m2 ** 2 - 3, abs=1e-7)
        assert sorted(got.cs[i]) == sorted(set(part.tolist()))
        assert got.md[i] == pytest.approx(np.median(part))
        assert got.pr[i] == pytest.approx(np.prod(part))


def test_sql_named_window_and_two_column_aggregates(s):
    rows = [("a", 1.0, 0), ("a", 3.0, 1), ("b", 2.0, 2), ("a", 5.0, 3), ("a", 4.0, 7)]
    df = s.createDataFrame(rows, ["g", "v", "id"])
    df.createOrReplaceTempView("nw")
    q = s.sql("SELECT id, SUM(v) OVER w AS f, row_number() OVER w2 AS r FROM nw "
              "WINDOW w AS (PARTITION BY g ORDER BY id), w2 AS (ORDER BY v DESC) ORDER BY id").toPandas()
    assert q.f.tolist() == [1.0, 4.0, 2.0, 9.0, 13.0] and q.r.tolist() == [5, 3, 4, 1, 2]
    q = s.sql("SELECT id, corr(v, id) OVER (PARTITION BY g) AS c, covar_samp(v, id) OVER (PARTITION BY g "
              "ORDER BY id) AS cs, count_if(v > 2) OVER (PARTITION BY g) AS ci, any_value(v) OVER "
              "(PARTITION BY g ORDER BY id) AS av, approx_count_distinct(v) OVER (PARTITION BY g) AS d "
              "FROM nw ORDER BY id").toPandas()
    a = np.array([1.0, 3.0, 5.0, 4.0]), np.array([0.0, 1.0, 3.0, 7.0])
    assert q.c[0] == pytest.approx(np.corrcoef(*a)[0, 1]) and np.isnan(q.c[2])   # one row in g=b
    assert q.cs[1] == pytest.approx(1.0) and q.cs[4] == pytest.approx(np.cov(*a)[0, 1])
    assert q.ci.tolist() == [3, 3, 0, 3, 3] and q.av.tolist() == [1.0, 1.0, 2.0, 1.0, 1.0]
    assert q.d.tolist() == [4, 4, 1, 4, 4]


def _range_and_moments(sess):
    rng = np.random.default_rng(11)
    n = 3000
    pdf = pd.DataFrame({"g": rng.choice(["a", "b", "c"], n), "v": rng.integers(0, 200, n).astype(float),
                        "id": np.arange(n)})
    df = sess.createDataFrame(pdf)
    w = Window.partitionBy("g").orderBy(F.col("v").desc()).rangeBetween(-7, 3)
    w2 = Window.partitionBy("g").orderBy("id").rowsBetween(-20, 5)
    return df.select("id", F.sum("v").over(w).alias("s"), F.max("v").over(w).alias("m"),
                     F.count("*").over(w).alias("c"), F.skewness("v").over(w2).alias("sk"),
                     F.corr("v", "id").over(w2).alias("co")).toPandas().sort_values("id").reset_index(drop=True)


@pytest.mark.gpu
def test_range_frames_and_moments_gpu_match_cpu(s):
    a = _range_and_moments(s)
    b = _range_and_moments(Session(SessionConf().set("o3s.device", "cuda")))
    assert a.c.tolist() == b.c.tolist() and a.m.tolist() == b.m.tolist()
    for k in ("s", "sk", "co"):
        assert np.allclose(a[k].to_numpy(float), b[k].to_numpy(float), rtol=1e-9, atol=1e-9, equal_nan=True), k
