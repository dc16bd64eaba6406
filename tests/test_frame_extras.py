"""Rest of the DataFrame surface (sort, dedupe, multiset ops, stat functions, pivot,
unpivot, pandas UDFs) on one rank against pandas, and on two gloo ranks against one."""
import math
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch.multiprocessing as mp

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.sql import functions as F


@pytest.fixture(scope="module")
def s():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _pdf(n=400, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 20, n).astype(float)
    a[rng.uniform(size=n) < 0.05] = np.nan
    return pd.DataFrame({"a": a, "b": rng.choice(["x", "y", "zz", None], n), "c": rng.normal(size=n),
                         "k": rng.integers(0, 5, n)})


def _frame_ops(s):
    """Deterministic results of every operator under test (python values only)."""
    df = s.createDataFrame(_pdf())
    o = s.createDataFrame(_pdf(300, seed=1))
    r = {}
    r["sort"] = [tuple(x) for x in df.orderBy("k", F.col("b").desc(), "c").select("k", "b", "c").collect()]
    r["sort_nulls"] = [x.a for x in df.orderBy(F.col("a").asc_nulls_last()).select("a").collect()]
    r["dedupe"] = [tuple(x) for x in df.dropDuplicates(["k", "b"]).select("k", "b").collect()]
    r["distinct_n"] = df.select("a", "b").distinct().count()
    two = df.select("k", "b")
    other = o.select("k", "b")
    r["intersect"] = sorted(tuple(map(str, x)) for x in two.intersect(other).collect())
    r["except_all_n"] = two.exceptAll(other).count()
    r["intersect_all_n"] = two.intersectAll(other).count()
    r["subtract_n"] = two.subtract(other).count()
    r["quant"] = df.approxQuantile("c", [0.0, 0.1, 0.5, 0.9, 1.0], 0.0)
    r["corr"] = df.corr("c", "k")
    r["cov"] = df.cov("c", "k")
    r["pivot"] = [tuple(map(str, x)) for x in df.groupBy("k").pivot("b", ["x", "y"]).count().orderBy("k").collect()]
    r["rep"] = sorted(tuple(map(str, x)) for x in df.repartition("k").select("k", "b", "c").collect())
    r["rebalance_n"] = df.filter(F.col("k") == 1).repartition().count()
    r["crosstab"] = [tuple(map(str, x)) for x in df.crosstab("k", "b").collect()]
    r["apply"] = sorted(tuple(x) for x in df.groupBy("k").applyInPandas(
        lambda g: pd.DataFrame({"k": [g.k.iloc[0]], "n": [len(g)]}), "k long, n long").collect())
    r["apply_key"] = sorted(tuple(x) for x in df.groupBy("k").applyInPandas(
        lambda key, g: pd.DataFrame({"k": [key[0]], "n": [len(g)]}), "k long, n long").collect())
    # cogroup: per key the row counts of both sides (keys 0..4 on the left, 2..6 on the right)
    o2 = s.createDataFrame(_pdf(300, seed=1).assign(k=lambda d: d.k + 2))
    r["cogroup"] = sorted(tuple(x) for x in df.groupBy("k").cogroup(o2.groupBy("k")).applyInPandas(
        lambda key, a, b: pd.DataFrame({"k": [key[0]], "na": [len(a)], "nb": [len(b)]}),
        "k long, na long, nb long").collect())
    from orange3_spark_amd.sql import Window
    w = Window.partitionBy("k").orderBy("c")
    r["window"] = sorted((int(x.k), round(x.c, 12), int(x.rn), float(x.run)) for x in df.select(
        "k", "c", F.row_number().over(w).alias("rn"), F.sum("c").over(w).alias("run")).collect())
    r["window_global"] = [int(x.rn) for x in df.select(
        F.rank().over(Window.orderBy("a")).alias("rn")).collect()]
    return r


def test_frame_ops_match_pandas(s):
    r = _frame_ops(s)
    p = _pdf()
    assert r["apply_key"] == r["apply"] == sorted((int(k), int(n)) for k, n in p.k.value_counts().items())
    o2 = _pdf(300, seed=1).k + 2
    ca, cb = p.k.value_counts(), o2.value_counts()
    assert r["cogroup"] == [(k, int(ca.get(k, 0)), int(cb.get(k, 0))) for k in range(7)]
    exp = p.assign(bb=p.b.fillna("￿")).sort_values(["k", "bb", "c"], ascending=[True, False, True],
                                                         kind="stable")
    # Spark: descending puts nulls last -> None after all strings
    exp_rows = [(k, (None if b == "￿" else b), c) for k, b, c in zip(exp.k, exp.bb, exp.c)]
    got = r["sort"]
    assert [g[0] for g in got] == [e[0] for e in exp_rows]
    for (k1, b1, c1), (k2, b2, c2) in zip(got, got[1:]):
        if k1 == k2:
            assert (b2 is None) or (b1 is not None and b1 >= b2)
            if b1 == b2:
                assert c1 <= c2
    sn = r["sort_nulls"]
    nn = [v for v in sn if not (v is None or (isinstance(v, float) and math.isnan(v)))]
    assert nn == sorted(nn) and all(v is None or math.isnan(v) for v in sn[len(nn):])
    first = p.drop_duplicates(["k", "b"])
    assert r["dedupe"] == [(k, b) for k, b in zip(first.k, first.b)]
    assert r["distinct_n"] == len(p[["a", "b"]].astype(str).drop_duplicates())
    q = np.sort(p.c.values)
    n = len(q)
    assert r["quant"] == [q[int(math.floor(pr * (n - 1)))] for pr in (0.0, 0.1, 0.5, 0.9, 1.0)]
    assert r["corr"] == pytest.approx(np.corrcoef(p.c, p.k)[0, 1], rel=1e-10)
    assert r["cov"] == pytest.approx(np.cov(p.c, p.k)[0, 1], rel=1e-10)
    o = _pdf(300, seed=1)
    key = lambda d: list(zip(d.k, d.b.fillna("<null>")))  # noqa: E731
    from collections import Counter
    ca, cb = Counter(key(p)), Counter(key(o))
    assert r["except_all_n"] == sum((ca - cb).values())
    assert r["intersect_all_n"] == sum((ca & cb).values())
    assert r["subtract_n"] == len(set(ca) - set(cb))
    assert len(r["intersect"]) == len(set(ca) & set(cb))
    pv = p.groupby("k").b.value_counts().unstack()
    for row in r["pivot"]:
        k = int(float(row[0]))
        for j, v in enumerate(("x", "y")):
            e = pv.loc[k].get(v)
            assert (row[1 + j] == "None") if (e is None or np.isnan(e)) else int(float(row[1 + j])) == int(e)
    assert r["rebalance_n"] == int((p.k == 1).sum())
    assert r["apply"] == sorted((int(k), int(v)) for k, v in p.k.value_counts().items())


def test_replace_unpivot_tail_json(s):
    df = s.createDataFrame(pd.DataFrame({"a": [1.0, 2.0, 3.0], "b": ["x", "y", "x"], "c": [4.0, 5.0, 6.0]}))
    assert df.replace("x", "X").toPandas().b.tolist() == ["X", "y", "X"]
    assert df.replace({1.0: 10.0, 3.0: None}, subset=["a"]).toPandas().a.tolist()[:2] == [10.0, 2.0]
    assert df.na.replace(["x", "y"], ["p", "q"], "b").toPandas().b.tolist() == ["p", "q", "p"]
    u = df.unpivot("b", ["a", "c"], "var", "val").toPandas()
    assert u["var"].tolist() == ["a", "c"] * 3 and u.val.tolist() == [1.0, 4.0, 2.0, 5.0, 3.0, 6.0]
    assert [r.a for r in df.tail(2)] == [2.0, 3.0]
    assert df.toJSON()[0] == '{"a": 1.0, "b": "x", "c": 4.0}'
    assert df.toDF("p", "q", "r").columns == ["p", "q", "r"] and not df.isEmpty() and df.isLocal()
    assert df.transform(lambda d, k: d.limit(k), 1).count() == 1
    assert df.freqItems(["b"], 0.5).collect()[0].b_freqItems == ["x"]
    sb = df.sampleBy("b", {"x": 1.0, "y": 0.0}, seed=1).toPandas()
    assert sb.b.tolist() == ["x", "x"]
    assert df.sortWithinPartitions(F.col("a").desc()).toPandas().a.tolist() == [3.0, 2.0, 1.0]
    assert "Physical Layout" in df.explain()
    out = df.mapInPandas(lambda it: (p.assign(d=p.a * 2) for p in it), "a double, b string, c double, d double")
    assert out.toPandas().d.tolist() == [2.0, 4.0, 6.0]


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


def _work(rank, world, port, out):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import json
    conf = SessionConf().set("o3s.device", "cpu").set("spark.master", "spmd" if world > 1 else "local")
    r = _frame_ops(Session(conf))
    if rank == 0:
        with open(out, "w") as f:
            json.dump(r, f, default=str)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_frame_ops_world2_match_world1(tmp_path):
    import json
    _work(0, 1, _free_port(), str(tmp_path / "w1.json"))
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_work, args=(r, 2, port, str(tmp_path / "w2.json"))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    a = json.load(open(tmp_path / "w1.json"))
    b = json.load(open(tmp_path / "w2.json"))
    for k in a:
        if isinstance(a[k], float):                    # partial sums combine in a different order
            assert a[k] == pytest.approx(b[k], rel=1e-12), k
        elif k == "window":
            assert [t[:3] for t in a[k]] == [t[:3] for t in b[k]]
            assert np.allclose([t[3] for t in a[k]], [t[3] for t in b[k]], rtol=1e-12)
        else:
            assert a[k] == b[k], k


@pytest.mark.gpu
def test_frame_ops_gpu_match_cpu(s):
    a = _frame_ops(s)
    b = _frame_ops(Session(SessionConf().set("o3s.device", "cuda")))
    for k in a:
        if isinstance(a[k], float):
            assert a[k] == pytest.approx(b[k], rel=1e-9), k
        elif k == "quant":
            assert np.allclose(a[k], b[k], rtol=1e-12), k
        elif k == "window":                            # device scans sum in another order
            assert [t[:3] for t in a[k]] == [t[:3] for t in b[k]]
            assert np.allclose([t[3] for t in a[k]], [t[3] for t in b[k]], rtol=1e-12)
        else:
            assert repr(a[k]) == repr(b[k]), k            # NaN-aware


def test_rollup_cube_grouping_id_and_misc_surface(tmp_path):
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.sql import functions as F, Observation
    s = Session(SessionConf().set("o3s.device", "cpu"))
    pdf = pd.DataFrame({"a": ["x", "x", "y", "y", "y"], "b": [1, 2, 1, 1, 2], "v": [1.0, 2.0, 3.0, 4.0, 5.0]})
    df = s.createDataFrame(pdf)
    r = df.rollup("a", "b").agg(F.sum("v").alias("sv"), F.grouping_id().alias("g")).toPandas()
    assert len(r) == 4 + 2 + 1
    tot = r[r.g == 3]
    assert len(tot) == 1 and tot.sv.iloc[0] == 15.0 and tot.a.iloc[0] is None
    sub = r[r.g == 1].set_index("a").sv.to_dict()
    assert sub == {"x": 3.0, "y": 12.0}
    c = df.cube("a", "b").agg(F.count("v").alias("n"), F.grouping("a").alias("ga")).toPandas()
    assert len(c) == 4 + 2 + 2 + 1
    byb = c[(c.ga == 1) & c.b.notna()].set_index("b").n.to_dict()
    assert byb == {1: 3, 2: 2}
    # pandas reference for the full rollup
    ref = pdf.groupby(["a", "b"]).v.sum().to_dict()
    got = {(a, int(b)): v for a, b, v, g in zip(r.a, r.b, r.sv, r.g) if g == 0}
    assert got == ref
    # colRegex, offset, observe, to(schema), global temp views, writeTo, inputFiles
    assert df.select(df.colRegex("`[ab]`")).columns == ["a", "b"]
    assert [x.v for x in df.offset(3).collect()] == [4.0, 5.0]
    ob = Observation("m")
    assert df.observe(ob, F.max("v").alias("mx"), F.count("v").alias("n")) is df
    assert ob.get == {"mx": 5.0, "n": 5}
    t = df.to("v double, b bigint")
    assert t.columns == ["v", "b"] and t.dtypes[1][1] in ("bigint", "long")
    df.createOrReplaceGlobalTempView("gv")
    assert s.table("global_temp.gv").count() == 5
    assert s.catalog.dropGlobalTempView("gv")
    s.conf.set("o3s.warehouse", str(tmp_path / "wh")) if hasattr(s.conf, "set") else None
    df.write.parquet(str(tmp_path / "p"))
    rd = s.read.parquet(str(tmp_path / "p"))
    assert rd.inputFiles() and all(f.endswith(".parquet") for f in rd.inputFiles())
    rs = s.read.schema("x string, y long, z double").parquet(str(tmp_path / "p"))
    assert rs.columns == ["x", "y", "z"]
    assert df.sparkSession is s and not df.isStreaming and df.sameSemantics(df)
    assert df.withWatermark("b", "1 minute") is df
    import pyarrow as pa
    m = df.mapInArrow(lambda it: (pa.RecordBatch.from_pydict({"w": [x * 2 for x in b.column("v").to_pylist()]})
                                  for b in it), "w double")
    assert [r_.w for r_ in m.collect()] == [2.0, 4.0, 6.0, 8.0, 10.0]


def test_pivot_on_grouping_column():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    df = s.createDataFrame(pd.DataFrame({"k": [1, 2, 1, 3], "x": [1.0, 2.0, 3.0, 4.0]}))
    r = df.groupBy("k").pivot("k").sum("x").orderBy("k").toPandas()
    assert list(r.columns) == ["k", "1", "2", "3"]
    assert r["1"].tolist()[0] == 4.0 and r["2"].tolist()[1] == 2.0 and r["3"].tolist()[2] == 4.0
    assert r["1"].isna().tolist() == [False, True, True]
