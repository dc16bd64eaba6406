"""DataFrame ops, catalog ("Hive") and SQL engine on the CPU path (vs pandas)."""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.frame import functions as Fn


@pytest.fixture()
def s(tmp_path):
    return Session(SessionConf().set("o3s.device", "cpu").set("spark.sql.warehouse.dir", str(tmp_path / "wh")))


def _pdf():
    return pd.DataFrame({"id": [1, 2, 3, 4, 5, 6], "g": ["a", "b", "a", "c", "b", "a"],
                         "x": [1.0, np.nan, 3.0, 4.0, 5.0, 6.0], "y": [10, 20, 30, 40, 50, 60]})


def test_dataframe_basics(s):
    df = s.createDataFrame(_pdf())
    assert df.count() == 6 and df.columns == ["id", "g", "x", "y"]
    assert dict(df.dtypes)["g"] == "string" and dict(df.dtypes)["x"] == "double"
    f = df.fillna(0.0, subset=["x"])
    assert f.toPandas()["x"].tolist() == [1.0, 0.0, 3.0, 4.0, 5.0, 6.0]
    assert df.fillna("zz").toPandas()["g"].tolist() == ["a", "b", "a", "c", "b", "a"]
    w = df.withColumn("z", df["y"] * 2 + 1).filter(Fn.col("z") > 50)
    assert w.toPandas()["z"].tolist() == [61, 81, 101, 121]
    assert df.where("y >= 30 AND g = 'a'").count() == 2
    d = df.select("g").distinct().orderBy("g").toPandas()["g"].tolist()
    assert d == ["a", "b", "c"]
    agg = df.groupBy("g").agg(Fn.sum("y").alias("sy"), Fn.count("*").alias("n")).orderBy("g").toPandas()
    assert agg["sy"].tolist() == [100, 70, 40] and agg["n"].tolist() == [3, 2, 1]
    assert df.limit(2).count() == 2
    s1 = df.sample(False, 0.5, seed=3)
    s2 = df.sample(False, 0.5, seed=3)
    assert s1.toPandas()["id"].tolist() == s2.toPandas()["id"].tolist()
    a, b = df.randomSplit([0.5, 0.5], seed=1)
    assert a.count() + b.count() == 6
    assert df.dropna().count() == 5
    desc = df.describe("y").toPandas()
    assert float(desc[desc.summary == "mean"]["y"].iloc[0]) == 35.0


def test_join(s):
    df = s.createDataFrame(_pdf())
    dim = s.createDataFrame(pd.DataFrame({"g": ["a", "b"], "name": ["AA", "BB"]}))
    j = df.join(dim, "g", "inner").orderBy("id").toPandas()
    assert j["name"].tolist() == ["AA", "BB", "AA", "BB", "AA"]
    lj = df.join(dim, "g", "left").orderBy("id").toPandas()
    assert lj["name"].tolist()[3] is None


def test_catalog_and_sql(s):
    df = s.createDataFrame(_pdf())
    s.sql("CREATE DATABASE IF NOT EXISTS shop")
    df.write.saveAsTable("shop.orders")
    assert "shop" in [r.databaseName for r in s.sql("show databases").collect()]
    assert s.tableNames("shop") == ["orders"]
    t = s.table("shop.orders")
    assert t.count() == 6
    r = s.sql("SELECT g, SUM(y) AS total, COUNT(*) AS n FROM shop.orders WHERE y > 10 GROUP BY g "
              "HAVING COUNT(*) >= 1 ORDER BY total DESC").toPandas()
    assert r["g"].tolist() == ["a", "b", "c"] and r["total"].tolist() == [90, 70, 40]
    df.createOrReplaceTempView("t")
    r2 = s.sql("select id, y * 2 as yy, case when y > 30 then 'hi' else 'lo' end as lvl from t "
               "where g in ('a', 'c') order by id limit 3").toPandas()
    assert r2["yy"].tolist() == [20, 60, 80] and r2["lvl"].tolist() == ["lo", "lo", "hi"]
    r3 = s.sql("SELECT CAST(id AS double) AS d, isnan(x) AS nx FROM t WHERE g LIKE 'b%'").toPandas()
    assert r3["d"].tolist() == [2.0, 5.0] and r3["nx"].tolist() == [True, False]
    assert s.sql("SELECT COUNT(DISTINCT g) AS k FROM t").collect()[0].k == 3
    r4 = s.sql("SELECT t.id, d.name FROM t JOIN dim d ON t.g = d.g ORDER BY t.id") if False else None
    from orange3_spark_amd.utils.data_utils import format_sql
    assert format_sql("select a,b from t where x=1").startswith("SELECT a,")


def test_parquet_and_csv_roundtrip(s, tmp_path):
    df = s.createDataFrame(_pdf())
    df.write.parquet(str(tmp_path / "p"))
    back = s.read.parquet(str(tmp_path / "p")).toPandas()
    assert back["y"].tolist() == _pdf()["y"].tolist()
    assert np.isnan(back["x"].iloc[1])
    df.write.mode("overwrite").csv(str(tmp_path / "c"))
    c = s.read.csv(str(tmp_path / "c"), header=True, inferSchema=True).toPandas()
    assert c["y"].tolist() == _pdf()["y"].tolist()


def test_orange_conversions(s):
    from orange3_spark_amd.utils import data_utils as D
    pdf = pd.DataFrame({"a": np.arange(20, dtype=float), "k": [1, 2] * 10, "s": list("xy" * 10)})
    t = D.pandas_to_orange(pdf)
    names = [v.name for v in t.domain.attributes]
    assert names == ["a", "k"] and type(t.domain.attributes[1]).__name__ == "DiscreteVariable"
    assert [v.name for v in t.domain.metas] == ["s"]
    back = D.orange_to_pandas(t)
    assert back["k"].tolist() == ["1", "2"] * 10 and back["s"].tolist() == list("xy" * 10)
    df = s.createDataFrame(t)
    assert df.count() == 20


def test_sql_resolves_function_library_and_registered_udfs():
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    s = Session(SessionConf().set("o3s.device", "cpu"))
    df = s.createDataFrame(pd.DataFrame({"name": ["Ann", "bob"], "x": [1.25, -2.0]}))
    df.createOrReplaceTempView("udf_t")
    s.udf.register("plus1", lambda v: v + 1, "double")
    rows = s.sql("SELECT upper(name) AS u, substring(name, 1, 2) AS s2, concat(name, '_', name) AS c, "
                 "plus1(x) AS p, round(x, 1) AS r, regexp_replace(name, 'b', 'B') AS rr, "
                 "PLUS1(plus1(x)) AS pp FROM udf_t").collect()
    assert rows[0].u == "ANN" and rows[0].s2 == "An" and rows[0].c == "Ann_Ann"
    assert rows[0].p == 2.25 and rows[1].pp == 0.0
    assert rows[0].r == 1.3 and rows[1].r == -2.0            # HALF_UP like Spark
    assert rows[1].rr == "BoB"
    import pytest
    with pytest.raises(SyntaxError):
        s.sql("SELECT no_such_fn(x) FROM udf_t")


def test_jdbc_and_text_sources(tmp_path):
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    s = Session(SessionConf().set("o3s.device", "cpu"))
    df = s.createDataFrame(pd.DataFrame({"a": [1, 2, 3], "b": ["x", "y", "z"]}))
    url = f"jdbc:sqlite:{tmp_path / 'db.sqlite'}"
    df.write.jdbc(url, "tab", mode="overwrite")
    assert [r.a for r in s.read.jdbc(url, "tab", predicates=["a >= 2"]).collect()] == [2, 3]
    q = s.read.format("jdbc").option("url", url).option("dbtable", "(SELECT a * 10 AS a10 FROM tab) q").load()
    assert [r.a10 for r in q.collect()] == [10, 20, 30]
    df.write.jdbc(url, "tab", mode="append")
    assert s.read.jdbc(url, "tab").count() == 6
    import pytest
    with pytest.raises(ValueError):
        df.write.jdbc(url, "tab")                         # default mode: error if it exists
    df.select("b").write.text(str(tmp_path / "txt"))
    assert [r.value for r in s.read.text(str(tmp_path / "txt")).collect()] == ["x", "y", "z"]
    assert s.read.text(str(tmp_path / "txt"), wholetext=True).count() == 1


def test_catalog_extras(tmp_path):
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    s = Session(SessionConf().set("o3s.device", "cpu").set("spark.sql.warehouse.dir", str(tmp_path / "wh")))
    s.createDataFrame(pd.DataFrame({"a": [1, 2], "b": ["x", "y"]})).write.saveAsTable("t1")
    c = s.catalog
    assert [col.name for col in c.listColumns("t1")] == ["a", "b"]
    c.cacheTable("t1")
    assert c.isCached("t1") and c.table("t1").count() == 2
    c.uncacheTable("t1")
    assert not c.isCached("t1")
    assert c.getTable("t1").database == "default" and c.databaseExists("default")
    assert c.functionExists("regexp_replace") and not c.functionExists("nope")
    s.udf.register("twice", lambda v: 2 * v, "double")
    assert c.functionExists("twice")
    s.createDataFrame(pd.DataFrame({"z": [1.0]})).write.parquet(str(tmp_path / "pq"))
    assert c.createTable("t2", path=str(tmp_path / "pq")).columns == ["z"]


def test_sql_grouping_sets_offset_and_statistical_aggregates():
    import math
    import numpy as np
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    s = Session(SessionConf().set("o3s.device", "cpu"))
    pdf = pd.DataFrame({"a": ["x", "x", "y", "y", "y"], "b": [1, 2, 1, 1, 2], "v": [1.0, 2.0, 3.0, 4.0, 5.0],
                        "w": [2.0, 1.0, 7.0, 3.0, 5.0]})
    s.createDataFrame(pdf).createOrReplaceTempView("gs")
    r = s.sql("SELECT a, b, sum(v) AS sv, grouping_id() AS g FROM gs GROUP BY ROLLUP(a, b)").toPandas()
    assert len(r) == 7 and r[r.g == 3].sv.iloc[0] == 15.0
    c = s.sql("SELECT a, b, count(*) AS n FROM gs GROUP BY a, b WITH CUBE").toPandas()
    assert len(c) == 9
    g = s.sql("SELECT a, b, max(v) AS m FROM gs GROUP BY GROUPING SETS ((a), (b), ())").toPandas()
    assert len(g) == 2 + 2 + 1
    assert g[g.a.isna() & g.b.isna()].m.iloc[0] == 5.0
    assert g[(g.b == 2)].m.iloc[0] == 5.0 and g[g.a == "x"].m.iloc[0] == 2.0
    o = s.sql("SELECT v FROM gs ORDER BY v LIMIT 2 OFFSET 1").toPandas()
    assert o.v.tolist() == [2.0, 3.0]
    st = s.sql("SELECT corr(v, w) AS c, stddev_pop(v) AS sp, skewness(v) AS sk, collect_list(b) AS cl, "
               "percentile_approx(v, 0.5) AS med, first(a) AS fa FROM gs").collect()[0]
    assert math.isclose(st.c, np.corrcoef(pdf.v, pdf.w)[0, 1], rel_tol=1e-9)
    assert math.isclose(st.sp, pdf.v.std(ddof=0), rel_tol=1e-9)
    assert abs(st.sk) < 1e-9 and st.cl == [1, 2, 1, 1, 2] and st.med == 3.0 and st.fa == "x"
