"""pyspark.sql.functions surface, explode, new aggregates (CPU)."""
import math

import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.sql import functions as F


@pytest.fixture(scope="module")
def s():
    return Session(SessionConf().set("o3s.device", "cpu"))


@pytest.fixture(scope="module")
def df(s):
    return s.createDataFrame(pd.DataFrame({
        "name": ["  Alice ", "bob", "Carol", None], "x": [1.5, -2.25, 3.0, 4.0], "k": [1, 2, 1, 2],
        "d": ["2024-01-31", "2024-02-29", "2023-12-25", None], "tags": ["a,b", "c", "", "d,e,f"]}))


def test_string_functions(df):
    r = df.select(F.upper(F.trim("name")).alias("u"), F.length("name").alias("n"),
                  F.substring("name", 3, 2).alias("sub"), F.concat_ws("-", "name", "k").alias("cw"),
                  F.regexp_replace("name", "[aeiou]", "_").alias("rr"),
                  F.regexp_extract("d", r"(\d+)-(\d+)", 2).alias("re")).toPandas()
    assert r.u.tolist() == ["ALICE", "BOB", "CAROL", None]
    assert r.n.tolist()[:3] == [8, 3, 5] and (r.n.isna().iloc[3] or r.n.iloc[3] is None)
    assert r["sub"].tolist()[1:3] == ["b", "ro"]
    assert r.cw.tolist() == ["  Alice -1", "bob-2", "Carol-1", "2"]
    assert r.rr.tolist()[1] == "b_b"
    assert r["re"].tolist()[:3] == ["01", "02", "12"]


def test_math_and_null_functions(df):
    r = df.select(F.round("x", 1).alias("r"), F.bround(F.lit(2.5)).alias("b"), F.floor("x").alias("f"),
                  F.pow("x", 2).alias("p"), F.greatest("x", "k").alias("g"), F.isnull("name").alias("nn"),
                  F.signum("x").alias("sg")).toPandas()
    assert r.r.tolist() == [1.5, -2.3, 3.0, 4.0]            # HALF_UP away from zero
    assert r.b.tolist()[0] == 2.0                             # HALF_EVEN
    assert r.f.tolist() == [1.0, -3.0, 3.0, 4.0]
    assert r.p.tolist()[1] == pytest.approx(5.0625)
    assert r.g.tolist() == [1.5, 2.0, 3.0, 4.0]
    assert r.nn.tolist() == [False, False, False, True]


def test_dates(df):
    r = df.select(F.year("d").alias("y"), F.month("d").alias("m"), F.dayofmonth("d").alias("dd"),
                  F.date_add("d", 1).alias("n"), F.datediff("d", F.lit("2024-01-01")).alias("dd2")).toPandas()
    assert r.y.tolist()[:3] == [2024, 2024, 2023]
    assert r.n.tolist()[:2] == ["2024-02-01", "2024-03-01"]
    assert r.dd2.tolist()[:3] == [30, 59, -7]


def test_arrays_and_explode(df):
    arr = df.select("k", F.split("tags", ",").alias("t"))
    r = arr.select("k", F.size("t").alias("n"), F.array_contains("t", "c").alias("hasc")).toPandas()
    assert r.n.tolist() == [2, 1, 1, 3] and r.hasc.tolist() == [False, True, False, False]
    ex = arr.select("k", F.explode("t").alias("tag")).toPandas()
    assert ex.tag.tolist() == ["a", "b", "c", "", "d", "e", "f"]
    assert ex.k.tolist() == [1, 1, 2, 1, 2, 2, 2]
    pe = arr.select(F.posexplode("t")).toPandas()
    assert pe["pos"].tolist() == [0, 1, 0, 0, 0, 1, 2]


def test_new_aggregates_and_expr(df):
    g = df.groupBy("k").agg(F.first("name").alias("f"), F.last("x").alias("l"),
                            F.collect_list("x").alias("cl"), F.sumDistinct("k").alias("sd")).toPandas()
    g = g.set_index("k")
    assert g.loc[1, "f"] == "  Alice " and g.loc[2, "l"] == 4.0
    assert g.loc[1, "cl"] == [1.5, 3.0] and g.loc[2, "sd"] == 2
    r = df.select(F.expr("x * 2 + k").alias("e")).toPandas()
    assert r.e.tolist() == [4.0, -2.5, 7.0, 10.0]


def test_rand_and_ids_are_deterministic(df):
    a = df.select(F.rand(7).alias("r"), F.randn(7).alias("z"), F.monotonically_increasing_id().alias("i")).toPandas()
    b = df.select(F.rand(7).alias("r"), F.randn(7).alias("z")).toPandas()
    assert a.r.tolist() == b.r.tolist() and all(0 <= v < 1 for v in a.r)
    assert a.i.tolist() == [0, 1, 2, 3] and all(math.isfinite(v) for v in a.z)


def test_udf(df):
    plus = F.udf(lambda v, k: v * 10 + k, "double")
    r = df.select(plus("x", "k").alias("u")).toPandas()
    assert r.u.tolist() == [16.0, -20.5, 31.0, 42.0]
    up = F.udf(lambda s: s.upper())
    assert df.select(up("name").alias("n")).toPandas().n.tolist()[1] == "BOB"
    _ = np


def test_ml_functions_vector_array_roundtrip():
    import numpy as np
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.ml.feature import HashingTF, VectorAssembler
    from orange3_spark_amd.ml.functions import array_to_vector, predict_batch_udf, vector_to_array
    s = Session(SessionConf().set("o3s.device", "cpu"))
    df = VectorAssembler(inputCols=["a", "b"], outputCol="v").transform(
        s.createDataFrame(pd.DataFrame({"a": [1.0, 2.0, -1.5], "b": [3.0, 4.0, 0.25]})))
    arr = df.withColumn("arr", vector_to_array("v"))
    assert [r.arr for r in arr.select("arr").collect()] == [[1.0, 3.0], [2.0, 4.0], [-1.5, 0.25]]
    back = arr.withColumn("v2", array_to_vector("arr")).select("v2").collect()
    assert np.allclose([r.v2.toArray() for r in back], [[1, 3], [2, 4], [-1.5, 0.25]])
    tf = HashingTF(inputCol="w", outputCol="tf", numFeatures=16).transform(
        s.createDataFrame(pd.DataFrame({"w": [["a", "b", "a"], ["c"]]})))
    dense = [r.x for r in tf.select(vector_to_array("tf").alias("x")).collect()]
    assert len(dense[0]) == 16 and sum(dense[0]) == 3.0 and sum(dense[1]) == 1.0
    pred = predict_batch_udf(lambda: (lambda x: x.sum(axis=1)), return_type="double", batch_size=2)
    assert [r.p for r in df.select(pred("v").alias("p")).collect()] == [4.0, 6.0, -1.25]


def test_extended_function_surface():
    import json as _json
    import math
    import numpy as np
    import pandas as pd
    from scipy import stats
    from orange3_spark_amd import Session, SessionConf
    import orange3_spark_amd.sql.functions as F
    s = Session(SessionConf().set("o3s.device", "cpu"))
    df = s.createDataFrame(pd.DataFrame({
        "s": ["a.b.c", "Robert", "hello"], "d": ["2024-01-31", "2024-02-15 10:30:00", "2023-12-01"],
        "j": ['{"a": {"b": [1, 2]}, "c": "x"}', '{"a": {"b": [3]}}', "not json"],
        "n": [5, -3, 10], "t": ["x", "x", "y"]}))
    r = df.select(
        F.substring_index("s", ".", 2).alias("si"), F.soundex("s").alias("sx"), F.levenshtein("s", "t").alias("lv"),
        F.ascii("s").alias("asc"), F.base64("t").alias("b64"), F.hex("n").alias("hx"), F.conv("n", 10, 2).alias("cv"),
        F.crc32("t").alias("crc"), F.translate("s", "abc", "xy").alias("tr"), F.locate("l", "s").alias("lc"),
        F.format_string("%s-%d", "t", "n").alias("fs"), F.get_json_object("j", "$.a.b[0]").alias("gj"),
        F.get_json_object("j", "$.c").alias("gc"), F.weekofyear("d").alias("wk"), F.quarter("d").alias("q"),
        F.last_day("d").alias("ld"), F.add_months("d", 1).alias("am"), F.date_trunc("month", "d").alias("dt"),
        F.unix_timestamp("d", "yyyy-MM-dd").alias("ut"), F.nvl(F.lit(None), "n").alias("nv"),
        F.nullif("t", F.lit("x")).alias("ni"), F.factorial(F.lit(5)).alias("fa"), F.shiftleft("n", 2).alias("sl"),
        F.xxhash64("t").alias("xx")).toPandas()
    assert list(r.si) == ["a.b", "Robert", "hello"] and r.sx[1] == "R163" and r.lv[2] == 5
    assert r.asc[0] == 97 and r.b64[0] == "eA==" and r.hx[0] == "5" and r.cv[0] == "101"
    assert r.tr[0] == "x.y." and r.lc[2] == 3 and r.fs[0] == "x-5"
    assert r.gj[0] == "1" and r.gj[1] == "3" and r.gj[2] is None and r.gc[0] == "x"
    assert r.wk[0] == 5 and r.q[1] == 1 and r.ld[1] == "2024-02-29" and r.am[0] == "2024-02-29"
    assert r.dt[1] == "2024-02-01 00:00:00" and r.nv[0] == 5 and r.ni[2] == "y" and (pd.isna(r.ni[0]) or r.ni[0] is None)
    assert r.fa[0] == 120 and r.sl[0] == 20 and r.xx[0] == r.xx[1] != r.xx[2]
    a = s.createDataFrame(pd.DataFrame({"k": [1, 2]})).select(
        F.sequence(F.lit(1), F.lit(4)).alias("seq"), F.array(F.lit(3), F.lit(1), F.lit(3)).alias("arr"))
    a = a.select("seq", "arr", F.array_join("arr", "|").alias("aj"), F.array_position("arr", 1).alias("ap"),
                 F.array_remove("arr", 3).alias("ar"), F.slice("seq", 2, 2).alias("sc"),
                 F.array_union("arr", "seq").alias("au"), F.array_intersect("arr", "seq").alias("ai"),
                 F.array_except("seq", "arr").alias("ae"), F.array_max("seq").alias("mx"),
                 F.array_sort("arr").alias("so"), F.arrays_zip("seq", "arr").alias("z"),
                 F.to_json(F.struct("seq")).alias("tj"), F.map_keys(F.create_map(F.lit("a"), F.lit(1))).alias("mk"))
    row = a.collect()[0]
    assert row.seq == [1, 2, 3, 4] and row.aj == "3|1|3" and row.ap == 2 and row.ar == [1] and row.sc == [2, 3]
    assert row.au == [3, 1, 2, 4] and row.ai == [3, 1] and row.ae == [2, 4] and row.mx == 4.0 and row.so == [1, 3, 3]
    assert row.z[0] == [1, 3] and _json.loads(row.tj) == {"seq": [1, 2, 3, 4]} and row.mk == ["a"]
    e = s.createDataFrame(pd.DataFrame({"id": [1, 2]})).withColumn(
        "v", F.when(F.col("id") == 1, F.array(F.lit(7), F.lit(8))).otherwise(F.array()))
    assert e.select("id", F.explode_outer("v").alias("x")).count() == 3
    rng = np.random.default_rng(1)
    pdf = pd.DataFrame({"x": rng.normal(size=400), "y": rng.normal(size=400)})
    st = s.createDataFrame(pdf).agg(F.skewness("x").alias("sk"), F.kurtosis("x").alias("ku"),
                                    F.corr("x", "y").alias("c"), F.covar_samp("x", "y").alias("cs"),
                                    F.percentile_approx("x", [0.25, 0.75]).alias("q")).collect()[0]
    assert math.isclose(st.sk, stats.skew(pdf.x), rel_tol=1e-9)
    assert math.isclose(st.ku, stats.kurtosis(pdf.x), rel_tol=1e-9)
    assert math.isclose(st.c, np.corrcoef(pdf.x, pdf.y)[0, 1], rel_tol=1e-9)
    assert math.isclose(st.cs, np.cov(pdf.x, pdf.y)[0, 1], rel_tol=1e-9)
    xs = np.sort(pdf.x.to_numpy())
    assert st.q == [xs[99], xs[299]]
    pu = F.pandas_udf(lambda v: v * 2, "double")
    assert [r.p for r in s.createDataFrame(pd.DataFrame({"v": [1.0, 2.5]})).select(pu("v").alias("p")).collect()] \
        == [2.0, 5.0]


def test_higher_order_and_round_out_functions():
    import pandas as pd
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.sql import functions as F
    s = Session(SessionConf().set("o3s.device", "cpu"))
    df = s.createDataFrame(pd.DataFrame({"id": [1, 2, 3], "t": ["ab cd", "x", "Hello"], "v": [1.0, 2.0, 4.0]}))
    a = df.withColumn("arr", F.array(F.col("v"), F.col("v") * 2, F.lit(5.0)))
    r = a.select(F.transform("arr", lambda x: x * 10).alias("tr"), F.transform("arr", lambda x, i: x + i).alias("ti"),
                 F.filter("arr", lambda x: x > 3).alias("fi"), F.exists("arr", lambda x: x > 7).alias("ex"),
                 F.forall("arr", lambda x: x > 0).alias("fa"),
                 F.aggregate("arr", F.lit(0.0), lambda acc, x: acc + x, lambda acc: acc * 2).alias("ag"),
                 F.zip_with("arr", "arr", lambda x, y: x * y).alias("zw"),
                 F.transform("arr", lambda x: x + F.col("id")).alias("outer")).collect()
    assert r[0].tr == [10.0, 20.0, 50.0] and r[0].ti == [1.0, 3.0, 7.0] and r[1].fi == [4.0, 5.0]
    assert [x.ex for x in r] == [False, False, True] and all(x.fa for x in r)
    assert [x.ag for x in r] == [16.0, 22.0, 34.0] and r[2].zw == [16.0, 64.0, 25.0] and r[2].outer == [7.0, 11.0, 8.0]
    m = df.select(F.create_map(F.lit("a"), F.col("v"), F.lit("b"), F.col("v") * 3).alias("m")).select(
        F.transform_values("m", lambda k, v: v + 1).alias("tv"), F.map_filter("m", lambda k, v: v > 3).alias("mf"),
        F.transform_keys("m", lambda k, v: F.upper(k)).alias("tk")).collect()
    assert m[1].tv == {"a": 3.0, "b": 7.0} and m[1].mf == {"b": 6.0} and m[0].tk == {"A": 1.0, "B": 3.0}
    g = s.createDataFrame(pd.DataFrame({"k": ["a", "a", "b", "b", "b"], "x": [1.0, 3.0, 2.0, 2.0, 5.0],
                                        "y": [5, 1, 2, 9, 3], "b": [True, False, True, True, True]}))
    got = {row.k: row for row in g.groupBy("k").agg(
        F.median("x").alias("md"), F.mode("x").alias("mo"), F.product("x").alias("p"),
        F.count_if(F.col("x") > 1.5).alias("ci"), F.bool_and("b").alias("ba"), F.bool_or("b").alias("bo"),
        F.max_by("x", "y").alias("mb"), F.min_by("x", "y").alias("nb")).collect()}
    assert (got["a"].md, got["a"].mo, got["a"].p, got["a"].ci, got["a"].ba, got["a"].mb, got["a"].nb) == \
        (2.0, 1.0, 3.0, 1, False, 1.0, 3.0)
    assert (got["b"].md, got["b"].mo, got["b"].p, got["b"].ci, got["b"].ba, got["b"].bo) == (2.0, 2.0, 20.0, 3, True, True)
    g.createOrReplaceTempView("hof")
    q = s.sql("SELECT k, median(x) AS md, max_by(x, y) AS mb, count_if(x > 1.5) AS ci FROM hof GROUP BY k").collect()
    assert {row.k: (row.md, row.mb, row.ci) for row in q} == {"a": (2.0, 1.0, 1), "b": (2.0, 2.0, 3)}
    row = df.select(F.like("t", "a%").alias("l"), F.ilike("t", "h%").alias("il"), F.left("t", F.lit(2)).alias("le"),
                    F.split_part("t", F.lit(" "), F.lit(2)).alias("sp"), F.overlay("t", F.lit("ZZ"), F.lit(1)).alias("ov"),
                    F.width_bucket("v", F.lit(0.0), F.lit(4.0), F.lit(4)).alias("wb"),
                    F.try_divide("v", F.col("v") - 1).alias("td"), F.pmod(F.col("v") - 3, F.lit(2.0)).alias("pm"),
                    F.nvl2("t", F.lit(1), F.lit(0)).alias("n2"),
                    F.array_insert(F.array(F.col("v")), F.lit(1), F.lit(9.0)).alias("ai")).collect()
    assert [x.l for x in row] == [True, False, False] and row[2].il and row[0].le == "ab" and row[0].sp == "cd"
    assert row[0].ov == "ZZ cd" and [x.wb for x in row] == [2, 3, 5] and row[0].td is None and row[1].td == 2.0
    assert row[0].pm == 0.0 and row[0].n2 == 1 and row[1].ai == [9.0, 2.0]
    st = s.createDataFrame(pd.DataFrame({"id": [1, 2]}))
    st = st.select("id", F.array(F.struct(F.col("id").alias("a"), (F.col("id") * 2).alias("b"))).alias("s"))
    assert st.select("id", F.inline("s")).collect()[1].b == 4


def test_column_string_predicates_and_null_safe_eq(s):
    d = s.createDataFrame(pd.DataFrame({"a": ["apple", "banana", None, "cherry_pie", "a%b"],
                                        "n": [1, 2, None, 4, 6]}))
    r = d.select(F.col("a").startswith("a").alias("sw"), F.col("a").endswith("e").alias("ew"),
                 F.col("a").contains("an").alias("c"), F.col("a").like("%an_na").alias("l"),
                 F.col("a").rlike("^c.*e$").alias("r"), F.col("a").like("a\\%b").alias("esc"),
                 F.col("a").ilike("APP%").alias("il"), F.col("a").substr(2, 3).alias("sub"),
                 F.col("n").eqNullSafe(None).alias("ens"), F.col("n").eqNullSafe(2).alias("en2"),
                 F.col("n").cast("long").bitwiseAND(3).alias("band")).collect()
    assert [x.sw for x in r] == [True, False, None, False, True]
    assert [x.ew for x in r] == [True, False, None, True, False]
    assert [x.c for x in r] == [False, True, None, False, False]
    assert [x.l for x in r] == [False, True, None, False, False]
    assert [x.r for x in r] == [False, False, None, True, False]
    assert [x.esc for x in r] == [False, False, None, False, True]   # escaped % is literal
    assert [x.il for x in r] == [True, False, None, False, False]
    assert [x.sub for x in r] == ["ppl", "ana", None, "her", "%b"]
    assert [x.ens for x in r] == [False, False, True, False, False]  # null <=> null is true
    assert [x.en2 for x in r] == [False, True, False, False, False]  # never null
    assert [x.band for x in r][:2] == [1, 2] and r[4].band == 2


def test_tumbling_and_sliding_windows(s):
    """window(ts, dur) = the one window holding ts; window(ts, dur, slide) repeats each row
    once per overlapping window (Spark's sliding expansion), groupBy(window(...)) included."""
    ts = ["2024-01-01 00:01:00", "2024-01-01 00:07:30", "2024-01-01 00:12:00"]
    d = s.createDataFrame(pd.DataFrame({"ts": ts, "v": [1.0, 2.0, 3.0]}))
    tw = d.select("v", F.window("ts", "10 minutes")).collect()
    assert [(r.v, r.window.start) for r in tw] == [(1.0, "2024-01-01 00:00:00"), (2.0, "2024-01-01 00:00:00"),
                                                   (3.0, "2024-01-01 00:10:00")]
    sw = d.select("v", F.window("ts", "10 minutes", "5 minutes")).collect()
    got = [(r.v, r.window.start, r.window.end) for r in sw]
    assert got == [(1.0, "2023-12-31 23:55:00", "2024-01-01 00:05:00"),
                   (1.0, "2024-01-01 00:00:00", "2024-01-01 00:10:00"),
                   (2.0, "2024-01-01 00:00:00", "2024-01-01 00:10:00"),
                   (2.0, "2024-01-01 00:05:00", "2024-01-01 00:15:00"),
                   (3.0, "2024-01-01 00:05:00", "2024-01-01 00:15:00"),
                   (3.0, "2024-01-01 00:10:00", "2024-01-01 00:20:00")]
    # every (row, window) pair satisfies start <= ts < end, 3 windows per row for slide = dur / 3
    sw3 = d.select("ts", F.window("ts", "15 minutes", "5 minutes")).collect()
    assert len(sw3) == 9 and all(r.window.start <= r.ts < r.window.end for r in sw3)
    agg = sorted((tuple(r.window), r["sum(v)"]) for r in
                 d.groupBy(F.window("ts", "10 minutes", "5 minutes")).agg(F.sum("v")).collect())
    assert [a[1] for a in agg] == [1.0, 3.0, 5.0, 3.0]
    with pytest.raises(ValueError):
        F.window("ts", "5 minutes", "10 minutes")


def test_percentile_stack_and_misc_functions(s):
    pdf = pd.DataFrame({"g": ["a", "b", "a", "b", "a"], "v": [1.0, 2.0, 3.0, 4.0, 5.0], "k": [1, 2, 3, 4, 2],
                        "t": ["Hi there. How are you?", "x", "y", "z", "w"]})
    d = s.createDataFrame(pdf)
    out = d.groupBy("g").agg(F.percentile("v", 0.5).alias("p"), F.percentile("v", [0.25, 0.75]).alias("pp"),
                             F.median("v").alias("m")).orderBy("g").collect()
    for r in out:
        vs = pdf.v[pdf.g == r.g].to_numpy()
        assert r.p == pytest.approx(np.percentile(vs, 50)) == pytest.approx(r.m)
        assert r.pp == pytest.approx(list(np.percentile(vs, [25, 75])))
    st = d.select("g", F.stack(2, "k", "v")).collect()
    assert [(r.g, r.col0) for r in st] == [(g, float(x)) for g, k, v in zip(pdf.g, pdf.k, pdf.v) for x in (k, v)]
    r = d.select(F.typeof("v").alias("tv"), F.ceiling("v").alias("c"), F.btrim(F.lit("xxaxx"), "x").alias("b"),
                 F.sentences("t").alias("se"), F.to_char("v", "$999,999.00").alias("tc"),
                 F.to_number(F.lit("1,234.5"), "9,999.9").alias("tn"),
                 F.try_to_number(F.lit("abc"), "999").alias("bad")).collect()[0]
    assert (r.tv, r.c, r.b, r.tc, r.tn, r.bad) == ("double", 1.0, "a", "$1.00", 1234.5, None)
    assert r.se == [["Hi", "there"], ["How", "are", "you"]]
    with pytest.raises(RuntimeError, match="not true"):
        d.select(F.assert_true(F.col("v") > 2)).collect()
    assert d.select(F.assert_true(F.col("v") > 0).alias("ok")).collect()[0].ok is None
    with pytest.raises(ValueError):
        d.select(F.to_number(F.lit("abc"), "999")).collect()


def test_struct_fields_and_window_group_keys(s):
    """groupBy(window(...)) keeps Row keys; window.start / getField / SQL w.start read fields."""
    ts = ["2024-01-01 00:01:00", "2024-01-01 00:07:30", "2024-01-01 00:12:00"]
    d = s.createDataFrame(pd.DataFrame({"ts": ts, "v": [1.0, 2.0, 3.0]}))
    g = d.groupBy(F.window("ts", "10 minutes")).agg(F.sum("v").alias("s")).orderBy("window.start")
    rows = g.collect()
    assert [(r.window.start, r.window.end, r.s) for r in rows] == [
        ("2024-01-01 00:00:00", "2024-01-01 00:10:00", 3.0), ("2024-01-01 00:10:00", "2024-01-01 00:20:00", 3.0)]
    assert g.select("window.start", "s").columns == ["start", "s"]
    assert [r[0] for r in g.select(F.col("window").getField("end")).collect()] == [
        "2024-01-01 00:10:00", "2024-01-01 00:20:00"]
    d.createOrReplaceTempView("tw_struct")
    got = sorted(tuple(r) for r in s.sql("SELECT w.start AS st, sum(v) AS sv FROM (SELECT window(ts, '10 minutes') "
                                         "AS w, v FROM tw_struct) GROUP BY w.start").collect())
    assert got == [("2024-01-01 00:00:00", 3.0), ("2024-01-01 00:10:00", 3.0)]


def test_struct_with_and_drop_fields(s):
    d = s.createDataFrame(pd.DataFrame({"a": [1, 2], "b": ["x", "y"]}))
    st = d.select(F.struct("a", "b").alias("s"))
    r = st.select(F.col("s").withField("c", F.col("s").getField("a") * 10).alias("s2")).collect()
    assert [(x.s2.a, x.s2.b, x.s2.c) for x in r] == [(1, "x", 10), (2, "y", 20)]
    r = st.select(F.col("s").withField("a", F.lit(0)).dropFields("b").alias("s3")).collect()
    assert [tuple(x.s3.__fields__) for x in r] == [("a",), ("a",)] and [x.s3.a for x in r] == [0, 0]
