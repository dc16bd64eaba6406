"""Spark 3.4 / 3.5 sql.functions additions (DataFrame API and SQL), checked against values
worked out by hand from Spark's documented semantics."""
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.sql import functions as F


@pytest.fixture(scope="module")
def df():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    d = s.createDataFrame([("a", 5, "x y&z", "[1,2,3]", '{"k":1,"j":2}', "2024-03-06"),
                           ("a", 3, "abc123def45", "[]", "{}", "2024-03-09"),
                           ("b", 6, "q", "x", "[1]", "2024-03-10")], ["g", "v", "s", "ja", "jo", "d"])
    d.createOrReplaceTempView("f35")
    return d


def test_bit_aggregates_and_array_agg(df):
    r = df.groupBy("g").agg(F.bit_and("v").alias("ba"), F.bit_or("v").alias("bo"), F.bit_xor("v").alias("bx"),
                            F.array_agg("v").alias("aa")).orderBy("g").toPandas()
    assert r.ba.tolist() == [1, 6] and r.bo.tolist() == [7, 6] and r.bx.tolist() == [6, 6]
    assert r.aa.tolist() == [[5, 3], [6]]
    q = df.sparkSession.sql("SELECT g, bit_xor(v) AS x FROM f35 GROUP BY g ORDER BY g").toPandas() \
        if hasattr(df, "sparkSession") else None
    if q is not None:
        assert q.x.tolist() == [6, 6]


def test_scalar_additions(df):
    r = df.select(F.bit_count("v").alias("bc"), F.weekday("d").alias("wd"), F.day("d").alias("dy"),
                  F.date_from_unix_date(F.lit(19000)).alias("du"), F.json_array_length("ja").alias("jl"),
                  F.json_object_keys("jo").alias("jk"), F.regexp_count("s", F.lit(r"\d+")).alias("rc"),
                  F.regexp_substr("s", F.lit(r"\d+")).alias("rs"),
                  F.replace("s", F.lit("abc"), F.lit("Z")).alias("rp"), F.substr("s", F.lit(2), F.lit(3)).alias("ss"),
                  F.url_encode("s").alias("ue"), F.url_decode(F.url_encode("s")).alias("ud"),
                  F.position(F.lit("c"), "s").alias("po"), F.negate("v").alias("ng"),
                  F.try_multiply("v", F.lit(2)).alias("tm"), F.try_subtract("v", F.lit(1)).alias("ts"),
                  F.make_timestamp(F.lit(2024), F.lit(1), F.lit(2), F.lit(3), F.lit(4), F.lit(5.5)).alias("mt"),
                  F.map_contains_key(F.create_map(F.lit("k"), "v"), "k").alias("mk"),
                  F.named_struct(F.lit("a"), "v").alias("ns"), F.uuid().alias("u")).toPandas()
    assert r.bc.tolist() == [2, 2, 2] and r.wd.tolist() == [2, 5, 6] and r.dy.tolist() == [6, 9, 10]
    assert r.du.tolist() == ["2022-01-08"] * 3
    assert r.jl.tolist()[:2] == [3, 0] and r.jl.isna().tolist()[2]
    assert r.jk.tolist()[:2] == [["k", "j"], []]
    assert r.rc.tolist() == [0, 2, 0] and r.rs.tolist() == [None, "123", None]
    assert r.rp.tolist() == ["x y&z", "Z123def45", "q"] and r.ss.tolist() == [" y&", "bc1", ""]
    assert r.ue.tolist()[0] == "x+y%26z" and r.ud.tolist() == ["x y&z", "abc123def45", "q"]
    assert r.po.tolist() == [0, 3, 0] and r.ng.tolist() == [-5, -3, -6]
    assert r.tm.tolist() == [10, 6, 12] and r.ts.tolist() == [4, 2, 5]
    assert r.mt.tolist()[0] == "2024-01-02 03:04:05.5" and r.mk.tolist() == [True] * 3
    assert [x.a for x in r.ns.tolist()] == [5, 3, 6] and len(set(r.u.tolist())) == 3


def test_sql_spellings(df):
    s = Session.getOrCreate() if not hasattr(df, "sparkSession") else df.sparkSession
    q = s.sql("SELECT regexp_count(s, '[a-z]') AS c, url_encode(s) AS u, weekday(d) AS w FROM f35").toPandas()
    assert q.c.tolist() == [3, 6, 1] and q.w.tolist() == [2, 5, 6]


def test_from_csv_and_schema_of_csv():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    d = s.createDataFrame([("1,abc,2.5", '{"a": 3, "b": "z"}'), ("7,,x", "{}")], ["t", "j"])
    r = d.select(F.from_csv("t", "a INT, b STRING, c DOUBLE").alias("r"),
                 F.from_json("j", "STRUCT<a: INT, b: STRING>").alias("q")).toPandas()
    assert [(x.a, x.b, x.c) for x in r.r] == [(1, "abc", 2.5), (7, None, None)]   # malformed field -> null
    assert [(x.a, x.b) for x in r.q] == [(3, "z"), (None, None)]
    ddl = d.select(F.schema_of_csv(F.lit("1,abc,2.5")).alias("x")).toPandas().x[0]
    assert ddl == "STRUCT<_c0: INT, _c1: STRING, _c2: DOUBLE>"


def test_map_zip_with():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    d = s.createDataFrame([(1,)], ["id"]).select(
        F.create_map(F.lit("a"), F.lit(1), F.lit("b"), F.lit(2)).alias("m1"),
        F.create_map(F.lit("b"), F.lit(10), F.lit("c"), F.lit(20)).alias("m2"))
    r = d.select(F.map_zip_with("m1", "m2", lambda k, v1, v2: F.coalesce(v1, F.lit(0)) + F.coalesce(v2, F.lit(0)))
                 .alias("z")).toPandas().z[0]
    assert {k: int(v) for k, v in r.items()} == {"a": 1, "b": 12, "c": 20}


def test_histogram_numeric():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    d = s.createDataFrame([("a", float(v)) for v in [1, 2, 2, 3, 10, 11, 12, 30]], ["g", "v"])
    h = d.groupBy("g").agg(F.histogram_numeric("v", 3).alias("h")).toPandas().h[0]
    assert [(r.x, r.y) for r in h] == [(2.0, 4.0), (11.0, 3.0), (30.0, 1.0)]   # counts sum to the rows
    d.createOrReplaceTempView("hn35")
    h2 = s.sql("SELECT histogram_numeric(v, 2) AS h FROM hn35").toPandas().h[0]
    assert [r.y for r in h2] == [7.0, 1.0] and h2[0].x == pytest.approx(41 / 7)


def test_datetime_epoch_and_misc_builtins():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    d = s.createDataFrame([("2024-03-06 10:20:30", "Ab1-x", 3, "a,b,c", 1709720430123)], ["t", "s", "n", "csv", "ms"])
    r = d.select(F.unix_seconds("t").alias("us"), F.unix_date("t").alias("ud"), F.unix_millis("t").alias("um"),
                 F.timestamp_millis("ms").alias("tm"), F.date_part(F.lit("YEAR"), "t").alias("y"),
                 F.extract(F.lit("hour"), "t").alias("h"),
                 F.convert_timezone(F.lit("UTC"), F.lit("Asia/Tokyo"), "t").alias("ct"), F.mask("s").alias("m"),
                 F.find_in_set(F.lit("b"), "csv").alias("fs"), F.elt(F.lit(2), F.lit("x"), F.lit("y")).alias("el"),
                 F.chr(F.lit(65)).alias("ch"), F.shiftrightunsigned(F.lit(-1), 60).alias("sr"),
                 F.to_binary(F.lit("4142")).alias("tb"), F.printf(F.lit("%d-%s"), "n", "s").alias("pf")).toPandas()
    row = r.iloc[0]
    assert (row.us, row.ud, row.um) == (1709720430, 19788, 1709720430000)
    assert row.tm == "2024-03-06 10:20:30.123" and (row.y, row.h) == (2024, 10)
    assert row.ct == "2024-03-06 19:20:30" and row.m == "Xxn-x" and row.fs == 2 and row.el == "y"
    assert row.ch == "A" and row.sr == 15 and row.tb == b"AB" and row.pf == "3-Ab1-x"


def test_sql_extract_from():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    s.createDataFrame([("2024-03-06 10:20:30", "a,b")], ["t", "c"]).createOrReplaceTempView("ex35")
    q = s.sql("SELECT extract(YEAR FROM t) AS y, EXTRACT(minute FROM t) AS m, date_part('MONTH', t) AS mo, "
              "find_in_set('b', c) AS f FROM ex35").toPandas()
    assert q.to_dict("list") == {"y": [2024], "m": [20], "mo": [3], "f": [2]}


def test_shiftrightunsigned_width_and_url_encode_java_safe_set():
    """>>> shifts an int column as a 32-bit value and a bigint as 64-bit (Spark
    ShiftRightUnsigned); url_encode keeps java.net.URLEncoder's safe set ('*' stays,
    '~' is encoded)."""
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.sql import functions as F
    s = Session(SessionConf().set("o3s.device", "cpu"))
    df = s.createDataFrame({"a": [-1, 8], "t": ["a b~c*d", "é"]})
    df = df.withColumn("ai", df.a.cast("int"))
    got = df.select(F.shiftrightunsigned("ai", 28).alias("i"), F.shiftrightunsigned("a", 60).alias("l"),
                    F.url_encode("t").alias("u")).collect()
    assert [tuple(r) for r in got] == [(15, 15, "a+b%7Ec*d"), (0, 0, "%C3%A9")]
