"""DataFrame op timings on the GPU (20M-row range frame: groupBy / join / sort / window
-style ops), one JSON line."""
import sys, time, json, os
sys.path.insert(0, os.getcwd())
import torch
from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.sql import functions as F
s = Session(SessionConf().set("o3s.device", "cuda"))
n = 20_000_000
df = s.range(n).withColumn("k", F.col("id") % 1000).withColumn("v", F.rand(seed=1)).cache()
df.count()
res = {}
sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
def t(name, fn):
    sync(); a = time.perf_counter(); out = fn(); sync()
    res[name] = round(time.perf_counter() - a, 4)
t("groupBy_count", lambda: df.groupBy("k").count().count())
t("groupBy_agg", lambda: df.groupBy("k").agg(F.sum("v"), F.avg("v"), F.max("v")).count())
t("filter_count", lambda: df.filter(F.col("v") > 0.5).count())
t("orderBy_limit", lambda: df.orderBy(F.col("v").desc()).limit(10).collect())
t("sample", lambda: df.sample(False, 0.1, seed=3).count())
small = s.range(1000).withColumn("k", F.col("id")).withColumn("name", F.col("id") * 2)
t("join_small", lambda: df.join(small, "k").count())
t("distinct_k", lambda: df.select("k").distinct().count())
t("describe", lambda: df.describe("v").collect())
print(json.dumps(res))
res2 = {}
def t2(name, fn):
    sync(); a = time.perf_counter()
    try:
        fn()
        sync()
        res2[name] = round(time.perf_counter() - a, 4)
    except Exception as e:  # noqa: BLE001
        res2[name] = f"error: {type(e).__name__}: {str(e)[:80]}"
t2("withColumn_expr", lambda: df.withColumn("z", F.col("v") * 2 + F.col("k")).count())
t2("fillna", lambda: df.fillna(0.0).count())
t2("dropna", lambda: df.dropna().count())
t2("union", lambda: df.union(df).count())
t2("orderBy_full", lambda: df.orderBy("v").count())
t2("dropDuplicates", lambda: df.dropDuplicates(["k"]).count())
t2("pivot", lambda: df.filter(F.col("k") < 10).groupBy("k").pivot("k").count().count())
t2("sql_groupby", lambda: (df.createOrReplaceTempView("t"), s.sql("SELECT k, COUNT(*) c, AVG(v) a FROM t GROUP BY k").count()))
t2("toPandas_1M", lambda: df.limit(1_000_000).toPandas())
from orange3_spark_amd.sql.window import Window
t2("window_rank_1M", lambda: df.limit(1_000_000).withColumn("r", F.row_number().over(Window.partitionBy("k").orderBy("v"))).count())
t2("string_ops_1M", lambda: df.limit(1_000_000).withColumn("s", F.concat(F.lit("x"), F.col("k").cast("string"))).filter(F.col("s").startswith("x1")).count())
print(json.dumps(res2))
# condition joins / SQL subqueries (this round)
res3 = {}
def t3(name, fn):
    sync(); a = time.perf_counter()
    try:
        fn(); sync()
        res3[name] = round(time.perf_counter() - a, 4)
    except Exception as e:  # noqa: BLE001
        res3[name] = f"error: {type(e).__name__}: {str(e)[:80]}"
dims = s.range(1000).withColumn("uid", F.col("id")).withColumn("lo", F.col("id") / 1000.0).withColumn("hi", F.col("id") / 1000.0 + 0.0005)
t3("cond_join_equi_20Mx1K", lambda: df.join(dims, df.k == dims.uid).count())
t3("cond_join_equi_residual_20Mx1K", lambda: df.join(dims, (df.k == dims.uid) & (df.v > dims.lo)).count())
part = df.limit(1_000_000)
t3("band_join_nested_loop_1Mx1K", lambda: part.join(dims, (part.v >= dims.lo) & (part.v < dims.hi)).count())
dims.createOrReplaceTempView("dims")
t3("sql_exists_20M", lambda: s.sql("SELECT count(*) FROM t WHERE EXISTS (SELECT 1 FROM dims WHERE dims.uid = t.k AND dims.lo < 0.5)").collect())
t3("sql_in_subquery_20M", lambda: s.sql("SELECT count(*) FROM t WHERE k IN (SELECT uid FROM dims WHERE lo < 0.5)").collect())
print(json.dumps(res3))
