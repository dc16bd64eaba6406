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
