"""RDD / SparkContext API (orange3_spark_amd/rdd.py): semantics against plain-Python
references on one rank, and world-size invariance of every shuffle on 2 gloo ranks."""
import json
import os
import socket
from collections import Counter, defaultdict

import pytest
import torch.multiprocessing as mp

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.rdd import StatCounter, portable_hash


@pytest.fixture(scope="module")
def sc():
    return Session(SessionConf().set("o3s.device", "cpu")).sparkContext


def test_word_count_and_narrow_ops(sc):
    lines = ["a b c", "b c", "c", "", "d a"]
    r = sc.parallelize(lines, 3)
    assert r.getNumPartitions() == 3
    wc = dict(r.flatMap(str.split).map(lambda w: (w, 1)).reduceByKey(lambda a, b: a + b).collect())
    assert wc == dict(Counter(" ".join(lines).split()))
    assert r.filter(bool).count() == 4
    assert r.map(len).collect() == [len(x) for x in lines]
    assert r.glom().map(len).sum() == len(lines)
    assert r.mapPartitionsWithIndex(lambda i, it: [(i, sum(1 for _ in it))]).collect() == [(0, 1), (1, 2), (2, 2)]
    assert sc.range(10).keyBy(lambda x: x % 3).countByKey() == {0: 4, 1: 3, 2: 3}
    assert sc.range(7).zipWithIndex().collect() == [(i, i) for i in range(7)]
    assert sorted(sc.range(6, numSlices=3).zipWithUniqueId().values().collect()) == [0, 1, 2, 3, 4, 5]


def test_actions(sc):
    r = sc.parallelize(list(range(1, 101)), 4)
    assert r.sum() == 5050 and r.count() == 100 and r.first() == 1
    assert r.reduce(lambda a, b: a + b) == 5050
    assert r.fold(0, lambda a, b: a + b) == 5050
    assert r.aggregate((0, 0), lambda acc, x: (acc[0] + x, acc[1] + 1), lambda a, b: (a[0] + b[0], a[1] + b[1])) \
        == (5050, 100)
    assert r.top(3) == [100, 99, 98] and r.takeOrdered(2) == [1, 2] and r.take(3) == [1, 2, 3]
    assert r.max() == 100 and r.min() == 1 and abs(r.mean() - 50.5) < 1e-12
    st = r.stats()
    assert st.count() == 100 and abs(st.sampleStdev() - StatCounter(range(1, 101)).sampleStdev()) < 1e-12
    edges, counts = r.histogram([0, 50, 101])
    assert counts == [49, 51]
    assert sc.emptyRDD().isEmpty() and not r.isEmpty()
    assert len(r.takeSample(False, 10, seed=1)) == 10
    with pytest.raises(ValueError):
        sc.emptyRDD().reduce(lambda a, b: a)


def test_pair_shuffles(sc):
    a = sc.parallelize([(1, "a"), (2, "b"), (2, "bb"), (3, "c")], 2)
    b = sc.parallelize([(2, "x"), (3, "y"), (3, "yy"), (4, "z")], 3)
    assert sorted(a.join(b).collect()) == [(2, ("b", "x")), (2, ("bb", "x")), (3, ("c", "y")), (3, ("c", "yy"))]
    assert sorted(a.leftOuterJoin(b).collect())[0] == (1, ("a", None))
    assert (4, (None, "z")) in a.rightOuterJoin(b).collect()
    assert len(a.fullOuterJoin(b).collect()) == 6
    assert sorted(a.subtractByKey(b).collect()) == [(1, "a")]
    g = {k: sorted(v) for k, v in a.groupByKey().collect()}
    assert g == {1: ["a"], 2: ["b", "bb"], 3: ["c"]}
    cg = dict(a.cogroup(b).mapValues(lambda vs: (len(vs[0]), len(vs[1]))).collect())
    assert cg[3] == (1, 2) and cg[4] == (0, 1)
    assert sorted(a.aggregateByKey(0, lambda acc, v: acc + len(v), lambda x, y: x + y).collect()) == \
        [(1, 1), (2, 3), (3, 1)]
    assert sorted(a.foldByKey("", lambda x, y: x + y).collect())[1][1] in ("bbb", "bbb")
    assert sorted(sc.parallelize([3, 1, 3, 2, 1]).distinct().collect()) == [1, 2, 3]
    assert sorted(sc.parallelize([1, 2, 3, 4]).intersection(sc.parallelize([3, 4, 5])).collect()) == [3, 4]
    assert sorted(sc.parallelize([1, 2, 3, 4]).subtract(sc.parallelize([3, 4, 5])).collect()) == [1, 2]
    assert a.lookup(2) == ["b", "bb"]
    assert a.partitionBy(4).getNumPartitions() == 4


def test_sorting_and_repartition(sc):
    import random
    data = [random.Random(3).randint(0, 1000) for _ in range(500)]
    r = sc.parallelize(data, 5)
    assert r.sortBy(lambda x: x).collect() == sorted(data)
    assert r.sortBy(lambda x: x, ascending=False, numPartitions=3).collect() == sorted(data, reverse=True)
    kv = r.map(lambda x: (x % 17, x))
    assert [k for k, _ in kv.sortByKey().collect()] == sorted(x % 17 for x in data)
    rp = r.repartition(7)
    assert rp.getNumPartitions() == 7 and sorted(rp.collect()) == sorted(data)
    assert sorted(r.coalesce(2).collect()) == sorted(data)
    assert sorted(r.union(r).collect()) == sorted(data + data)
    assert len(sc.parallelize([1, 2]).cartesian(sc.parallelize("ab")).collect()) == 4
    s1, s2 = r.randomSplit([0.3, 0.7], seed=4)
    assert s1.count() + s2.count() == 500
    assert 0 < r.sample(False, 0.2, seed=1).count() < 200


def test_shared_variables_and_files(sc, tmp_path):
    bc = sc.broadcast({"k": 3})
    assert sc.range(4).map(lambda x: x * bc.value["k"]).collect() == [0, 3, 6, 9]
    acc = sc.accumulator(0)
    sc.range(10).foreach(lambda x: acc.add(x))
    assert acc.value == 45
    lacc = sc.accumulator([])
    sc.parallelize(["x", "y"]).foreach(lambda v: lacc.add([v]))
    assert sorted(lacc.value) == ["x", "y"]
    out = tmp_path / "txt"
    sc.parallelize(["l1", "l2", "l3"], 2).saveAsTextFile(str(out))
    assert (out / "_SUCCESS").exists()
    assert sorted(sc.textFile(str(out)).collect()) == ["l1", "l2", "l3"]
    assert len(sc.wholeTextFiles(str(out)).collect()) == 2
    sc.parallelize([{"a": 1}, {"a": 2}]).saveAsPickleFile(str(tmp_path / "pk"))
    assert sorted(d["a"] for d in sc.pickleFile(str(tmp_path / "pk")).collect()) == [1, 2]


def test_dataframe_bridge(sc):
    df = sc.parallelize([(1, 2.0, "x"), (2, 3.5, "y"), (3, -1.0, "z")]).toDF(["a", "b", "c"])
    assert df.columns == ["a", "b", "c"] and df.count() == 3
    assert df.rdd.map(lambda row: row.a * row.b).collect() == [2.0, 7.0, -3.0]
    assert sc.session.createDataFrame(sc.parallelize([{"k": 1}, {"k": 5}])).agg({"k": "sum"}).collect()[0][0] == 6
    assert sc.sql is not None        # falls through to the session


def test_portable_hash_is_process_independent():
    import subprocess
    import sys
    code = ("from orange3_spark_amd.rdd import portable_hash; "
            "print(portable_hash(('key', 3, 2.5, None, b'x')), portable_hash('word'))")
    outs = {subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           env={**os.environ, "PYTHONHASHSEED": str(seed)}).stdout for seed in (1, 2)}
    assert len(outs) == 1
    assert portable_hash(1) == portable_hash(1.0)


# ------------------------------------------------------------------ 2-rank invariance
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rdd_work(rank, world, port, out):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), PYTHONHASHSEED=str(rank + 11))
    from orange3_spark_amd import Session, SessionConf
    s = Session(SessionConf().set("o3s.device", "cpu").set("spark.master", "spmd" if world > 1 else "local"))
    sc = s.sparkContext
    words = [f"w{(i * 7) % 23}" for i in range(400)]
    r = sc.parallelize(words, 5)
    res = {
        "wc": sorted(r.map(lambda w: (w, 1)).reduceByKey(lambda a, b: a + b).collect()),
        "group": sorted((k, sorted(v)) for k, v in r.map(lambda w: (w[:2], w)).groupByKey(3).collect()),
        "sorted": r.sortBy(lambda w: (len(w), w)).collect(),
        "distinct": sorted(r.distinct().collect()),
        "zip": r.zipWithIndex().collect()[:50],
        "join": sorted(r.map(lambda w: (w, 1)).distinct().join(sc.parallelize([("w3", "x"), ("w5", "y")])).collect()),
        "count": r.count(),
        "stats": sc.range(1000, numSlices=7).stats().asDict(),
        "take": r.take(5),
        "repart": sorted(r.repartition(4).collect()),
    }
    acc = sc.accumulator(0)
    r.foreach(lambda w: acc.add(1))
    res["acc"] = acc.value
    df = r.map(lambda w: (w, len(w))).toDF(["w", "n"])
    res["df_sum"] = df.agg({"n": "sum"}).collect()[0][0]
    res["df_count"] = df.count()
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


def test_rdd_world_size_invariance(tmp_path):
    _rdd_work(0, 1, _free_port(), str(tmp_path / "w1.json"))
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rdd_work, args=(r, 2, port, str(tmp_path / "w2.json"))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    a = json.load(open(tmp_path / "w1.json"))
    b = json.load(open(tmp_path / "w2.json"))
    for k in a:
        if k == "stats":
            for kk in a[k]:
                assert a[k][kk] == pytest.approx(b[k][kk], rel=1e-12), kk
        else:
            assert a[k] == b[k], k


def test_script_widget_sc_is_spark_context():
    from orangecontrib.spark_amd.widgets.data.owscript import OWScript
    from orangecontrib.spark_amd.widgets.base import SharedSession
    s = Session(SessionConf().set("o3s.device", "cpu"))
    SharedSession._session = s
    w = OWScript()
    w.current_script = lambda: "out_object = sc.parallelize(range(10)).map(lambda x: x * x).sum()"
    w.commit()
    assert w.out_object == 285, w.console_output
