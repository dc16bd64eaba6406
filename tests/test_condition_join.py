"""Condition joins (``a.join(b, <Column expression>, how)``) == a row-by-row nested-loop
oracle, for every join type: pure equi conditions (both key columns kept), equi + residual,
non-equi (nested loop), qualified names after ``alias``, ``other[c]`` references resolved in
the result, and SQL ON clauses that are not plain equalities.  Also at world_size 2 (gloo)."""
import math

import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.frame import expr as F
from orange3_spark_amd.frame import join as J


@pytest.fixture(scope="module")
def s():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _pdf():
    rng = np.random.default_rng(3)
    a = pd.DataFrame({"id": rng.integers(0, 12, 60).astype(float), "t": rng.normal(size=60),
                      "tag": rng.choice(["p", "q", None], 60)})
    a.loc[::13, "id"] = None
    b = pd.DataFrame({"uid": rng.integers(0, 15, 25), "t": rng.normal(size=25), "lo": rng.normal(size=25) - 0.5})
    return a, b


def _null(v):
    return v is None or (isinstance(v, float) and math.isnan(v))


def _oracle(a, b, pred, how):
    ar, br = a.to_dict("records"), b.to_dict("records")
    out, hit_r = [], set()
    for i, x in enumerate(ar):
        m = [j for j, y in enumerate(br) if pred(x, y)]
        if how == "left_semi":
            if m:
                out.append(tuple(x.values()))
            continue
        if how == "left_anti":
            if not m:
                out.append(tuple(x.values()))
            continue
        for j in m:
            out.append(tuple(x.values()) + tuple(br[j].values()))
            hit_r.add(j)
        if not m and how in ("left", "outer"):
            out.append(tuple(x.values()) + (None,) * len(b.columns))
    if how in ("right", "outer"):
        for j, y in enumerate(br):
            if j not in hit_r:
                out.append((None,) * len(a.columns) + tuple(y.values()))
    return sorted(tuple("None" if _null(v) else repr(round(v, 9) if isinstance(v, float) else v) for v in r)
                  for r in out)


def _rows(df):
    return sorted(tuple("None" if _null(v) else repr(round(v, 9) if isinstance(v, float) else v) for v in r)
                  for r in df.collect())


def _eq(x, y):
    return not _null(x["id"]) and x["id"] == y["uid"]


CASES = {
    "equi": (lambda a, b: a.id == b.uid, _eq),
    "equi_residual": (lambda a, b: (a.id == b.uid) & (a.t < b["t"]), lambda x, y: _eq(x, y) and x["t"] < y["t"]),
    "non_equi": (lambda a, b: (a.t > b.lo) & (a.t < b.lo + 0.2), lambda x, y: y["lo"] < x["t"] < y["lo"] + 0.2),
    "or": (lambda a, b: (a.id == b.uid) | (a["t"] > b["t"] + 2.0), lambda x, y: _eq(x, y) or x["t"] > y["t"] + 2.0),
}


@pytest.mark.parametrize("how", ["inner", "left", "right", "outer", "left_semi", "left_anti"])
@pytest.mark.parametrize("case", list(CASES))
def test_condition_join_matches_oracle(s, how, case):
    pa, pb = _pdf()
    a, b = s.createDataFrame(pa), s.createDataFrame(pb)
    cond, pred = CASES[case]
    out = a.join(b, cond(a, b), how)
    assert _rows(out) == _oracle(pa, pb, pred, how)
    if how not in ("left_semi", "left_anti"):
        assert out.columns == ["id", "t", "tag", "uid", "t_r", "lo"]


def test_nested_loop_blocks(s, monkeypatch):
    """The nested-loop path walks left rows in blocks; tiny blocks give the same pairs."""
    pa, pb = _pdf()
    a, b = s.createDataFrame(pa), s.createDataFrame(pb)
    want = _rows(a.join(b, a.t < b.lo, "left"))
    monkeypatch.setattr(J, "_PAIR_BLOCK", 7)
    assert _rows(a.join(b, a.t < b.lo, "left")) == want


def test_side_references_in_result(s):
    pa, pb = _pdf()
    a, b = s.createDataFrame(pa), s.createDataFrame(pb)
    j = a.join(b, (a.id == b.uid) & (a.t < b.t))
    # b.t is the renamed right column in the result; a.t the left one
    got = j.select(a.t.alias("x"), b.t.alias("y")).collect()
    ref = j.select("t", "t_r").collect()
    assert [tuple(r) for r in got] == [tuple(r) for r in ref]
    assert j.drop(b.t).columns == ["id", "t", "tag", "uid", "lo"]
    assert j.drop(b.uid).columns == ["id", "t", "tag", "t_r", "lo"]


def test_alias_qualified_and_ambiguity(s):
    pa, pb = _pdf()
    a, b = s.createDataFrame(pa).alias("a"), s.createDataFrame(pb).alias("b")
    out = a.join(b, (F.col("a.id") == F.col("b.uid")) & (F.col("a.t") < F.col("b.t")), "inner")
    want = _oracle(pa, pb, lambda x, y: _eq(x, y) and x["t"] < y["t"], "inner")
    assert _rows(out) == want
    assert len(a.select(F.col("a.t")).collect()) == len(pa)
    with pytest.raises(ValueError, match="ambiguous"):
        a.join(b, F.col("t") > 0.0)


def test_self_join_by_alias(s):
    pa, _ = _pdf()
    d = s.createDataFrame(pa)
    x, y = d.alias("x"), d.alias("y")
    out = x.join(y, (F.col("x.id") == F.col("y.id")) & (F.col("x.t") < F.col("y.t")))
    # pandas NaN ids stay NaN (not null) in the frame, and NaN = NaN in a Spark join key
    want = _oracle(pa, pa, lambda u, v: (u["id"] == v["id"] or (_null(u["id"]) and _null(v["id"])))
                   and u["t"] < v["t"], "inner")
    assert _rows(out) == want


def test_list_of_conditions_and_cross_with_condition(s):
    pa, pb = _pdf()
    a, b = s.createDataFrame(pa), s.createDataFrame(pb)
    l1 = _rows(a.join(b, [a.id == b.uid, a.t < b.t]))
    l2 = _rows(a.join(b, (a.id == b.uid) & (a.t < b.t)))
    assert l1 == l2
    assert _rows(a.join(b, a.t < b.lo, "cross")) == _rows(a.join(b, a.t < b.lo, "inner"))


def test_sql_non_equi_on(s):
    pa, pb = _pdf()
    s.createDataFrame(pa).createOrReplaceTempView("ta")
    s.createDataFrame(pb).createOrReplaceTempView("tb")
    out = s.sql("SELECT a.id, a.t, b.t AS bt FROM ta a JOIN tb b ON a.id = b.uid AND a.t < b.t")
    want = sorted((repr(x["id"]), repr(round(x["t"], 9)), repr(round(y["t"], 9)))
                  for x in pa.to_dict("records") for y in pb.to_dict("records")
                  if _eq(x, y) and x["t"] < y["t"])
    assert _rows(out) == want
    band = s.sql("SELECT * FROM ta JOIN tb ON ta.t BETWEEN tb.lo AND tb.lo + 0.3")
    assert _rows(band) == _oracle(pa, pb, lambda x, y: y["lo"] <= x["t"] <= y["lo"] + 0.3, "inner")


def _dist_worker(rank, world, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    sess = Session(SessionConf().set("o3s.device", "cpu").set("spark.master", "spmd"))
    pa, pb = _pdf()
    a, b = sess.createDataFrame(pa), sess.createDataFrame(pb)
    res = {"n": len(a)}
    for how in ("inner", "left", "right", "outer", "left_anti"):
        res[how] = _local_rows(a.join(b, (a.id == b.uid) & (a.t < b.t + 0.5), how))
    res["nl"] = _local_rows(a.join(b, a.t < b.lo, "outer"))
    q.put((rank, res))


def _local_rows(df):
    """This rank's rows (collect() would gather every rank's)."""
    cols = [df._col(c).to_pylist() for c in df.columns]
    return sorted(tuple("None" if _null(v) else repr(round(v, 9) if isinstance(v, float) else v) for v in r)
                  for r in zip(*cols))


def test_condition_join_world2():
    import multiprocessing as mp
    import socket
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    pa, pb = _pdf()
    assert 0 < got[0]["n"] < len(pa) and got[0]["n"] + got[1]["n"] == len(pa)   # really sharded
    for how in ("inner", "left", "right", "outer", "left_anti"):
        merged = sorted(got[0][how] + got[1][how])
        assert merged == _oracle(pa, pb, lambda x, y: _eq(x, y) and x["t"] < y["t"] + 0.5, how), how
    assert sorted(got[0]["nl"] + got[1]["nl"]) == _oracle(pa, pb, lambda x, y: x["t"] < y["lo"], "outer")


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["inner", "left", "right", "outer", "left_semi", "left_anti"])
def test_gpu_condition_join_matches_oracle(how):
    """Columns on cuda:0: hash keys, residual and nested-loop blocks == the row oracle."""
    g = Session(SessionConf().set("o3s.device", "cuda"))
    pa, pb = _pdf()
    a, b = g.createDataFrame(pa), g.createDataFrame(pb)
    assert a._col("t").data.is_cuda
    for case in CASES:
        cond, pred = CASES[case]
        assert _rows(a.join(b, cond(a, b), how)) == _oracle(pa, pb, pred, how), case


def test_self_join_with_shared_column_objects(s):
    """``df.join(df.withColumn(..), df.id == df2.id)`` and ``x.id == y.id`` after alias: the
    frames share column objects, but each reference names the frame it was taken from, so
    the equality is a join key (not a trivially-true residual -> cross product)."""
    pa = pd.DataFrame({"id": [1.0, 2.0, 3.0, 2.0], "t": [0.1, 0.2, 0.3, 0.4]})
    df = s.createDataFrame(pa)
    df2 = df.withColumn("z", F.col("t") * 2)
    out = df.join(df2, df.id == df2.id)
    want = sum(1 for i in pa.id for j in pa.id if i == j)
    assert out.count() == want == 6
    x, y = df.alias("x"), df.alias("y")
    assert x.join(y, x.id == y.id).count() == 6
    r = x.join(y, (x.id == y.id) & (x.t < y.t)).collect()
    assert len(r) == 1
    # residual predicates also take the side from the frame the reference came from
    assert df.join(df2, (df.id == df2.id) & (df2.z > 0.5)).count() == sum(
        1 for i, _ in pa.itertuples(index=False, name=None) for j, tj in pa.itertuples(index=False, name=None)
        if i == j and tj * 2 > 0.5)


def test_self_join_unresolvable_equality_raises(s):
    pa = pd.DataFrame({"id": [1.0, 2.0], "t": [0.1, 0.2]})
    df = s.createDataFrame(pa)
    other = df.select("t", F.col("id").alias("id2"))
    with pytest.raises((ValueError, KeyError)):
        df.join(other, F.col("id") == F.col("id")).count()
