"""SparkSQL surface beyond single SELECTs (the "Data Frame" widget runs arbitrary
``hc.sql(query)``, reference orangecontrib/spark/widgets/data/spark_sql_dataframe.py:83-94):
CTEs, IN / EXISTS / scalar subqueries (correlated EXISTS as semi / anti joins), INTERSECT /
EXCEPT [ALL], comma joins with qualified WHERE, JOIN USING / NATURAL / SEMI / ANTI, joins
on subqueries, LATERAL VIEW, inline VALUES tables, CREATE VIEW, INSERT INTO / OVERWRITE.
Each checked against a pandas / Python oracle."""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf


@pytest.fixture(scope="module")
def s(tmp_path_factory):
    conf = SessionConf().set("o3s.device", "cpu").set("spark.sql.warehouse.dir",
                                                       str(tmp_path_factory.mktemp("wh")))
    sess = Session(conf)
    sess.createDataFrame(_t()).createOrReplaceTempView("t")
    sess.createDataFrame(_u()).createOrReplaceTempView("u")
    return sess


def _t():
    rng = np.random.default_rng(5)
    return pd.DataFrame({"k": rng.integers(0, 8, 40), "v": rng.normal(size=40).round(6),
                         "g": rng.choice(["a", "b", "c"], 40)})


def _u():
    rng = np.random.default_rng(6)
    return pd.DataFrame({"k": rng.integers(3, 12, 15), "w": rng.normal(size=15).round(6)})


def _rows(df):
    return sorted(tuple(r) for r in df.collect())


def test_cte_chain(s):
    got = _rows(s.sql("WITH a AS (SELECT k, v FROM t WHERE v > 0), b AS (SELECT k, v FROM a WHERE k > 2) "
                      "SELECT k, v FROM b"))
    t = _t()
    assert got == sorted(map(tuple, t[(t.v > 0) & (t.k > 2)][["k", "v"]].itertuples(index=False)))
    with pytest.raises(KeyError):                       # CTE names do not leak out of the statement
        s.sql("SELECT * FROM a").collect()


def test_in_and_scalar_subqueries(s):
    t, u = _t(), _u()
    got = _rows(s.sql("SELECT k, v FROM t WHERE k IN (SELECT k FROM u WHERE w > 0)"))
    keys = set(u[u.w > 0].k)
    assert got == sorted(map(tuple, t[t.k.isin(keys)][["k", "v"]].itertuples(index=False)))
    got = _rows(s.sql("SELECT k FROM t WHERE k NOT IN (SELECT k FROM u)"))
    assert got == sorted((k,) for k in t.k if k not in set(u.k))
    got = s.sql("SELECT k, (SELECT max(w) FROM u) AS mw FROM t WHERE v > 1").collect()
    assert all(r.mw == pytest.approx(u.w.max()) for r in got) and len(got) == int((t.v > 1).sum())
    with pytest.raises(ValueError, match="more than one row"):
        s.sql("SELECT (SELECT k FROM u) AS x FROM t").collect()


def test_correlated_exists(s):
    t, u = _t(), _u()
    got = _rows(s.sql("SELECT k, v FROM t WHERE EXISTS (SELECT 1 FROM u WHERE u.k = t.k AND u.w > 0.2)"))
    ok = {k for k, w in zip(u.k, u.w) if w > 0.2}
    assert got == sorted((k, v) for k, v in zip(t.k, t.v) if k in ok)
    got = _rows(s.sql("SELECT k, v FROM t tt WHERE v < 0 AND NOT EXISTS (SELECT 1 FROM u WHERE u.k = tt.k)"))
    assert got == sorted((k, v) for k, v in zip(t.k, t.v) if v < 0 and k not in set(u.k))


@pytest.mark.parametrize("op,fn", [
    ("INTERSECT", lambda a, b: sorted(set(a) & set(b))),
    ("EXCEPT", lambda a, b: sorted(set(a) - set(b))),
    ("MINUS", lambda a, b: sorted(set(a) - set(b))),
    ("INTERSECT ALL", lambda a, b: sorted((pd.Series(a).value_counts().combine(
        pd.Series(b).value_counts(), min, 0)).pipe(lambda c: [k for k, n in c.items() for _ in range(int(n))]))),
    ("EXCEPT ALL", lambda a, b: sorted((pd.Series(a).value_counts().sub(
        pd.Series(b).value_counts(), fill_value=0)).pipe(lambda c: [k for k, n in c.items() for _ in range(max(int(n), 0))]))),
])
def test_set_operations(s, op, fn):
    t, u = _t(), _u()
    got = [r[0] for r in _rows(s.sql(f"SELECT k FROM t {op} SELECT k FROM u"))]
    assert got == fn(list(t.k), list(u.k))


def test_comma_join_using_natural_semi_anti(s):
    t, u = _t(), _u()
    m = t.merge(u, on="k")
    want = sorted(zip(m.k, m.v, m.w))
    assert _rows(s.sql("SELECT x.k, x.v, y.w FROM t x, u y WHERE x.k = y.k")) == want
    assert _rows(s.sql("SELECT k, v, w FROM t JOIN u USING (k)")) == want
    assert _rows(s.sql("SELECT k, v, w FROM t NATURAL JOIN u")) == want
    semi = _rows(s.sql("SELECT * FROM t LEFT SEMI JOIN u ON t.k = u.k"))
    assert semi == sorted(map(tuple, t[t.k.isin(set(u.k))].itertuples(index=False)))
    anti = _rows(s.sql("SELECT * FROM t LEFT ANTI JOIN u ON t.k = u.k"))
    assert anti == sorted(map(tuple, t[~t.k.isin(set(u.k))].itertuples(index=False)))
    q = _rows(s.sql("SELECT t.k, q.w2 FROM t JOIN (SELECT k, w * 2 AS w2 FROM u) q ON t.k = q.k"))
    assert q == sorted(zip(m.k, (m.w * 2)))


def test_lateral_view_and_values(s):
    got = _rows(s.sql("SELECT k, e FROM t LATERAL VIEW explode(array(k, k + 1)) tt AS e WHERE v > 1"))
    t = _t()
    assert got == sorted((k, e) for k, v in zip(t.k, t.v) if v > 1 for e in (k, k + 1))
    vals = s.sql("SELECT x, y FROM VALUES (1, 'a'), (2, 'b'), (3, NULL) AS tab(x, y) WHERE x > 1").collect()
    assert [tuple(r) for r in vals] == [(2, "b"), (3, None)]


def test_views_and_inserts(s):
    s.sql("CREATE OR REPLACE TEMP VIEW big AS SELECT k, v FROM t WHERE v > 0")
    t = _t()
    assert s.sql("SELECT count(*) AS n FROM big").collect()[0].n == int((t.v > 0).sum())
    s.sql("CREATE TABLE tab_ins AS SELECT k, v, g FROM t WHERE k = 1")
    n0 = int((t.k == 1).sum())
    s.sql("INSERT INTO tab_ins VALUES (99, 1.5, 'z'), (98, -1.5, 'y')")
    s.sql("INSERT INTO TABLE tab_ins SELECT k, w, 'u' FROM u WHERE k = 5")
    n_u = int((_u().k == 5).sum())
    got = s.sql("SELECT k, v, g FROM tab_ins").collect()
    assert len(got) == n0 + 2 + n_u
    assert (99, 1.5, "z") in [tuple(r) for r in got]
    s.sql("INSERT INTO tab_ins (k, g) VALUES (77, 'n')")           # unlisted column -> NULL
    r = [x for x in s.sql("SELECT * FROM tab_ins").collect() if x.k == 77][0]
    assert r.g == "n" and (r.v is None or r.v != r.v)
    s.sql("INSERT OVERWRITE TABLE tab_ins SELECT k, v, g FROM t WHERE k = 2")
    assert s.sql("SELECT count(*) AS n FROM tab_ins").collect()[0].n == int((t.k == 2).sum())
    with pytest.raises(ValueError, match="temporary view"):
        s.sql("INSERT INTO t VALUES (1, 1.0, 'a')")
    s.sql("DROP TABLE tab_ins")


def test_ordinals_aliases_filter_case_nulls(s):
    t = _t()
    got = [tuple(r) for r in s.sql("SELECT g, count(*) FROM t GROUP BY 1 ORDER BY 2 DESC, 1").collect()]
    vc = t.g.value_counts()
    assert got == sorted(((g, int(n)) for g, n in vc.items()), key=lambda x: (-x[1], x[0]))
    got = _rows(s.sql("SELECT k AS key, sum(v) AS sv FROM t GROUP BY key"))
    want = t.groupby("k").v.sum()
    assert [r[0] for r in got] == list(want.index) and np.allclose([r[1] for r in got], want.values)
    r = s.sql("SELECT count(*) FILTER (WHERE v > 0) AS c, sum(v) FILTER (WHERE k < 3) AS sv FROM t").collect()[0]
    assert r.c == int((t.v > 0).sum()) and r.sv == pytest.approx(t.v[t.k < 3].sum())
    got = [r.c for r in s.sql("SELECT CASE k WHEN 1 THEN 'one' WHEN 2 THEN 'two' ELSE 'many' END AS c FROM t")
           .collect()]
    assert got == [{1: "one", 2: "two"}.get(k, "many") for k in t.k]
    s.createDataFrame(pd.DataFrame({"x": [2.0, None, 1.0, None, 3.0]})).createOrReplaceTempView("nl")
    assert [r.x for r in s.sql("SELECT x FROM nl ORDER BY x NULLS LAST").collect()][:3] == [1.0, 2.0, 3.0]
    assert [r.x for r in s.sql("SELECT x FROM nl ORDER BY x DESC NULLS FIRST").collect()][2:] == [3.0, 2.0, 1.0]


def test_sql_functions_and_operators(s):
    t = _t()
    r = s.sql("SELECT k DIV 3 AS d, IF(v > 0, 'p', 'n') AS sgn, nvl(NULL, k) AS nk, nullif(k, 2) AS nn, "
              "array(k, k + 1)[1] AS a1, typeof(v) AS tv FROM t").collect()
    for row, k, v in zip(r, t.k, t.v):
        assert row.d == k // 3 and row.sgn == ("p" if v > 0 else "n") and row.nk == k and row.a1 == k + 1
        assert (row.nn is None) if k == 2 else row.nn == k
        assert row.tv == "double"
    got = _rows(s.sql("SELECT g FROM t WHERE g RLIKE '^[ab]$' AND g NOT ILIKE 'B'"))
    assert got == sorted((g,) for g in t.g if g == "a")
    d = s.sql("SELECT CAST('2024-03-05' AS DATE) AS d").collect()[0].d
    assert str(d).startswith("2024-03-05")


def test_pivot_sample_show_explain_cache(s):
    t = _t()
    out = s.sql("SELECT * FROM (SELECT k, g, v FROM t) PIVOT (sum(v) FOR g IN ('a', 'b' AS bee))").collect()
    p = t.pivot_table(index="k", columns="g", values="v", aggfunc="sum")
    for r in out:
        assert r.a == pytest.approx(p.loc[r.k, "a"]) if not np.isnan(p.loc[r.k, "a"]) else r.a is None
        assert r.bee == pytest.approx(p.loc[r.k, "b"]) if not np.isnan(p.loc[r.k, "b"]) else r.bee is None
    n = s.sql("SELECT count(*) AS n FROM t TABLESAMPLE (50 PERCENT)").collect()[0].n
    assert 0 < n < len(t)
    assert s.sql("SELECT * FROM t TABLESAMPLE (7 ROWS)").count() == 7
    assert [r.col_name for r in s.sql("SHOW COLUMNS FROM t").collect()] == ["k", "v", "g"]
    fns = {r.function for r in s.sql("SHOW FUNCTIONS").collect()}
    assert {"abs", "explode", "nvl", "if"} <= fns
    plan = s.sql("EXPLAIN SELECT g, count(*) FROM t JOIN u ON t.k = u.k WHERE v > 0 GROUP BY g").collect()[0].plan
    assert "BroadcastHashJoin" in plan and "Filter" in plan and "HashAggregate" in plan
    s.sql("CACHE TABLE tc AS SELECT k FROM t WHERE k > 5")
    assert s.catalog.isCached("tc") and s.sql("SELECT count(*) AS n FROM tc").collect()[0].n == int((t.k > 5).sum())
    s.sql("UNCACHE TABLE tc")
    assert not s.catalog.isCached("tc")


def test_bitwise_and_null_safe_operators(s):
    s.createDataFrame(pd.DataFrame({"a": [5, 6, 12], "b": [3.0, None, 10.0]})).createOrReplaceTempView("bt")
    got = [tuple(r) for r in s.sql("SELECT a & 3, a | 1, a ^ 1, ~a, a + 1 & 6, b <=> NULL FROM bt").collect()]
    assert got == [(a & 3, a | 1, a ^ 1, ~a, (a + 1) & 6, b is None) for a, b in ((5, 3.0), (6, None), (12, 10.0))]


def test_set_truncate_rename_drop_view(s):
    s.sql("SET spark.sql.shuffle.partitions=16")
    assert s.conf.get("spark.sql.shuffle.partitions") == "16"
    assert s.sql("SET spark.sql.shuffle.partitions").collect()[0].value == "16"
    assert any(r.key == "spark.sql.shuffle.partitions" for r in s.sql("SET").collect())
    s.sql("RESET spark.sql.shuffle.partitions")
    assert s.conf.get("spark.sql.shuffle.partitions") is None
    s.sql("CREATE TABLE tr1 AS SELECT k, v FROM t WHERE k < 4")
    s.sql("ALTER TABLE tr1 RENAME TO tr2")
    assert s.catalog.tableExists("tr2") and not s.catalog.tableExists("tr1")
    s.sql("TRUNCATE TABLE tr2")
    assert s.sql("SELECT count(*) AS n FROM tr2").collect()[0].n == 0
    assert s.table("tr2").columns == ["k", "v"]
    s.sql("DROP TABLE tr2")
    s.sql("CREATE TEMP VIEW tv1 AS SELECT 1 AS one")
    s.sql("ALTER VIEW tv1 RENAME TO tv2")
    assert s.sql("SELECT one FROM tv2").collect()[0].one == 1
    s.sql("DROP VIEW tv2")
    s.sql("DROP VIEW IF EXISTS tv2")
    with pytest.raises(KeyError):
        s.sql("DROP VIEW tv2")


def test_union_distinct(s):
    t = _t()
    got = _rows(s.sql("SELECT k FROM t UNION DISTINCT SELECT k FROM t"))
    assert got == sorted((k,) for k in set(t.k))
    assert s.sql("SELECT k FROM t UNION ALL SELECT k FROM t").count() == 2 * len(t)


def test_set_operation_chains_are_left_associative(s):
    """A EXCEPT B EXCEPT C == (A EXCEPT B) EXCEPT C; mixed chains evaluate left to right;
    INTERSECT binds tighter; a trailing ORDER BY / LIMIT applies to the combined result
    (pandas/python-set oracle)."""
    import pandas as pd
    s.createDataFrame(pd.DataFrame({"x": [1, 2, 3, 3]})).createOrReplaceTempView("sa")
    s.createDataFrame(pd.DataFrame({"x": [1, 2]})).createOrReplaceTempView("sb")
    s.createDataFrame(pd.DataFrame({"x": [1, 4]})).createOrReplaceTempView("sc")

    def xs(q):
        return sorted(r.x for r in s.sql(q).collect())
    assert xs("SELECT x FROM sa EXCEPT SELECT x FROM sb EXCEPT SELECT x FROM sc") == [3]
    assert xs("SELECT x FROM sa MINUS SELECT x FROM sc") == [2, 3]
    # (A UNION ALL B) UNION C: the final UNION DISTINCT removes A's duplicates too
    assert xs("SELECT x FROM sa UNION ALL SELECT x FROM sb UNION SELECT x FROM sc") == [1, 2, 3, 4]
    # (A UNION B) UNION ALL C keeps C's duplicate of 1
    assert xs("SELECT x FROM sa UNION SELECT x FROM sb UNION ALL SELECT x FROM sc") == [1, 1, 2, 3, 4]
    # A UNION (B INTERSECT C): INTERSECT first
    assert xs("SELECT x FROM sa UNION SELECT x FROM sb INTERSECT SELECT x FROM sc") == [1, 2, 3]
    assert xs("SELECT x FROM sb INTERSECT SELECT x FROM sc UNION SELECT x FROM sa") == [1, 2, 3]
    # parentheses override
    assert xs("SELECT x FROM sa EXCEPT (SELECT x FROM sb EXCEPT SELECT x FROM sc)") == [1, 3]
    # ORDER BY / LIMIT after the last branch order / cut the whole union
    got = [r.x for r in s.sql("SELECT x FROM sa UNION ALL SELECT x FROM sc ORDER BY x DESC LIMIT 3").collect()]
    assert got == [4, 3, 3]
    got = [r.x for r in s.sql("SELECT x FROM sc UNION ALL SELECT x FROM sa ORDER BY x LIMIT 2").collect()]
    assert got == [1, 1]
    assert xs("SELECT x FROM sa INTERSECT ALL SELECT x FROM sa EXCEPT ALL SELECT x FROM sb") == [3, 3]
    # set operation inside a subquery / CTE
    assert xs("SELECT x FROM (SELECT x FROM sa EXCEPT SELECT x FROM sb) q WHERE x > 0") == [3]
    assert xs("WITH q AS (SELECT x FROM sb UNION SELECT x FROM sc) SELECT x FROM q") == [1, 2, 4]
