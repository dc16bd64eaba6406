"""Vectorised equi-join (key codes + stable sort + searchsorted) == the row-by-row
reference join, for every join type, with duplicates, nulls, NaN keys, multi-column
and string keys."""
import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.frame import join as J


def _rows(df):
    def norm(v):
        if v is None:
            return "None"
        if isinstance(v, float) and v != v:
            return "nan"
        return repr(v)
    return sorted(tuple(norm(v) for v in r) for r in df.collect())


@pytest.fixture(scope="module")
def s():
    return Session(SessionConf().set("o3s.device", "cpu"))


def _frames(s):
    rng = np.random.default_rng(0)
    a = pd.DataFrame({"k": rng.integers(0, 30, 400).astype(float), "k2": rng.integers(0, 3, 400),
                      "name": rng.choice(["x", "y", None, "z"], 400), "v": rng.normal(size=400)})
    a.loc[::17, "k"] = np.nan
    a.loc[::23, "k"] = None
    b = pd.DataFrame({"k": rng.integers(0, 40, 90).astype(float), "k2": rng.integers(0, 3, 90),
                      "name": rng.choice(["x", "y", "w", None], 90), "w": rng.normal(size=90)})
    b.loc[::11, "k"] = np.nan
    return s.createDataFrame(a), s.createDataFrame(b)


@pytest.mark.parametrize("how", ["inner", "left", "right", "outer", "left_semi", "left_anti"])
@pytest.mark.parametrize("on", [["k"], ["k", "k2"], ["name"], ["name", "k2"]])
def test_vector_join_matches_reference(s, monkeypatch, how, on):
    a, b = _frames(s)
    got = _rows(a.join(b, on, how))
    monkeypatch.setattr(J, "_key_codes", lambda *x: None)
    ref = _rows(a.join(b, on, how))
    assert got == ref


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["inner", "left", "right", "outer", "left_semi", "left_anti"])
def test_gpu_vector_join_matches_reference(monkeypatch, how):
    g = Session(SessionConf().set("o3s.device", "cuda"))
    a, b = _frames(g)
    for on in (["k"], ["k", "k2"], ["name"]):
        got = _rows(a.join(b, on, how))
        with monkeypatch.context() as m:
            m.setattr(J, "_key_codes", lambda *x: None)
            ref = _rows(a.join(b, on, how))
        assert got == ref


@pytest.mark.gpu
def test_gpu_groupby_segmented_matches_cpu():
    """groupBy aggregates by segmented reductions on the device == the CPU result."""
    from orange3_spark_amd.sql import functions as F
    rng = np.random.default_rng(2)
    pdf = pd.DataFrame({"k": rng.integers(0, 50, 20000), "s": rng.choice(["a", "b", None], 20000),
                        "v": rng.normal(size=20000)})
    pdf.loc[::13, "v"] = np.nan
    res = []
    for dev in ("cpu", "cuda"):
        d = Session(SessionConf().set("o3s.device", dev)).createDataFrame(pdf)
        out = d.groupBy("k", "s").agg(F.count("v"), F.sum("v"), F.avg("v"), F.min("v"), F.max("v"),
                                      F.stddev("v"), F.first("v")).collect()
        res.append(sorted(tuple("None" if x is None else ("nan" if isinstance(x, float) and x != x else
                                                          (round(x, 9) if isinstance(x, float) else x))
                                for x in r) for r in out))
    assert res[0] == res[1]
