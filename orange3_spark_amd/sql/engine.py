"""SQL execution over catalog tables / temp views (``session.sql``)."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from ..frame import column as C
from ..frame import expr as E
from ..frame.dataframe import DataFrame
from .parser import AggCall, Select, _AggExpr, _as_agg_expr, parse


def _strings_df(session, data: dict) -> DataFrame:
    cols = OrderedDict((k, C.StringColumn(np.array(v, dtype=object)) if not isinstance(v, C.Column) else v)
                       for k, v in data.items())
    local = DataFrame(session.local_view(), cols)
    return DataFrame(session, OrderedDict(), 0)._from_full(local._cols) if session.comm.world_size > 1 else \
        DataFrame(session, cols)


def execute(session, query: str) -> DataFrame:
    stmt = parse(query)
    kind = stmt[0]
    cat = session.catalog
    if kind == "show_databases":
        return _strings_df(session, {"databaseName": cat.databaseNames()})
    if kind == "show_tables":
        db = stmt[1] or cat.currentDatabase()
        names = cat.tableNames(db)
        return _strings_df(session, {"namespace": [db] * len(names), "tableName": names,
                                     "isTemporary": ["true" if n in cat._temp else "false" for n in names]})
    if kind == "use":
        cat.setCurrentDatabase(stmt[1])
        return session.emptyDataFrame()
    if kind == "create_database":
        cat.createDatabase(stmt[1], ifNotExists=True)
        return session.emptyDataFrame()
    if kind == "drop_table":
        if cat.tableExists(stmt[1]) or not stmt[2]:
            if stmt[1] in cat._temp:
                cat.dropTempView(stmt[1])
            else:
                cat.dropTable(stmt[1])
        return session.emptyDataFrame()
    if kind == "drop_database":
        cat.dropDatabase(stmt[1])
        return session.emptyDataFrame()
    if kind == "describe":
        df = cat.table(stmt[1])
        return _strings_df(session, {"col_name": df.columns, "data_type": [t for _, t in df.dtypes],
                                     "comment": [None] * len(df.columns)})
    if kind == "ctas":
        df = run_select(session, stmt[2])
        cat.saveAsTable(df, stmt[1], "error")
        return session.emptyDataFrame()
    if kind == "create_view":
        # persistent views are kept as session views too (there is no metastore to hold a plan)
        _, name, sel, glob, _replace = stmt
        df = run_select(session, sel)
        if glob:
            df.createOrReplaceGlobalTempView(name)
        else:
            df.createOrReplaceTempView(name)
        return session.emptyDataFrame()
    if kind == "insert":
        return _insert(session, *stmt[1:])
    return run_select(session, stmt[1])


def _insert(session, name, cols, src, overwrite) -> DataFrame:
    """INSERT INTO / OVERWRITE a catalog table, by position (or by the listed columns)."""
    cat = session.catalog
    if name in cat._temp:
        raise ValueError(f"Inserting into the temporary view {name} is not allowed (it has no storage)")
    target = cat.table(name)
    tcols = list(cols) if cols else target.columns
    if src[0] == "values":
        rows = src[1]
        if any(len(r) != len(tcols) for r in rows):
            raise ValueError(f"INSERT VALUES rows must have {len(tcols)} values")
        new = _values_frame(session, rows, tcols)
    else:
        new = run_select(session, src[1])
        if len(new.columns) != len(tcols):
            raise ValueError(f"INSERT source has {len(new.columns)} columns, {name} expects {len(tcols)}")
        new = new.toDF(*tcols)
    missing = [c for c in target.columns if c not in tcols]
    for c in missing:                                    # unlisted columns get NULL
        new = new.withColumn(c, E.lit(None))
    types = dict(target.dtypes)
    new = new.select(*[E.col(c).cast(types[c]).alias(c) if types[c] not in ("string",) else E.col(c)
                       for c in target.columns])
    cat.saveAsTable(new, name, "overwrite" if overwrite else "append")
    return session.emptyDataFrame()


def _values_frame(session, rows, names=None) -> DataFrame:
    """Inline table (VALUES ...): built on rank 0, rows spread like createDataFrame."""
    width = len(rows[0]) if rows else 0
    names = list(names) if names else [f"col{i + 1}" for i in range(width)]
    return session.createDataFrame([tuple(r) for r in rows], names)


def run_select(session, s: Select) -> DataFrame:
    if s.ctes:
        return _with_ctes(session, s)
    if s.values is not None:
        df = _values_frame(session, s.values, s.value_names)
    elif s.subquery is not None:
        df = run_select(session, s.subquery)
    elif s.table is not None:
        df = session.catalog.table(s.table)
    else:
        df = DataFrame(session, OrderedDict(_dummy=C.NumericColumn(_zeros(session))), 1 if session.rank == 0 else 0)
    for j in s.joins:
        right = run_select(session, j.subquery) if j.subquery is not None else session.catalog.table(j.table)
        df = _sql_join(df, right, j, s.alias or (s.table or "").split(".")[-1])
    for lv in s.laterals:
        from . import functions as F
        gen = lv.gen
        if lv.outer and getattr(gen, "_generator", None) in ("explode", "posexplode"):
            gen = (F.explode_outer if gen._generator == "explode" else F.posexplode_outer)(gen)
        names = list(lv.names) or ["col"]
        if getattr(gen, "_generator", "").startswith("posexplode"):
            df = df.select("*", gen)
            df = df.withColumnRenamed("pos", names[0]).withColumnRenamed("col", names[1] if len(names) > 1 else "col")
        else:
            df = df.select("*", gen.alias(names[0]))
    if s.where is not None:
        df = _where(session, df, s)
    has_agg = any(isinstance(it.expr, (AggCall, _AggExpr)) for it in s.items) or s.group_by
    if has_agg:
        df = _aggregate(df, s)
    else:
        sel = []
        for it in s.items:
            if isinstance(it.expr, str) and it.expr == "*":
                sel += [c for c in df.columns if c != "_dummy"]
            else:
                sel.append(it.expr.alias(it.alias) if it.alias else it.expr)
        order_exprs = s.order_by
        from .window import window_refs
        if order_exprs and window_refs([e for e in sel if isinstance(e, E.Expr)]):
            # ORDER BY applies after the window functions (which re-partition rows)
            df = df.select(*sel)
            df = df.orderBy(*[e for e, _ in order_exprs], ascending=[a for _, a in order_exprs])
            sel, order_exprs = None, []
        if order_exprs:
            # order by may reference columns not selected: sort first
            df = df.orderBy(*[e for e, _ in order_exprs], ascending=[a for _, a in order_exprs])
            order_exprs = []
        if sel is not None:
            df = df.select(*sel)
        if s.distinct:
            df = df.distinct()
    if s.order_by and has_agg:
        keys = []
        for e, a in s.order_by:
            if isinstance(e, (AggCall, _AggExpr)):
                keys.append((E.col(_as_agg_expr(e).text), a))
            else:
                keys.append((e, a))
        df = df.orderBy(*[k for k, _ in keys], ascending=[a for _, a in keys])
    if s.offset is not None:
        df = df.offset(s.offset)
    if s.limit is not None:
        df = df.limit(s.limit)
    if s.union is not None:
        other = run_select(session, s.union)
        if len(other.columns) != len(df.columns):
            raise ValueError(f"{s.setop.upper()} needs the same number of columns on both sides")
        other = other.toDF(*df.columns)                 # set operations match columns by position
        if s.setop == "intersect":
            df = df.intersectAll(other) if s.union_all else df.intersect(other)
        elif s.setop == "except":
            df = df.exceptAll(other) if s.union_all else df.subtract(other)
        else:
            df = df.union(other)
            if not s.union_all:
                df = df.distinct()
    return df


def _with_ctes(session, s: Select) -> DataFrame:
    """WITH a AS (...), b AS (...) SELECT ...: each CTE visible (as a view) to the later ones
    and the body only; views of the same names are restored afterwards."""
    import dataclasses
    cat = session.catalog
    saved = {name: cat._temp.get(name) for name, _ in s.ctes}
    try:
        for name, q in s.ctes:
            cat.registerTempView(name, run_select(session, q))
        return run_select(session, dataclasses.replace(s, ctes=[]))
    finally:
        for name, df in saved.items():
            if df is None:
                cat.dropTempView(name)
            else:
                cat.registerTempView(name, df)


def _where(session, df: DataFrame, s: Select) -> DataFrame:
    """WHERE: [NOT] EXISTS conjuncts become left semi / anti joins with the subquery's
    relation on the subquery's WHERE (correlated references resolve to the outer side);
    the remaining conjuncts filter."""
    from ..frame.join import _conjuncts
    from .parser import ExistsExpr
    rest = []
    for c in _conjuncts(s.where):
        if isinstance(c, ExistsExpr) and c.sub.where is not None and not c.sub.group_by \
                and not c.sub.joins and c.sub.table is not None:
            outer_name = s.alias or (s.table or "").split(".")[-1]
            left = df if df.__dict__.get("_aliases") else df.alias(outer_name)
            right = session.catalog.table(c.sub.table).alias(c.sub.alias or c.sub.table.split(".")[-1])
            df = left.join(right, c.sub.where, "left_anti" if c.neg else "left_semi")
        else:
            rest.append(c)
    for c in rest:
        df = df.filter(c)
    return df


def _zeros(session):
    import torch
    return torch.zeros(1 if session.rank == 0 else 0, dtype=torch.int32, device=session.device)


def _sql_join(left: DataFrame, right: DataFrame, j, left_name: str = "") -> DataFrame:
    if j.natural or j.using:
        cols = j.using or [c for c in left.columns if c in set(right.columns)]
        return left.join(right, cols, j.how) if cols else left.join(right, None, "cross")
    if j.how == "cross" or j.on is None:
        # through the condition join so that "a.k" / "b.k" in WHERE and SELECT pick their side
        if not left.__dict__.get("_aliases"):
            left = left.alias(left_name)
        right = right.alias(j.alias or (j.table or "").split(".")[-1])
        return left.join(right, E.lit(True), "inner")
    # support equi-joins "a.x = b.y" (and conjunctions of them)
    keys = _equi_keys(j.on)
    if keys is None:                     # general ON condition: hash keys + residual / nested loop
        if not left.__dict__.get("_aliases"):
            left = left.alias(left_name)
        right = right.alias(j.alias or (j.table or "").split(".")[-1])
        return left.join(right, j.on, j.how)
    lk, rk = zip(*keys)
    if list(lk) == list(rk):
        return left.join(right, list(lk), j.how)
    r2 = right
    for a, b in keys:
        if a != b:
            r2 = r2.withColumnRenamed(b, a)
    return left.join(r2, list(lk), j.how)


def _equi_keys(cond):
    name = getattr(cond, "name", "")
    import re
    parts = [p.strip("() ") for p in re.split(r"\bAND\b", name)]
    out = []
    for p in parts:
        m = re.fullmatch(r"\(?\s*([\w.]+)\s*=\s*([\w.]+)\s*\)?", p)
        if not m:
            return None
        out.append((m.group(1).split(".")[-1], m.group(2).split(".")[-1]))
    return out


def _aggregate(df: DataFrame, s: Select) -> DataFrame:
    keys = list(s.group_by)
    aggs: "OrderedDict[str, AggCall]" = OrderedDict()
    post = []
    for it in s.items:
        if isinstance(it.expr, str) and it.expr == "*":
            raise ValueError("SELECT * with GROUP BY is not supported")
        ae = _as_agg_expr(it.expr) if isinstance(it.expr, (AggCall, _AggExpr)) else None
        if ae is not None:
            for a in ae.aggs:
                aggs[a.text] = a
            post.append((ae, it.alias or ae.text))
        else:
            post.append((it.expr, it.alias or it.expr.name))
    if s.having is not None:
        for a in _as_agg_expr(s.having).aggs:
            aggs[a.text] = a
    for e, _ in s.order_by:
        if isinstance(e, (AggCall, _AggExpr)):
            for a in _as_agg_expr(e).aggs:
                aggs[a.text] = a
    agg_objs = [a.built.alias(a.text) if a.built is not None else E.Agg(a.fn, a.arg, a.text, a.distinct)
                for a in aggs.values()]
    if s.grouping == "rollup":
        g = df.rollup(*keys).agg(*agg_objs)
    elif s.grouping == "cube":
        g = df.cube(*keys).agg(*agg_objs)
    elif s.grouping == "sets":
        from ..frame.grouping_sets import GroupingSets
        g = GroupingSets(df, keys, s.grouping_sets).agg(*agg_objs)
    else:
        g = df.groupBy(*keys).agg(*agg_objs)
    names = {k: k for k in aggs}
    if s.having is not None:
        g = g.filter(_as_agg_expr(s.having).build(names))
    sel = []
    for e, alias in post:
        if isinstance(e, _AggExpr):
            sel.append(e.build(names).alias(alias))
        else:
            sel.append(E.col(e.name).alias(alias) if e.name in g.columns else e.alias(alias))
    extra = [k for k in aggs if k not in {a for _, a in post}]
    out = g.select(*sel, *[E.col(k) for k in extra if s.order_by])
    return out
