"""SQL execution over catalog tables / temp views (``session.sql``)."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from ..frame import column as C
from ..frame import expr as E
from ..frame.dataframe import DataFrame
from .parser import AggCall, Select, SetOp, _AggExpr, _as_agg_expr, parse


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
    if kind == "set":
        _, key, val = stmt
        if key is None:
            pairs = sorted(session.conf.getAll())
            return _strings_df(session, {"key": [k for k, _ in pairs], "value": [str(v) for _, v in pairs]})
        if val is not None:
            session.conf.set(key, val)
        return _strings_df(session, {"key": [key], "value": [str(session.conf.get(key, "<undefined>"))]})
    if kind == "reset":
        if stmt[1] is not None:
            session.conf.remove(stmt[1])
        return session.emptyDataFrame()
    if kind == "truncate":
        name = stmt[1]
        if name in cat._temp:
            raise ValueError(f"TRUNCATE TABLE cannot be used on the temporary view {name}")
        cat.saveAsTable(cat.table(name).limit(0), name, "overwrite")
        return session.emptyDataFrame()
    if kind == "rename":
        _, old, new = stmt
        if old in cat._temp:
            cat.registerTempView(new, cat._temp[old])
            cat.dropTempView(old)
        else:
            df = cat.table(old)
            cat.saveAsTable(df, new, "error")
            cat.dropTable(old)
        return session.emptyDataFrame()
    if kind == "drop_view":
        _, name, if_exists = stmt
        dropped = cat.dropTempView(name) or (name.startswith("global_temp.")
                                             and cat.dropGlobalTempView(name.split(".", 1)[1]))
        if not dropped and not if_exists:
            raise KeyError(f"Table or view not found: {name}")
        return session.emptyDataFrame()
    if kind == "show_columns":
        return _strings_df(session, {"col_name": cat.table(stmt[1]).columns})
    if kind == "show_functions":
        from . import functions as F
        from .parser import _SQL_ONLY
        names = sorted({n for n in dir(F) if not n.startswith("_") and callable(getattr(F, n))
                        and not isinstance(getattr(F, n), type)} | set(_SQL_ONLY))
        return _strings_df(session, {"function": names})
    if kind == "explain":
        return _strings_df(session, {"plan": [_explain(stmt[1], stmt[2])]})
    if kind == "cache":
        _, name, sel, _lazy = stmt
        if sel is not None:
            run_select(session, sel).createOrReplaceTempView(name)
        cat.cacheTable(name)
        return session.emptyDataFrame()
    if kind == "uncache":
        cat.uncacheTable(stmt[1])
        return session.emptyDataFrame()
    if kind == "refresh":
        cat.refreshTable(stmt[1])
        return session.emptyDataFrame()
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


def _explain(stmt, text: str) -> str:
    """Execution outline of a statement (operators are eager device ops, so the 'plan' is the
    order in which they run)."""
    if stmt[0] != "select":
        return f"== Physical Plan ==\nExecute {stmt[0].upper()}: {text}"
    s = stmt[1]
    if isinstance(s, SetOp):
        return (f"== Physical Plan ==\n{s.op.capitalize()}{' All' if s.all else ''} (left: "
                + _explain(("select", s.left), text).splitlines()[1] + ", right: "
                + _explain(("select", s.right), text).splitlines()[1] + ")")
    steps = []
    if s.ctes:
        steps.append("WithCTE " + ", ".join(n for n, _ in s.ctes))
    src = s.table or ("VALUES" if s.values is not None else ("Subquery" if s.subquery is not None else "OneRow"))
    steps.append(f"Scan {src}" + (f" TABLESAMPLE {s.sample}" if s.sample else ""))
    for j in s.joins:
        kind = "BroadcastHashJoin" if (j.using or j.natural or j.on is not None) else "BroadcastNestedLoopJoin"
        steps.append(f"{kind} {j.how} {j.table or 'subquery'}" + (f" ON {j.on.name}" if j.on is not None else ""))
    if s.pivot:
        steps.append(f"Pivot FOR {s.pivot[1]}")
    steps += [f"Generate {lv.gen.name}" for lv in s.laterals]
    if s.where is not None:
        steps.append(f"Filter {s.where.name}")
    if s.group_by or any(isinstance(it.expr, (AggCall, _AggExpr)) for it in s.items):
        steps.append("HashAggregate (device segmented reduction + all-reduce)")
    if s.order_by:
        steps.append("Sort (range exchange + local sort)")
    steps.append("Project " + ", ".join(it.alias or (it.expr if isinstance(it.expr, str) else
                                                      getattr(it.expr, "name", None) or getattr(it.expr, "text", "?"))
                                          for it in s.items))
    if s.limit is not None:
        steps.append(f"Limit {s.limit}")
    return "== Physical Plan ==\n" + "\n".join(("+- " if i else "") + st for i, st in enumerate(steps))


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
    scalar = {"tinyint", "smallint", "int", "bigint", "float", "double", "boolean"}
    new = new.select(*[E.col(c).cast(types[c]).alias(c) if types[c] in scalar else E.col(c)
                       for c in target.columns])                  # numeric targets keep their type
    cat.saveAsTable(new, name, "overwrite" if overwrite else "append")
    return session.emptyDataFrame()


def _values_frame(session, rows, names=None) -> DataFrame:
    """Inline table (VALUES ...): every rank parses the same literal rows and createDataFrame
    keeps this rank's slice, like any local collection."""
    width = len(rows[0]) if rows else 0
    names = list(names) if names else [f"col{i + 1}" for i in range(width)]
    return session.createDataFrame([tuple(r) for r in rows], names)


def run_select(session, s) -> DataFrame:
    if s.ctes:
        return _with_ctes(session, s)
    if isinstance(s, SetOp):
        return _run_setop(session, s)
    if s.values is not None:
        df = _values_frame(session, s.values, s.value_names)
    elif s.subquery is not None:
        df = run_select(session, s.subquery)
    elif s.table is not None:
        df = session.catalog.table(s.table)
        if s.sample is not None:
            unit, n = s.sample
            df = df.sample(fraction=n / 100.0, seed=0) if unit == "percent" else df.limit(int(n))
    else:
        df = DataFrame(session, OrderedDict(_dummy=C.NumericColumn(_zeros(session))), 1 if session.rank == 0 else 0)
    for j in s.joins:
        right = run_select(session, j.subquery) if j.subquery is not None else session.catalog.table(j.table)
        df = _sql_join(df, right, j, s.alias or (s.table or "").split(".")[-1])
    if s.pivot is not None:
        df = _pivot(df, s.pivot)
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
    s = _resolve_ordinals(s)
    has_agg = any(isinstance(it.expr, (AggCall, _AggExpr)) for it in s.items) or s.group_by
    agg_out = None
    if has_agg:
        df = agg_out = _aggregate(df, s)
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
    if has_agg and getattr(agg_out, "_sql_extra", None):
        df = df.drop(*agg_out._sql_extra)
    if s.offset is not None:
        df = df.offset(s.offset)
    if s.limit is not None:
        df = df.limit(s.limit)
    return df


def _run_setop(session, s: SetOp) -> DataFrame:
    """Left-associative set operation (columns matched by position, named by the left
    side); a trailing ORDER BY / LIMIT / OFFSET applies to the combined rows."""
    df = run_select(session, s.left)
    other = run_select(session, s.right)
    if len(other.columns) != len(df.columns):
        raise ValueError(f"{s.op.upper()} needs the same number of columns on both sides")
    other = other.toDF(*df.columns)
    if s.op == "intersect":
        df = df.intersectAll(other) if s.all else df.intersect(other)
    elif s.op == "except":
        df = df.exceptAll(other) if s.all else df.subtract(other)
    else:
        df = df.union(other)
        if not s.all:
            df = df.distinct()
    if s.order_by:
        df = df.orderBy(*[e for e, _ in s.order_by], ascending=[a for _, a in s.order_by])
    if s.offset is not None:
        df = df.offset(s.offset)
    if s.limit is not None:
        df = df.limit(s.limit)
    return df


def _resolve_ordinals(s: Select) -> Select:
    """GROUP BY / ORDER BY <n> (1-based select position) and GROUP BY <select alias>."""
    import dataclasses

    def item(e):
        lit = getattr(e, "_literal", None)
        if isinstance(lit, int) and not isinstance(lit, bool):
            if not 1 <= lit <= len(s.items) or isinstance(s.items[lit - 1].expr, str):
                raise ValueError(f"ordinal {lit} is out of range of the select list")
            return s.items[lit - 1]
        return None

    aliases = {it.alias: it.expr for it in s.items if it.alias and not isinstance(it.expr, str)}
    changed = False
    groups = []
    for g in s.group_by:
        it = item(g)
        if it is not None:
            g, changed = it.expr, True
        elif getattr(g, "_colname", None) in aliases and not isinstance(aliases[g._colname], (AggCall, _AggExpr)):
            g, changed = aliases[g._colname].alias(g._colname), True
        groups.append(g)
    orders = []
    for e, a in s.order_by:
        it = item(e)
        if it is not None:
            e, changed = (E.col(it.alias or it.expr.name) if not isinstance(it.expr, (AggCall, _AggExpr))
                          else it.expr), True
        orders.append((e, a))
    return dataclasses.replace(s, group_by=groups, order_by=orders) if changed else s


def _pivot(df: DataFrame, spec) -> DataFrame:
    """FROM ... PIVOT (agg [AS a], ... FOR col IN (v [AS n], ...)): group by every column not
    pivoted or aggregated; one output column per (value, aggregate)."""
    aggs, col, vals = spec
    used = {col}
    built = []
    for a, alias in aggs:
        ae = _as_agg_expr(a)
        for c in ae.aggs:
            used.update(getattr(c.arg, "refs", ()) or ())
        if len(ae.aggs) != 1 or not isinstance(a, AggCall):
            raise ValueError("PIVOT supports plain aggregate calls")
        c = ae.aggs[0]
        ag = c.built if c.built is not None else E.Agg(c.fn, c.arg, c.text, c.distinct)
        built.append((ag, alias or c.text))
    keys = [c for c in df.columns if c not in used]
    values = [v for v, _ in vals]
    out = df.groupBy(*keys).pivot(col, values).agg(*[ag.alias(n) for ag, n in built])
    ren = {}
    for v, name in vals:
        for ag, n in built:
            src = str(v) if len(built) == 1 else f"{v}_{n}"
            ren[src] = (name or str(v)) if len(built) == 1 else f"{name or v}_{n}"
    for a, b in ren.items():
        if a in out.columns and a != b:
            out = out.withColumnRenamed(a, b)
    return out


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
            if e.name in g.columns:
                sel.append(E.col(e.name).alias(alias))
            elif alias in g.columns:                      # GROUP BY <select alias>
                sel.append(E.col(alias))
            else:
                sel.append(e.alias(alias))
    # aggregates only ORDER BY needs ride along for the sort and are dropped after it
    order_texts = [a.text for e, _ in s.order_by if isinstance(e, (AggCall, _AggExpr))
                   for a in _as_agg_expr(e).aggs]
    extra = [k for k in dict.fromkeys(order_texts) if k not in {a for _, a in post}]
    out = g.select(*sel, *[E.col(k) for k in extra])
    out._sql_extra = extra
    return out
