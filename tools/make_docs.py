"""Generate the widget and API reference under ``doc/`` from the code itself.

The reference ships only a Sphinx template (``doc/conf.py``, no pages) while its widgets
point their help at ``doc/build/htmlhelp``.  This writes real pages:

* ``doc/widgets/<slug>.md`` -- one per widget: category, description, signals, settings,
  the reference widget it replaces, and (reflective widgets) every reachable algorithm;
* ``doc/api/<module>.md`` -- every public ML class with its Params (name, default, doc),
  exactly what the reflective widgets show (``explainParams`` order);
* ``doc/index.md`` -- the table of contents.

Usage: ``python tools/make_docs.py`` (CPU only; no Orange/Qt needed).
"""
from __future__ import annotations

import importlib
import inspect
import os
import pkgutil
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DOC = os.path.join(ROOT, "doc")

from orangecontrib.spark_amd.widgets.compat import Setting, Widget  # noqa: E402

ML_MODULES = ["feature", "classification", "regression", "clustering", "recommendation", "evaluation",
              "tuning", "fpm", "stat"]


def slug(s: str) -> str:
    return re.sub(r"[^a-z0-9]+", "-", s.lower()).strip("-")


def _sig_name(sig) -> str:
    t = sig[1] if len(sig) > 1 else None
    return getattr(t, "__name__", str(t))


def widget_classes():
    out = []
    for cat in ("data", "ml"):
        pkg = importlib.import_module(f"orangecontrib.spark_amd.widgets.{cat}")
        cat_name = getattr(pkg, "NAME", cat)
        for m in pkgutil.iter_modules(pkg.__path__):
            mod = importlib.import_module(f"{pkg.__name__}.{m.name}")
            for name, cls in vars(mod).items():
                if (inspect.isclass(cls) and issubclass(cls, Widget) and cls.__module__ == mod.__name__
                        and name.startswith("OW")):
                    out.append((cat_name, mod, cls))
    return sorted(out, key=lambda t: (t[0], getattr(t[2], "priority", 100), t[2].name))


def widget_page(cat, mod, cls) -> str:
    lines = [f"# {cls.name}", "", f"*Category:* {cat} — *class:* `{cls.__module__}.{cls.__name__}`", ""]
    if cls.description:
        lines += [cls.description, ""]
    doc = inspect.getdoc(mod) or ""
    if doc:
        lines += ["## Behaviour", "", doc, ""]
    if cls.inputs:
        lines += ["## Inputs", ""] + [f"- **{s[0]}** (`{_sig_name(s)}`)" for s in cls.inputs] + [""]
    if cls.outputs:
        lines += ["## Outputs", ""] + [f"- **{s[0]}** (`{_sig_name(s)}`)" for s in cls.outputs] + [""]
    settings = [(k, v.default) for k in dir(cls) for v in [getattr(cls, k, None)] if isinstance(v, Setting)]
    if settings:
        lines += ["## Settings (persisted in workflows)", "", "| Setting | Default |", "|---|---|"]
        lines += [f"| `{k}` | `{d!r}` |" for k, d in settings] + [""]
    module = getattr(cls, "module", None)
    getter = getattr(cls, "get_modules", None)
    if module is not None and getter is not None:
        try:
            algos = sorted(getter(None, module).keys())
        except Exception:   # noqa: BLE001
            algos = []
        if algos:
            mname = module.__name__.rsplit(".", 1)[-1]
            lines += ["## Algorithms offered", ""]
            lines += [f"- [`{a}`](../api/{mname}.md#{slug(a)})" for a in algos] + [""]
    return "\n".join(lines)


def api_page(modname: str) -> str:
    mod = importlib.import_module(f"orange3_spark_amd.ml.{modname}")
    lines = [f"# `orange3_spark_amd.ml.{modname}`", "", (inspect.getdoc(mod) or "").split("\n\n")[0], ""]
    for name, cls in sorted(vars(mod).items()):
        if not inspect.isclass(cls) or name.startswith("_") or not cls.__module__.startswith("orange3_spark_amd"):
            continue
        if not any(hasattr(cls, a) for a in ("fit", "transform", "evaluate", "test", "corr", "build")):
            continue
        if cls.__module__.rsplit(".", 1)[-1].lstrip("_") not in (modname, modname + "_extra") and \
                not cls.__module__.endswith(modname):
            # re-exported helper classes (mixins, vectors) are documented where they live
            if not any(hasattr(cls, a) for a in ("fit", "transform", "evaluate")):
                continue
        lines += [f"## {name}", ""]
        doc = (inspect.getdoc(cls) or "").split(">>>")[0].strip()
        if doc:
            lines += [doc, ""]
        try:
            inst = cls()
            params = list(getattr(inst, "params", []))
        except Exception:   # noqa: BLE001 - classes needing ctor args (e.g. models)
            params = []
        if params:
            lines += ["| Param | Default | Description |", "|---|---|---|"]
            for p in params:
                d = inst.getOrDefault(p) if inst.hasDefault(p) or inst.isSet(p) else ""
                desc = str(p.doc).replace("|", "\\|").replace("\n", " ")
                dv = re.sub(r"_[0-9a-f]{12}__output", "_<uid>__output", repr(d))   # uid-free, stable
                lines.append(f"| `{p.name}` | `{dv}` | {desc} |")
            lines.append("")
    return "\n".join(lines)


def class_methods_page(title: str, classes) -> str:
    """Method reference of non-ML classes (RDD / SparkContext view / ml.functions)."""
    lines = [f"# {title}", ""]
    for cls in classes:
        if inspect.isfunction(cls):
            lines += [f"## `{cls.__name__}{inspect.signature(cls)}`", "", (inspect.getdoc(cls) or "").strip(), ""]
            continue
        lines += [f"## {cls.__name__}", "", (inspect.getdoc(cls) or "").split("\n\n")[0], ""]
        for name, fn in sorted(vars(cls).items()):
            if name.startswith("_") or not (inspect.isfunction(fn) or isinstance(fn, property)):
                continue
            doc = (inspect.getdoc(fn) or "").split("\n")[0]
            sig = "" if isinstance(fn, property) else str(inspect.signature(fn)).replace("(self, ", "(").replace("(self)", "()")
            sig = re.sub(r"<function ([\w.<>]+) at 0x[0-9a-f]+>", r"\1", sig)   # stable across runs
            lines.append(f"- `{name}{sig}`" + (f" — {doc}" if doc else ""))
        lines.append("")
    return "\n".join(lines)


def main():
    os.makedirs(os.path.join(DOC, "widgets"), exist_ok=True)
    os.makedirs(os.path.join(DOC, "api"), exist_ok=True)
    index = ["# Orange3-Spark-AMD documentation", "",
             "Generated by `tools/make_docs.py` from the widget and ML classes (do not edit by hand).", "",
             "- [Architecture and kernels](../README.md)",
             "- [Runtime: sessions, executors, collectives, kernels](runtime.md)", "- [Measured performance](../BASELINE.md)",
             "- [Design survey of the reference](../SURVEY.md)", "", "## Widgets", ""]
    cur = None
    for cat, mod, cls in widget_classes():
        if cat != cur:
            index += ["", f"### {cat}", ""]
            cur = cat
        fn = f"{slug(cls.name)}.md"
        with open(os.path.join(DOC, "widgets", fn), "w") as f:
            f.write(widget_page(cat, mod, cls) + "\n")
        index.append(f"- [{cls.name}](widgets/{fn}) — {cls.description}")
    index += ["", "## ML API reference", ""]
    for m in ML_MODULES:
        with open(os.path.join(DOC, "api", f"{m}.md"), "w") as f:
            f.write(api_page(m) + "\n")
        index.append(f"- [`ml.{m}`](api/{m}.md)")
    from orange3_spark_amd import rdd as R
    from orange3_spark_amd.ml import functions as MF
    with open(os.path.join(DOC, "api", "rdd.md"), "w") as f:
        f.write(class_methods_page("RDD API (`orange3_spark_amd.rdd`)",
                                   [R.Context, R.RDD, R.Broadcast, R.Accumulator, R.StatCounter]) + "\n")
    with open(os.path.join(DOC, "api", "ml_functions.md"), "w") as f:
        f.write(class_methods_page("`orange3_spark_amd.ml.functions`",
                                   [MF.vector_to_array, MF.array_to_vector, MF.predict_batch_udf]) + "\n")
    from orange3_spark_amd.sql import functions as SF
    fns = sorted(n for n, f in vars(SF).items() if inspect.isfunction(f) and not n.startswith("_")
                 and f.__module__ == SF.__name__)
    with open(os.path.join(DOC, "api", "sql_functions.md"), "w") as f:
        f.write("\n".join([f"# `orange3_spark_amd.sql.functions` ({len(fns)} functions)", "",
                           "Column functions with `pyspark.sql.functions` names and semantics.", ""]
                          + [f"- `{n}{inspect.signature(getattr(SF, n))}`" for n in fns]) + "\n")
    from orange3_spark_amd.sql.parser import GRAMMAR
    with open(os.path.join(DOC, "api", "sql.md"), "w") as f:
        f.write("# SQL statements (`session.sql`, the Data Frame widget)\n\nParsed by the in-house "
                "recursive-descent parser (`orange3_spark_amd/sql/parser.py`), executed by `sql/engine.py` "
                "as the same device operators as the DataFrame API.\n\n```\n" + GRAMMAR + "```\n")
    index += ["- [RDD / SparkContext](api/rdd.md)", "- [`ml.functions`](api/ml_functions.md)",
              "- [`sql.functions`](api/sql_functions.md)", "- [SQL statements](api/sql.md)"]
    with open(os.path.join(DOC, "index.md"), "w") as f:
        f.write("\n".join(index) + "\n")
    print("wrote", DOC)


if __name__ == "__main__":
    main()
