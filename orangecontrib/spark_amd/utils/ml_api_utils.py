"""Reflection over the pyspark.ml-compatible modules (the "method" lists of the generic
Estimator/Transformer/Evaluator widgets).

Reference: orangecontrib/spark/utils/ml_api_utils.py:7-83.  Same class predicates
(transform/fit/evaluate present, not abstract, no ``Java`` prefix, transformers exclude
``*Model``, evaluators exclude the ``Evaluator`` base), but introspection never starts a
session or a device (quirk Q9) and uses ``inspect.signature`` (quirk Q15).
"""
from __future__ import annotations

import inspect
from collections import OrderedDict

from orange3_spark_amd.ml.param import Params


def _classes(module):
    return [(n, c) for n, c in inspect.getmembers(module, inspect.isclass)
            if issubclass(c, Params) and not n.startswith(("_", "Java")) and not inspect.isabstract(c)]


def get_models(self=None, module=None):
    return {n: c for n, c in _classes(module) if "transform" in dir(c) and n.endswith("Model")}


def get_evaluators(self=None, module=None):
    return {n: c for n, c in _classes(module) if "evaluate" in dir(c) and n != "Evaluator"}


def get_transformers(self=None, module=None):
    return {n: c for n, c in _classes(module) if "transform" in dir(c) and "fit" not in dir(c)
            and not n.endswith("Model") and n not in ("PipelineModel",)}


def get_estimators(self=None, module=None):
    return {n: c for n, c in _classes(module) if "fit" in dir(c)}


def get_ml_modules():
    from orange3_spark_amd.ml import (classification, clustering, evaluation, feature, fpm, recommendation,
                                      regression, tuning)
    mods = [feature, classification, clustering, recommendation, regression, tuning, evaluation, fpm]
    return {m.__name__: [m, str(inspect.getdoc(m) or "").split(">>>")[0].strip()] for m in mods}


def get_module_info(module):
    return str(inspect.getdoc(module) or "").split(">>>")[0].strip()


def get_object_info(obj, sc=None):
    """(name, doc, OrderedDict param -> [index, default, doc], html) for a class."""
    sig = inspect.signature(obj)
    is_model = "java_model" in sig.parameters
    obj_name = f"{obj.__module__}.{obj.__name__}"
    obj_doc = str(inspect.getdoc(obj) or "").split(">>>")[0].strip()
    parameters = OrderedDict()
    for name, p in sig.parameters.items():
        if p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD):
            continue
        parameters[name] = [len(parameters), None if p.default is inspect.Parameter.empty else p.default]
    html = "<!DOCTYPE html><html><body>"
    html += f"<h4>{obj_name}{sig}</h4><p>{obj_doc}</p>"
    if not is_model:
        html += "<h6> Parameters: </h6><ul>"
        inst = obj()
        by_name = {p.name: p for p in inst.params}
        for name in parameters:
            doc = by_name[name].doc if name in by_name else ""
            parameters[name].append(doc)
            html += f"<li>{name}: {doc}</li>"
        html += "</ul>"
    html += "</body></html>"
    return obj_name, obj_doc, parameters, html


def get_dataframe_function_info(func_name: str) -> str:
    """HTML help for a DataFrame method (FillNa / Sample widgets; reference spark_api_utils.py:13-30)."""
    from orange3_spark_amd.frame.dataframe import DataFrame
    fn = getattr(DataFrame, func_name)
    doc = str(inspect.getdoc(fn) or "")
    return (f"<!DOCTYPE html><html><body><h4>{func_name}{inspect.signature(fn)}</h4><p>{doc}</p>"
            "</body></html>")
