"""``spark.udf``: registration of Python UDFs under a name, callable from SQL text.

In the reference, SQL reaches Spark through the Data Frame widget (``hc.sql(query)``,
orangecontrib/spark/widgets/data/spark_sql_dataframe.py:92) and scripts register Python
functions with ``spark.udf.register`` before querying.  Registered UDFs are row-wise host
functions (``sql.functions.udf``) resolved by name (case-insensitive) by the SQL parser,
after the built-in functions.
"""
from __future__ import annotations

import threading

_LOCK = threading.Lock()
_REGISTRY: dict = {}


class UDFRegistration:
    def register(self, name: str, f, returnType=None):
        from .functions import udf
        u = f if hasattr(f, "func") and returnType is None else udf(getattr(f, "func", f), returnType)
        with _LOCK:
            _REGISTRY[name.lower()] = u
        return u

    def registerJavaFunction(self, name, javaClassName, returnType=None):
        raise NotImplementedError("there is no JVM: register a Python function instead")

    def registerJavaUDAF(self, name, javaClassName):
        raise NotImplementedError("there is no JVM: register a Python function instead")


def lookup(name: str):
    with _LOCK:
        return _REGISTRY.get(name.lower())


def unregister(name: str) -> None:
    with _LOCK:
        _REGISTRY.pop(name.lower(), None)
