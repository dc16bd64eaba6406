"""Spark-ML-compatible persistence (``MLWritable`` / ``MLReadable``).

Directory layout written by Spark's ``DefaultParamsWriter`` and model writers, which we
reproduce so saved models interoperate with Spark tooling (beyond-ref: the reference
has no model persistence at all, SURVEY §5 "Checkpoint / resume"):

    <path>/metadata/part-00000     one-line JSON: class, timestamp, sparkVersion, uid,
                                   paramMap, defaultParamMap
    <path>/metadata/_SUCCESS
    <path>/data/part-00000-*.parquet   model data (coefficients, centres, trees, ...)

Model ``data`` schemas follow Spark's (e.g. LogisticRegressionModel: numClasses int,
numFeatures int, interceptVector vector, coefficientMatrix matrix, isMultinomial
boolean).  Vectors/matrices use Spark's VectorUDT/MatrixUDT parquet structs.
"""
from __future__ import annotations

import json
import os
import shutil
import time
import uuid
from typing import Any

import numpy as np

SPARK_VERSION = "3.5.1"

# python class -> JVM class name and back (filled by register())
_PY2JVM: dict[type, str] = {}
_JVM2PY: dict[str, type] = {}


def register(jvm_name: str):
    def deco(cls):
        _PY2JVM[cls] = jvm_name
        _JVM2PY[jvm_name] = cls
        cls._java_class = jvm_name
        return cls
    return deco


def jvm_name(obj_or_cls) -> str:
    cls = obj_or_cls if isinstance(obj_or_cls, type) else type(obj_or_cls)
    return _PY2JVM.get(cls) or f"orange3_spark_amd.{cls.__module__.split('.')[-1]}.{cls.__name__}"


_ML_MODULES = ("feature", "classification", "regression", "clustering", "recommendation", "evaluation", "fpm",
               "tuning", "base")


def py_class(jvm: str) -> type:
    if jvm in _JVM2PY:
        return _JVM2PY[jvm]
    import importlib
    for m in _ML_MODULES:                  # registration happens at import: load every ML module once
        importlib.import_module(f"orange3_spark_amd.ml.{m}")
    if jvm in _JVM2PY:
        return _JVM2PY[jvm]
    # accept our own fallback names
    for cls in _PY2JVM:
        if jvm.endswith("." + cls.__name__):
            return cls
    raise ValueError(f"unknown saved class {jvm}")


def _jsonable(v: Any):
    from .linalg import Matrix, SparseVector, Vector
    # Spark's JsonVectorConverter / JsonMatrixConverter forms
    if isinstance(v, SparseVector):
        return {"type": 0, "size": int(v.size), "indices": np.asarray(v.indices).tolist(),
                "values": np.asarray(v.values).tolist()}
    if isinstance(v, Vector):
        return {"type": 1, "values": np.asarray(v.toArray()).tolist()}
    if isinstance(v, Matrix):
        d = matrix_struct(v)
        if d["type"] == 1:
            d.pop("colPtrs"), d.pop("rowIndices")
        return {"class": "matrix", **d}
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if hasattr(v, "uid"):
        return v.uid
    return str(v)


def _is_rank0() -> bool:
    from ..session import Session
    s = Session.active()
    return s is None or s.comm.rank == 0


def _barrier():
    from ..session import Session
    s = Session.active()
    if s is not None and s.comm.world_size > 1:
        s.comm.barrier()


def prepare_path(path: str, overwrite: bool) -> None:
    if _is_rank0():
        if os.path.exists(path):
            if not overwrite:
                raise FileExistsError(f"Path {path} already exists. To overwrite it, please use write.overwrite().save(path)")
            shutil.rmtree(path)
        os.makedirs(path, exist_ok=True)
    _barrier()


def save_metadata(instance, path: str, extraMetadata: dict | None = None, paramMap: dict | None = None) -> None:
    if not _is_rank0():
        return
    meta = {
        "class": jvm_name(instance),
        "timestamp": int(round(time.time() * 1000)),
        "sparkVersion": SPARK_VERSION,
        "uid": instance.uid,
        "paramMap": paramMap if paramMap is not None else
        {p.name: _jsonable(v) for p, v in instance._paramMap.items()},
        "defaultParamMap": {p.name: _jsonable(v) for p, v in instance._defaultParamMap.items() if v is not None},
    }
    if extraMetadata:
        meta.update(extraMetadata)
    d = os.path.join(path, "metadata")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "part-00000"), "w") as f:
        f.write(json.dumps(meta, separators=(",", ":")) + "\n")
    open(os.path.join(d, "_SUCCESS"), "w").close()


def load_metadata(path: str, expected_class: str | None = None) -> dict:
    d = os.path.join(path, "metadata")
    files = sorted(f for f in os.listdir(d) if f.startswith("part-"))
    with open(os.path.join(d, files[0])) as f:
        meta = json.loads(f.readline())
    if expected_class and meta["class"] != expected_class:
        raise ValueError(f"Error loading metadata: Expected class name {expected_class} but found class name {meta['class']}")
    return meta


def apply_metadata(instance, meta: dict) -> None:
    """Restore uid + param values (skipping params this implementation lacks)."""
    set_uid(instance, meta["uid"])
    for name, v in meta.get("defaultParamMap", {}).items():
        if instance.hasParam(name):
            instance._defaultParamMap[instance.getParam(name)] = _from_json(instance, name, v)
    for name, v in meta.get("paramMap", {}).items():
        if instance.hasParam(name):
            instance._set(**{name: _from_json(instance, name, v)})


def set_uid(instance, uid: str) -> None:
    """Re-key an instance's params to a new uid (Param hashing depends on the parent uid)."""
    defaults = {p.name: v for p, v in instance._defaultParamMap.items()}
    values = {p.name: v for p, v in instance._paramMap.items()}
    instance.uid = uid
    instance._params = None
    instance._copy_params()
    instance._defaultParamMap = {instance.getParam(k): v for k, v in defaults.items()}
    instance._paramMap = {instance.getParam(k): v for k, v in values.items()}


def _from_json(instance, name, v):
    from .linalg import DenseMatrix, DenseVector, SparseVector
    if isinstance(v, dict) and "numRows" in v:
        if v.get("type") == 0:
            return matrix_from_struct(v)
        return DenseMatrix(v["numRows"], v["numCols"], v["values"], v.get("isTransposed", False))
    if isinstance(v, dict) and "values" in v and "type" in v:
        return SparseVector(v["size"], v["indices"], v["values"]) if v["type"] == 0 else DenseVector(v["values"])
    return v


_VEC_FIELDS = ("type", "size", "indices", "values")
_MAT_FIELDS = ("type", "numRows", "numCols", "colPtrs", "rowIndices", "values", "isTransposed")
_SPARK_SCALARS = {"int8": "byte", "int16": "short", "int32": "integer", "int64": "long", "float": "float",
                  "double": "double", "bool": "boolean", "string": "string", "large_string": "string",
                  "binary": "binary"}


def spark_type_json(t):
    """Spark SQL type JSON of an arrow type; VectorUDT / MatrixUDT structs are annotated
    as Spark does in the parquet footer (that is how Spark restores Vector columns)."""
    import pyarrow as pa
    if pa.types.is_struct(t):
        names = tuple(t.field(i).name for i in range(t.num_fields))
        sql = {"type": "struct", "fields": [spark_field_json(t.field(i)) for i in range(t.num_fields)]}
        if names == _VEC_FIELDS:
            return {"type": "udt", "class": "org.apache.spark.ml.linalg.VectorUDT",
                    "pyClass": "pyspark.ml.linalg.VectorUDT", "sqlType": sql}
        if names == _MAT_FIELDS:
            return {"type": "udt", "class": "org.apache.spark.ml.linalg.MatrixUDT",
                    "pyClass": "pyspark.ml.linalg.MatrixUDT", "sqlType": sql}
        return sql
    if pa.types.is_list(t) or pa.types.is_large_list(t):
        return {"type": "array", "elementType": spark_type_json(t.value_type),
                "containsNull": bool(t.value_field.nullable)}
    name = str(t)
    if name in _SPARK_SCALARS:
        return _SPARK_SCALARS[name]
    raise TypeError(f"no Spark SQL type for arrow type {t}")


def prim_list(t):
    """Arrow list type of a Scala primitive array (Array[Int] / Array[Long] /
    Array[Double] / Array[Float]): Spark writes those with non-null elements
    (``containsNull: false``)."""
    import pyarrow as pa
    return pa.list_(pa.field("element", t, False))


def spark_field_json(f) -> dict:
    return {"name": f.name, "type": spark_type_json(f.type), "nullable": bool(f.nullable), "metadata": {}}


def write_table(path: str, table, subdir: str = "data") -> None:
    """One Spark-style parquet part file under ``path/subdir`` (+ ``_SUCCESS``), with the
    footer metadata Spark writes: ``org.apache.spark.sql.parquet.row.metadata`` (the Spark
    schema JSON, including the Vector/Matrix UDT annotations) and the writer version."""
    import pyarrow.parquet as pq
    d = os.path.join(path, subdir)
    os.makedirs(d, exist_ok=True)
    row_meta = json.dumps({"type": "struct", "fields": [spark_field_json(f) for f in table.schema]},
                          separators=(",", ":"))
    table = table.replace_schema_metadata({"org.apache.spark.version": SPARK_VERSION,
                                           "org.apache.spark.sql.parquet.row.metadata": row_meta})
    pq.write_table(table, os.path.join(d, f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"), compression="snappy")
    open(os.path.join(d, "_SUCCESS"), "w").close()


def write_data(path: str, columns, subdir: str = "data", non_null=()) -> None:
    """Write one row-set of model data as a Spark-style parquet part file.  ``non_null``:
    top-level columns Spark declares NOT NULL (primitive case-class fields)."""
    if not _is_rank0():
        return
    import pyarrow as pa
    table = pa.table(columns) if not isinstance(columns, pa.Table) else columns
    if non_null:
        table = table.cast(pa.schema([f.with_nullable(f.name not in non_null) for f in table.schema]))
    write_table(path, table, subdir)


def read_data(path: str, subdir: str = "data"):
    import pyarrow as pa
    import pyarrow.parquet as pq
    d = os.path.join(path, subdir)
    files = sorted(f for f in os.listdir(d) if f.endswith(".parquet"))
    return pa.concat_tables([pq.read_table(os.path.join(d, f)) for f in files])


# ------------------------------------------------------------ VectorUDT / MatrixUDT
def vector_struct(v) -> dict:
    from .linalg import SparseVector
    if isinstance(v, SparseVector):
        return {"type": 0, "size": v.size, "indices": v.indices.tolist(), "values": v.values.tolist()}
    arr = np.asarray(v.toArray() if hasattr(v, "toArray") else v, dtype=np.float64)
    return {"type": 1, "size": None, "indices": None, "values": arr.tolist()}


def vector_from_struct(s):
    from .linalg import DenseVector, SparseVector
    if s["type"] == 0:
        return SparseVector(s["size"], s["indices"], s["values"])
    return DenseVector(s["values"])


def matrix_arrow_type():
    """Spark MatrixUDT sqlType (type 0 = sparse CSC, 1 = dense; values column-major unless
    isTransposed)."""
    import pyarrow as pa
    return pa.struct([pa.field("type", pa.int8(), False), pa.field("numRows", pa.int32(), False),
                      pa.field("numCols", pa.int32(), False), ("colPtrs", pa.list_(pa.field("element", pa.int32(), False))),
                      ("rowIndices", pa.list_(pa.field("element", pa.int32(), False))), ("values", pa.list_(pa.field("element", pa.float64(), False))),
                      pa.field("isTransposed", pa.bool_(), False)])


def matrix_struct(m) -> dict:
    """Matrix in Spark MatrixUDT form (type 1 = dense, column-major values; type 0 =
    sparse CSC with colPtrs / rowIndices)."""
    from .linalg import DenseMatrix, SparseMatrix
    if isinstance(m, SparseMatrix):
        return {"type": 0, "numRows": m.numRows, "numCols": m.numCols, "colPtrs": m.colPtrs.tolist(),
                "rowIndices": m.rowIndices.tolist(), "values": m.values.tolist(), "isTransposed": m.isTransposed}
    if not isinstance(m, DenseMatrix):
        m = DenseMatrix.from_array(np.asarray(m))
    return {"type": 1, "numRows": m.numRows, "numCols": m.numCols, "colPtrs": None, "rowIndices": None,
            "values": m.values.tolist(), "isTransposed": m.isTransposed}


def matrix_from_struct(s):
    from .linalg import DenseMatrix, SparseMatrix
    if s["type"] == 0:
        return SparseMatrix(s["numRows"], s["numCols"], s["colPtrs"], s["rowIndices"], s["values"], s["isTransposed"])
    return DenseMatrix(s["numRows"], s["numCols"], s["values"], s["isTransposed"])


def vec_col(vectors):
    import pyarrow as pa
    from ..io import vector_arrow_type
    return pa.array([vector_struct(v) for v in vectors], type=vector_arrow_type())


def mat_col(mats):
    import pyarrow as pa
    return pa.array([matrix_struct(m) for m in mats], type=matrix_arrow_type())


# --------------------------------------------------------------------- writer API
class MLWriter:
    def __init__(self, instance):
        self.instance = instance
        self.shouldOverwrite = False

    def overwrite(self):
        self.shouldOverwrite = True
        return self

    def session(self, s):
        return self

    def option(self, k, v):
        return self

    def save(self, path: str):
        prepare_path(path, self.shouldOverwrite)
        self.saveImpl(path)
        _barrier()

    def saveImpl(self, path: str):
        inst = self.instance
        save_metadata(inst, path, getattr(inst, "_extra_metadata", lambda: None)())
        if hasattr(inst, "_save_data"):
            inst._save_data(path)


class MLReader:
    def __init__(self, cls):
        self.cls = cls

    def session(self, s):
        return self

    def load(self, path: str):
        from ..session import DriverSession, Session
        s = Session.active()
        if isinstance(s, DriverSession):
            # driver of an executor pool: the executors read the files (a large model --
            # ALS factors -- then stays on them as a RemoteModel handle)
            return s.live_pool.apply(_exec_load, self.cls, os.path.abspath(path))
        meta = load_metadata(path)
        cls = py_class(meta["class"])
        if not issubclass(cls, self.cls) and not issubclass(self.cls, cls):
            raise ValueError(f"{path} holds a {meta['class']}, not a {self.cls.__name__}")
        if hasattr(cls, "_load_impl"):
            return cls._load_impl(path, meta)
        inst = cls()
        apply_metadata(inst, meta)
        return inst


def _exec_load(cls, path):
    return MLReader(cls).load(path)


class MLWritable:
    def write(self) -> MLWriter:
        return MLWriter(self)

    def save(self, path: str) -> None:
        self.write().save(path)


class MLReadable:
    @classmethod
    def read(cls) -> MLReader:
        return MLReader(cls)

    @classmethod
    def load(cls, path: str):
        return cls.read().load(path)


DefaultParamsWritable = MLWritable
DefaultParamsReadable = MLReadable
