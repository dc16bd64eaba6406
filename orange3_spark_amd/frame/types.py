"""Spark-SQL-shaped type names and schema objects for the columnar DataFrame.

The reference reaches these through ``pyspark.sql`` (``df.columns``/``df.dtypes`` in
orangecontrib/spark/base/spark_ml_transformer.py:105 and
widgets/ml/spark_ml_dataset.py:422, ``cast('double')`` at spark_ml_dataset.py:578).
Type strings follow Spark's ``simpleString`` so widget code that switches on them
keeps working.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch


class DataType:
    name = "?"

    def simpleString(self) -> str:
        return self.name

    def __repr__(self):
        return type(self).__name__ + "()"

    def __eq__(self, other):
        return type(self) is type(other) and self.simpleString() == other.simpleString()

    def __hash__(self):
        return hash(self.simpleString())

    def typeName(self) -> str:
        return self.name


class NumericType(DataType):
    torch_dtype: torch.dtype = torch.float64


class DoubleType(NumericType):
    name, torch_dtype = "double", torch.float64


class FloatType(NumericType):
    name, torch_dtype = "float", torch.float32


class IntegerType(NumericType):
    name, torch_dtype = "int", torch.int32


class LongType(NumericType):
    name, torch_dtype = "bigint", torch.int64


class ShortType(NumericType):
    name, torch_dtype = "smallint", torch.int16


class ByteType(NumericType):
    name, torch_dtype = "tinyint", torch.int8


class BooleanType(NumericType):
    name, torch_dtype = "boolean", torch.bool


class StringType(DataType):
    name = "string"


class VectorUDT(DataType):
    """ML vector (dense rows of a [n, d] device matrix, or CSR sparse)."""
    name = "vector"


class ArrayType(DataType):
    def __init__(self, elementType: DataType = None, containsNull: bool = True):
        self.elementType = elementType or StringType()
        self.containsNull = containsNull

    def simpleString(self):
        return f"array<{self.elementType.simpleString()}>"

    @property
    def name(self):
        return self.simpleString()

    def __repr__(self):
        return f"ArrayType({self.elementType!r})"


@dataclass
class StructField:
    name: str
    dataType: DataType
    nullable: bool = True
    metadata: dict = field(default_factory=dict)

    def simpleString(self):
        return f"{self.name}:{self.dataType.simpleString()}"


class StructType:
    def __init__(self, fields=None):
        self.fields: list[StructField] = list(fields or [])

    @property
    def names(self):
        return [f.name for f in self.fields]

    def add(self, name, dataType, nullable=True, metadata=None):
        self.fields.append(StructField(name, dataType, nullable, metadata or {}))
        return self

    def __getitem__(self, k):
        if isinstance(k, int):
            return self.fields[k]
        for f in self.fields:
            if f.name == k:
                return f
        raise KeyError(k)

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def simpleString(self):
        return "struct<" + ",".join(f.simpleString() for f in self.fields) + ">"

    def __repr__(self):
        return f"StructType({self.fields!r})"


_BY_NAME = {
    "double": DoubleType, "float": FloatType, "int": IntegerType, "integer": IntegerType,
    "bigint": LongType, "long": LongType, "smallint": ShortType, "short": ShortType,
    "tinyint": ByteType, "byte": ByteType, "boolean": BooleanType, "bool": BooleanType,
    "string": StringType, "str": StringType, "vector": VectorUDT,
}


def parse_type(t) -> DataType:
    if isinstance(t, DataType):
        return t
    if isinstance(t, type) and issubclass(t, DataType):
        return t()
    s = str(t).strip().lower()
    if s.startswith("array<") and s.endswith(">"):
        return ArrayType(parse_type(s[6:-1]))
    if s in _BY_NAME:
        return _BY_NAME[s]()
    raise ValueError(f"unknown data type {t!r}")


def parse_schema(ddl: str) -> StructType:
    """DDL schema string (``"a INT, b string"`` or ``"a: int, b: string"``) -> StructType."""
    st = StructType()
    depth, cur, parts = 0, "", []
    for ch in ddl:                      # split on top-level commas (array<...> may nest)
        depth += (ch == "<") - (ch == ">")
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    for p in parts:
        p = p.strip()
        if not p:
            continue
        name, _, typ = p.replace(":", " ", 1).partition(" ")
        st.add(name.strip().strip("`"), parse_type(typ.strip()))
    return st


def from_torch_dtype(dt: torch.dtype) -> DataType:
    return {
        torch.float64: DoubleType(), torch.float32: FloatType(), torch.float16: FloatType(),
        torch.bfloat16: FloatType(), torch.int64: LongType(), torch.int32: IntegerType(),
        torch.int16: ShortType(), torch.int8: ByteType(), torch.uint8: ShortType(),
        torch.bool: BooleanType(),
    }[dt]


def from_numpy_dtype(dt) -> DataType:
    dt = np.dtype(dt)
    if dt.kind == "f":
        return DoubleType() if dt.itemsize >= 8 else FloatType()
    if dt.kind in "iu":
        return {1: ByteType(), 2: ShortType(), 4: IntegerType()}.get(dt.itemsize, LongType())
    if dt.kind == "b":
        return BooleanType()
    return StringType()
