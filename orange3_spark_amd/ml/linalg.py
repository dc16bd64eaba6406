"""Small host-side vector/matrix types (``pyspark.ml.linalg`` surface).

Model coefficients, cluster centres and per-row vectors returned by ``collect()`` use
these; bulk data stays in device matrices (frame.column.VectorColumn).
"""
from __future__ import annotations

import numpy as np


class Vector:
    def toArray(self) -> np.ndarray:
        raise NotImplementedError

    def __len__(self):
        return self.size

    def norm(self, p):
        return float(np.linalg.norm(self.toArray(), p))

    def dot(self, other):
        o = other.toArray() if isinstance(other, Vector) else np.asarray(other)
        return float(np.dot(self.toArray(), o))

    def squared_distance(self, other):
        o = other.toArray() if isinstance(other, Vector) else np.asarray(other)
        d = self.toArray() - o
        return float(np.dot(d, d))

    def __eq__(self, other):
        if isinstance(other, Vector):
            return self.size == other.size and np.array_equal(self.toArray(), other.toArray())
        return NotImplemented

    def __hash__(self):
        return hash(tuple(self.toArray().tolist()))


class DenseVector(Vector):
    def __init__(self, ar):
        self.array = np.asarray(ar, dtype=np.float64).reshape(-1)

    @property
    def size(self):
        return int(self.array.shape[0])

    @property
    def values(self):
        return self.array

    def toArray(self):
        return self.array

    def numNonzeros(self):
        return int(np.count_nonzero(self.array))

    def __getitem__(self, i):
        return self.array[i]

    def __iter__(self):
        return iter(self.array)

    def __repr__(self):
        return "DenseVector([" + ", ".join(f"{v:.4g}" for v in self.array[:20]) + (", ..." if self.size > 20 else "") + "])"

    def __str__(self):
        return "[" + ",".join(repr(float(v)) for v in self.array) + "]"

    def __reduce__(self):
        return (DenseVector, (self.array.tolist(),))


class SparseVector(Vector):
    def __init__(self, size, *args):
        self._size = int(size)
        if len(args) == 1:
            a = args[0]
            items = sorted(a.items()) if isinstance(a, dict) else sorted(a)
            self.indices = np.array([i for i, _ in items], dtype=np.int32)
            self.values = np.array([v for _, v in items], dtype=np.float64)
        else:
            self.indices = np.asarray(args[0], dtype=np.int32)
            self.values = np.asarray(args[1], dtype=np.float64)

    @property
    def size(self):
        return self._size

    def toArray(self):
        a = np.zeros(self._size, dtype=np.float64)
        a[self.indices] = self.values
        return a

    def numNonzeros(self):
        return int(np.count_nonzero(self.values))

    def __getitem__(self, i):
        hit = np.nonzero(self.indices == i)[0]
        return float(self.values[hit[0]]) if hit.size else 0.0

    def __repr__(self):
        return f"SparseVector({self._size}, {{" + ", ".join(f"{i}: {v:.4g}" for i, v in zip(self.indices, self.values)) + "})"

    def __reduce__(self):
        return (SparseVector, (self._size, self.indices.tolist(), self.values.tolist()))


class Vectors:
    @staticmethod
    def dense(*elements):
        if len(elements) == 1 and not isinstance(elements[0], (int, float)):
            return DenseVector(elements[0])
        return DenseVector(list(elements))

    @staticmethod
    def sparse(size, *args):
        return SparseVector(size, *args)

    @staticmethod
    def zeros(size):
        return DenseVector(np.zeros(size))

    @staticmethod
    def squared_distance(v1, v2):
        return DenseVector(np.asarray(v1.toArray() if hasattr(v1, "toArray") else v1)).squared_distance(v2)

    @staticmethod
    def norm(v, p):
        return float(np.linalg.norm(v.toArray() if hasattr(v, "toArray") else np.asarray(v), p))


class Matrix:
    def toArray(self):
        raise NotImplementedError


class DenseMatrix(Matrix):
    """Column-major like Spark (``values`` are column-major unless isTransposed)."""

    def __init__(self, numRows, numCols, values, isTransposed=False):
        self.numRows, self.numCols = int(numRows), int(numCols)
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)
        self.isTransposed = bool(isTransposed)

    @staticmethod
    def from_array(a: np.ndarray) -> "DenseMatrix":
        a = np.asarray(a, dtype=np.float64)
        return DenseMatrix(a.shape[0], a.shape[1], a.reshape(-1, order="F"))

    def toArray(self):
        if self.isTransposed:
            return self.values.reshape(self.numRows, self.numCols)
        return self.values.reshape(self.numCols, self.numRows).T

    def __repr__(self):
        return f"DenseMatrix({self.numRows}, {self.numCols}, ...)"

    def __reduce__(self):
        return (DenseMatrix, (self.numRows, self.numCols, self.values.tolist(), self.isTransposed))

    def toSparse(self) -> "SparseMatrix":
        return SparseMatrix.from_array(self.toArray())

    def __eq__(self, other):
        return isinstance(other, Matrix) and np.array_equal(self.toArray(), other.toArray())


class SparseMatrix(Matrix):
    """Compressed sparse column matrix in Spark's layout (``colPtrs`` of length numCols+1,
    ``rowIndices`` / ``values`` per stored entry; with ``isTransposed`` the arrays are CSR
    of the matrix, i.e. CSC of its transpose -- pyspark.ml.linalg.SparseMatrix)."""

    def __init__(self, numRows, numCols, colPtrs, rowIndices, values, isTransposed=False):
        self.numRows, self.numCols = int(numRows), int(numCols)
        self.colPtrs = np.asarray(colPtrs, dtype=np.int32).reshape(-1)
        self.rowIndices = np.asarray(rowIndices, dtype=np.int32).reshape(-1)
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)
        self.isTransposed = bool(isTransposed)
        major = self.numRows if self.isTransposed else self.numCols
        if self.colPtrs.size != major + 1:
            raise ValueError(f"expected {major + 1} colPtrs, got {self.colPtrs.size}")
        if self.rowIndices.size != self.values.size or self.colPtrs[-1] != self.values.size:
            raise ValueError("rowIndices / values / colPtrs[-1] sizes differ")

    @staticmethod
    def from_array(a: np.ndarray) -> "SparseMatrix":
        a = np.asarray(a, dtype=np.float64)
        r, c = np.nonzero(a.T)                     # column-major order of the nonzeros
        ptr = np.zeros(a.shape[1] + 1, dtype=np.int32)
        np.add.at(ptr, r + 1, 1)
        return SparseMatrix(a.shape[0], a.shape[1], np.cumsum(ptr), c, a.T[r, c])

    def toArray(self):
        minor = self.numCols if self.isTransposed else self.numRows
        major = self.numRows if self.isTransposed else self.numCols
        out = np.zeros((major, minor), dtype=np.float64)
        seg = np.repeat(np.arange(major), np.diff(self.colPtrs))
        out[seg, self.rowIndices] = self.values
        return out if self.isTransposed else out.T

    def toDense(self) -> DenseMatrix:
        return DenseMatrix.from_array(self.toArray())

    def __eq__(self, other):
        return isinstance(other, Matrix) and np.array_equal(self.toArray(), other.toArray())

    def __repr__(self):
        return f"SparseMatrix({self.numRows}, {self.numCols}, nnz={self.values.size})"

    def __reduce__(self):
        return (SparseMatrix, (self.numRows, self.numCols, self.colPtrs.tolist(), self.rowIndices.tolist(),
                               self.values.tolist(), self.isTransposed))


class Matrices:
    @staticmethod
    def dense(numRows, numCols, values):
        return DenseMatrix(numRows, numCols, values)

    @staticmethod
    def sparse(numRows, numCols, colPtrs, rowIndices, values):
        return SparseMatrix(numRows, numCols, colPtrs, rowIndices, values)
