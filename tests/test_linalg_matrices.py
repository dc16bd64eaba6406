"""pyspark.ml.linalg matrices: SparseMatrix (Spark CSC layout), MatrixUDT parquet structs and
the JSON param forms (JsonVectorConverter / JsonMatrixConverter)."""
import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

from orange3_spark_amd.ml import util as U
from orange3_spark_amd.ml.linalg import DenseMatrix, Matrices, SparseMatrix, SparseVector, Vectors


def test_sparse_matrix_layout_matches_pyspark_doc_example():
    m = Matrices.sparse(3, 2, [0, 1, 3], [0, 2, 1], [9, 6, 8])
    assert np.array_equal(m.toArray(), [[9, 0], [0, 8], [0, 6]])
    t = SparseMatrix(2, 3, [0, 1, 3], [0, 2, 1], [9, 6, 8], isTransposed=True)   # CSR of a 2x3
    assert np.array_equal(t.toArray(), [[9, 0, 0], [0, 8, 6]])
    a = np.array([[1.0, 0, 2], [0, 3, 0]])
    sm = DenseMatrix.from_array(a).toSparse()
    assert sm.colPtrs.tolist() == [0, 1, 2, 3] and sm.rowIndices.tolist() == [0, 1, 0]
    assert sm.toDense() == DenseMatrix.from_array(a) and sm == DenseMatrix.from_array(a)


def test_matrix_udt_parquet_round_trip(tmp_path):
    mats = [Matrices.sparse(3, 2, [0, 1, 3], [0, 2, 1], [9, 6, 8]), DenseMatrix(2, 2, [1, 2, 3, 4])]
    pq.write_table(pa.table({"m": U.mat_col(mats)}), tmp_path / "m.parquet")
    back = [U.matrix_from_struct(r) for r in pq.read_table(tmp_path / "m.parquet").column("m").to_pylist()]
    assert isinstance(back[0], SparseMatrix) and back[0] == mats[0]
    assert isinstance(back[1], DenseMatrix) and np.array_equal(back[1].toArray(), [[1, 3], [2, 4]])


def test_param_json_forms():
    sv = SparseVector(5, [1, 3], [2.0, 4.0])
    assert U._jsonable(sv) == {"type": 0, "size": 5, "indices": [1, 3], "values": [2.0, 4.0]}
    assert U._jsonable(Vectors.dense([1.0, 2.0])) == {"type": 1, "values": [1.0, 2.0]}
    dm = DenseMatrix(1, 2, [1.0, 2.0])
    assert U._jsonable(dm) == {"class": "matrix", "type": 1, "numRows": 1, "numCols": 2, "values": [1.0, 2.0],
                               "isTransposed": False}
    for v in (sv, dm, Matrices.sparse(3, 2, [0, 1, 3], [0, 2, 1], [9, 6, 8])):
        r = U._from_json(None, "p", U._jsonable(v))
        assert np.array_equal(r.toArray(), v.toArray()) and type(r) is type(v)
