"""LibSVM reader with Spark's `spark.read.format("libsvm")` semantics.

The reference tests load their workloads this way
(core/src/test/scala/org/apache/spark/ml/regression/BaggingRegressorSuite.scala:12,
 core/src/test/scala/org/apache/spark/ml/classification/BaggingClassifierSuite.scala:12):
1-based feature indices in ascending order, numFeatures = max index, missing entries
are 0.0, values parsed with Java's Double.parseDouble (correctly rounded, as Python
float()).  Spark's reader yields SparseVector rows; `sparse=True` keeps them sparse
(SparseRows, CSR), which the engine ingests without a dense copy
(sbag_dataset_create_csr).
"""
import numpy as np


class SparseRows:
    """SparseVector rows in CSR form: indptr [N+1], indices / values [nnz] (indices
    strictly increasing within a row), shape (N, numFeatures).  Duck-compatible with
    scipy.sparse.csr_matrix (indptr / indices / data / shape)."""

    def __init__(self, indptr, indices, values, shape):
        self.indptr = np.ascontiguousarray(indptr, np.int64)
        self.indices = np.ascontiguousarray(indices, np.int32)
        self.data = np.ascontiguousarray(values, np.float64)
        self.shape = (int(shape[0]), int(shape[1]))

    @property
    def values(self):
        return self.data

    def toarray(self):
        X = np.zeros(self.shape, np.float64)
        rows = np.repeat(np.arange(self.shape[0]), np.diff(self.indptr))
        X[rows, self.indices] = self.data
        return X

    def __getitem__(self, rows):
        """Row selection (an index array or a slice) -> SparseRows."""
        idx = np.arange(self.shape[0])[rows]
        starts, ends = self.indptr[idx], self.indptr[idx + 1]
        lens = ends - starts
        indptr = np.concatenate([[0], np.cumsum(lens)])
        take = np.concatenate([np.arange(a, b) for a, b in zip(starts, ends)]) if len(idx) else \
            np.zeros(0, np.int64)
        return SparseRows(indptr, self.indices[take], self.data[take], (len(idx), self.shape[1]))


def is_sparse(X):
    return hasattr(X, "indptr") and hasattr(X, "indices") and hasattr(X, "shape")


def load_libsvm(path, num_features=None, sparse=False):
    labels, indptr, indices, values = [], [0], [], []
    max_idx = 0
    with open(path) as fh:
        for line in fh:
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            parts = line.split()
            labels.append(float(parts[0]))
            prev = 0
            for tok in parts[1:]:
                i, v = tok.split(":")
                i = int(i)
                if i < 1:
                    raise ValueError("libsvm indices are 1-based")
                if i <= prev:
                    raise ValueError("libsvm indices must be in ascending order")
                prev = i
                indices.append(i - 1)
                values.append(float(v))
                max_idx = max(max_idx, i)
            indptr.append(len(indices))
    F = num_features if num_features is not None else max_idx
    rows = SparseRows(indptr, indices, values, (len(labels), F))
    y = np.asarray(labels, np.float64)
    return (rows, y) if sparse else (rows.toarray(), y)
