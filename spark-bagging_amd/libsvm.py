"""LibSVM reader with Spark's `spark.read.format("libsvm")` semantics.

The reference tests load their workloads this way
(core/src/test/scala/org/apache/spark/ml/regression/BaggingRegressorSuite.scala:12,
 core/src/test/scala/org/apache/spark/ml/classification/BaggingClassifierSuite.scala:12):
1-based feature indices, numFeatures = max index, missing entries are 0.0,
values parsed with Java's Double.parseDouble (correctly rounded, as Python float()).
"""
import numpy as np


def load_libsvm(path, num_features=None):
    labels, rows = [], []
    max_idx = 0
    with open(path) as fh:
        for line in fh:
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            parts = line.split()
            labels.append(float(parts[0]))
            entries = []
            for tok in parts[1:]:
                i, v = tok.split(":")
                i = int(i)
                if i < 1:
                    raise ValueError("libsvm indices are 1-based")
                entries.append((i - 1, float(v)))
                max_idx = max(max_idx, i)
            rows.append(entries)
    F = num_features if num_features is not None else max_idx
    X = np.zeros((len(rows), F), np.float64)
    for r, entries in enumerate(rows):
        for i, v in entries:
            X[r, i] = v
    return X, np.asarray(labels, np.float64)
