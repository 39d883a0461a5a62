"""spark-bagging on MI355X: the bagging hot path of spark-ensemble
(BaggingRegressor / BaggingClassifier fit + transform with a DecisionTree base
learner) as HIP kernels for gfx950 behind a C ABI (include/sbag.h).

The directory name is not a Python identifier; import it with
`sbag_loader.load()` (repo root), which registers it as `spark_bagging_amd`.
"""
from . import _native  # noqa: F401
from ._native import (Context, DeviceDataset, NativeForest, IllegalArgumentException,  # noqa: F401
                      SparkException, SbagError, default_context, device_count)
from .libsvm import SparseRows, load_libsvm  # noqa: F401
from .ml import (BaggingClassificationModel, BaggingClassifier, BaggingRegressionModel,  # noqa: F401
                 BaggingRegressor, DecisionTreeClassifier, DecisionTreeModel,
                 DecisionTreeRegressor, Frame, even_partitions, java_string_hash)
from .gbm import (GBMClassificationModel, GBMClassifier, GBMRegressionModel,  # noqa: F401
                  GBMRegressor)
