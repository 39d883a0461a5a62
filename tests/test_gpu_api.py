"""GPU: the Spark-API mirror end to end -- BaggingRegressor / BaggingClassifier
.fit and .transform through libsbag, and the reference suites' only assertion on
models: a save/load round trip keeps the predictions (BaggingRegressorSuite.scala
:60-69, BaggingClassifierSuite.scala:45-52), here through Spark's on-disk layout."""
import os

import numpy as np
import pytest

import oracle
from conftest import DATA

import spark_bagging_amd as sb

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cpusmall():
    return sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))


@pytest.fixture(scope="module")
def vehicle():
    return sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))


def test_regressor_fit_transform_save_load(tmp_path, cpusmall):
    X, y = cpusmall
    est = (sb.BaggingRegressor().setBaseLearner(sb.DecisionTreeRegressor().setMaxDepth(6))
           .setNumBaseLearners(6).setReplacement(True).setSampleRatio(0.8))
    model = est.fit(sb.Frame(X, y))
    pred = model.transform(X)
    seed = oracle.DEFAULT_SEED_REGRESSOR
    counts = oracle.bag(True, 0.8, 0, 6, seed, [0, len(y)], len(y))
    subs = [oracle.subspace(0.8, X.shape[1], seed + i) for i in range(6)]
    orf = oracle.fit(X, y, counts, subs, max_depth=6, max_bins=32)
    np.testing.assert_allclose(pred, oracle.predict(orf, X), rtol=1e-5, atol=0)
    path = str(tmp_path / "reg")
    model.save(path)
    back = sb.BaggingRegressionModel.load(path)
    np.testing.assert_array_equal(back.transform(X), pred)
    rmse = lambda p: float(np.sqrt(np.mean((p - y) ** 2)))  # noqa: E731
    assert rmse(back.transform(X)) == rmse(pred)


def test_classifier_fit_transform_save_load(tmp_path, vehicle):
    X, y = vehicle
    est = (sb.BaggingClassifier().setBaseLearner(sb.DecisionTreeClassifier())
           .setNumBaseLearners(9).setReplacement(True).setSampleRatio(0.7))
    model = est.fit(sb.Frame(X, y))
    pred = model.transform(X)
    seed = oracle.DEFAULT_SEED_CLASSIFIER
    counts = oracle.bag(True, 0.7, 0, 9, seed, [0, len(y)], len(y))
    subs = [oracle.subspace(0.7, X.shape[1], seed + i) for i in range(9)]
    orf = oracle.fit(X, y, counts, subs, max_depth=5, max_bins=32, classification=True)
    assert (pred == oracle.predict(orf, X, classification=True)).all()
    path = str(tmp_path / "cls")
    model.save(path)
    back = sb.BaggingClassificationModel.load(path)
    assert (back.transform(X) == pred).all()


@pytest.mark.parametrize("cls", [False, True])
def test_transform_per_tree_for_sparse_and_device_inputs(cls):
    """transform(per_tree=True) returns (pred, per_tree [L x N]) for SparseVector rows and
    device datasets too, equal to the host-row path."""
    from spark_bagging_amd import _native as nat

    path = os.path.join(DATA, "vehicle.svm" if cls else "cpusmall.svm")
    dense = sb.Frame.from_libsvm(path, sparse=False)
    sparse = sb.Frame.from_libsvm(path, sparse=True)
    est = (sb.BaggingClassifier().setBaseLearner(sb.DecisionTreeClassifier()) if cls else
           sb.BaggingRegressor().setBaseLearner(sb.DecisionTreeRegressor())).setNumBaseLearners(5)
    est = est.setReplacement(True).setSampleRatio(0.8)
    model = est.fit(dense)
    want, want_pt = model.transform(dense.features, per_tree=True)
    got, got_pt = model.transform(sparse, per_tree=True)
    assert got_pt.shape == (5, dense.num_rows)
    np.testing.assert_array_equal(got_pt, want_pt)
    np.testing.assert_array_equal(got, want)
    ds = nat.DeviceDataset.from_numpy(dense.features, dense.label, sb.default_context(0))
    try:
        got, got_pt = model.transform(ds, per_tree=True)
    finally:
        ds.free()
    np.testing.assert_array_equal(got_pt, want_pt)
    np.testing.assert_array_equal(got, want)
