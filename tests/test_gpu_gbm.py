"""GPU parity of the GBM reuse of the bagging engine.

GBMRegressor (ml/regression/GBMRegressor.scala:196-456) draws its bags with the bagging
sampler and fits one DecisionTreeRegressor per iteration on fp64 pseudo-residuals.  The
booster fit (sbag_fit_booster: the bagging engine with one learner -- screened fp64 splits,
Spark's per-partition row-order sums) must give the oracle's trees bit for bit -- structure, thresholds, impurities,
gains, stats and leaf values -- and the boosted model the oracle's weights, subspaces and
predictions, also bit for bit.  Workload: data/cpusmall (GBMRegressorSuite.scala reads
the same file).
"""
import os

import numpy as np
import pytest

import oracle
from conftest import DATA
from parity_utils import assert_tree_equal

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return sb.default_context(0)


@pytest.fixture(scope="module")
def cpusmall():
    X, y = sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))
    return np.asarray(X, np.float64), y


def _booster_vs_oracle(ctx, X, y_lab, counts, sub, depth=5, bins=32, part=None, min_inst=1,
                       min_gain=0.0):
    ds = nat.DeviceDataset.from_numpy(X, np.zeros(len(X)), ctx)
    try:
        f = nat.fit_booster(ctx, ds, y_lab, counts, sub, partition_offsets=part, max_depth=depth,
                            max_bins=bins, min_instances_per_node=min_inst, min_info_gain=min_gain)
    finally:
        ds.free()
    orf = oracle.fit(X, y_lab, counts[None, :], [sub], max_depth=depth, max_bins=bins,
                     min_instances_per_node=min_inst, min_info_gain=min_gain, part=part)
    assert_tree_equal(f, 0, orf, 0)
    return f, orf


@pytest.mark.parametrize("labels", ["normal", "residual", "signs"])
def test_booster_tree_fp64_labels_bit_exact(ctx, cpusmall, labels):
    """One booster on arbitrary fp64 labels: every node field and stat bit-exact."""
    X, y = cpusmall
    rng = np.random.default_rng(7)
    lab = {"normal": rng.normal(size=len(y)) * 13.7,
           "residual": y - 0.1 * (y - y.mean()) / 3.0,
           "signs": np.sign(rng.normal(size=len(y)))}[labels]
    counts = oracle.bag(True, 1.0, 3, 4, 99, [0, len(y)], len(y))[0]
    sub = oracle.subspace(0.7, X.shape[1], 1234)
    _booster_vs_oracle(ctx, X, lab, counts, sub, depth=6)


@pytest.mark.parametrize("depth,bins,min_inst,min_gain", [(0, 32, 1, 0.0), (3, 2, 1, 0.0),
                                                          (8, 64, 20, 0.0), (5, 16, 1, 5.0)])
def test_booster_params(ctx, cpusmall, depth, bins, min_inst, min_gain):
    X, y = cpusmall
    lab = np.random.default_rng(depth).normal(size=len(y)) + y / 7.0
    counts = oracle.bag(False, 0.6, 0, 1, 5, [0, len(y)], len(y))[0]
    _booster_vs_oracle(ctx, X, lab, counts, np.arange(X.shape[1], dtype=np.int32), depth=depth,
                       bins=bins, min_inst=min_inst, min_gain=min_gain)


def test_booster_sampled_split_finding_partitions(ctx):
    """A subbag above max(maxBins^2, 1e4) rows takes Spark's split-finding sample
    (k_split_sample, 3 partitions); continuous features with repeats and zeros."""
    rng = np.random.default_rng(3)
    n, f = 30_000, 9
    X = np.round(rng.normal(size=(n, f)) * 4) / 4
    X[rng.random((n, f)) < 0.2] = 0.0
    lab = X[:, 0] * 1.3 - X[:, 3] + rng.normal(size=n) / 3
    part = [0, 9_000, 21_000, n]
    counts = oracle.bag(True, 1.0, 0, 1, 11, part, n)[0]
    _booster_vs_oracle(ctx, X, lab, counts, np.arange(f, dtype=np.int32), depth=7, part=part)


def test_booster_large_integer_labels(ctx):
    """Integer labels of ~1e5 at 1.2e5 rows: their sums of squares pass 2^53, so the exact
    integer engine cannot hold them and the fit is redone on the screened fp64 engine
    (sbag_host.cpp fit_range) -- a GBM's first booster sees the raw
    labels.  Bit-exact against the oracle; before, SBAG_EUNSUPPORTED."""
    rng = np.random.default_rng(17)
    n, f = 120_000, 6
    X = np.round(rng.normal(size=(n, f)) * 3) / 3
    lab = np.round(rng.normal(size=n) * 4e4 + 1e5 + X[:, 1] * 2e4)
    assert n * 8 * np.abs(lab).max() ** 2 > 2.0 ** 53
    counts = oracle.bag(True, 1.0, 0, 1, 21, [0, n], n)[0]
    _booster_vs_oracle(ctx, X, lab, counts, np.arange(f, dtype=np.int32), depth=6)


def test_bagging_large_integer_labels(ctx):
    """The same fallback for a bagging regressor (several replicas, P = 2)."""
    rng = np.random.default_rng(23)
    n, f = 100_000, 5
    X = np.round(rng.normal(size=(n, f)) * 2) / 2
    y = np.round(rng.normal(size=n) * 1e5 + 3e5 * (X[:, 0] > 0))
    part = [0, 40_000, n]
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    try:
        forest = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=77, learner_begin=0,
                         learner_end=3, max_depth=5, max_bins=32, partition_offsets=part,
                         impurity=nat.IMPURITY_VARIANCE)
    finally:
        ds.free()
    counts = oracle.bag(True, 1.0, 0, 3, 77, part, n)
    subs = [np.arange(f, dtype=np.int32)] * 3
    orf = oracle.fit(X, y, counts, subs, max_depth=5, max_bins=32, part=part)
    for t in range(3):
        assert_tree_equal(forest, t, orf, t)


@pytest.mark.parametrize("loss,lr,repl,ratio,sratio", [
    ("squared", 0.1, True, 1.0, 0.7),
    ("squared", 1.0, False, 0.8, 1.0),
    ("absolute", 0.5, True, 0.9, 0.5),
    ("huber", 0.3, False, 1.0, 0.8),
    ("quantile", 0.7, True, 1.0, 1.0),
])
def test_gbm_regressor_cpusmall_bit_exact(ctx, cpusmall, loss, lr, repl, ratio, sratio):
    """GBMRegressor.fit through the Spark-API mirror against the oracle's restatement of
    GBMRegressor.train: weights, subspaces, every booster and the predictions bit-exact."""
    X, y = cpusmall
    L = 8
    params = {"numBaseLearners": L, "learningRate": lr, "loss": loss, "replacement": repl,
              "sampleRatio": ratio, "subspaceRatio": sratio}
    est = sb.GBMRegressor().setBaseLearner(sb.DecisionTreeRegressor().setMaxDepth(4))
    model = est.fit(sb.Frame(X, y), params=params)
    w, subs, trees, const = oracle.gbm_regressor_fit(
        X, y, num_base_learners=L, learning_rate=lr, loss=loss, replacement=repl,
        sample_ratio=ratio, subspace_ratio=sratio, max_depth=4)
    assert model.weights == w and model.const == const
    assert len(model.models) == len(trees)
    for m, (sub, (nodes, stats)) in enumerate(zip(subs, trees)):
        assert list(model.subspaces[m]) == list(sub), f"booster {m} subspace"
        mn = model.models[m]
        for k in ("left", "right", "feature", "threshold", "prediction", "impurity", "gain"):
            a, b = mn.nodes[k], nodes[k]
            same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
            assert same.all(), f"booster {m} field {k}"
        assert (mn.stats == stats).all(), f"booster {m} stats"
    np.testing.assert_array_equal(model.transform(X), oracle.gbm_predict(w, subs, trees, const, X))


def test_gbm_validation_early_stopping(ctx, cpusmall, tmp_path):
    """validationIndicatorCol: terminateVal stops after numRound non-improving rounds and
    drops them (GBMRegressor.scala:289, BoostingParams.scala:159-172); save / load keeps the
    predictions (GBMRegressorSuite's assertion)."""
    X, y = cpusmall
    v = np.zeros(len(y), bool)
    v[::4] = True
    est = (sb.GBMRegressor().setBaseLearner(sb.DecisionTreeRegressor().setMaxDepth(3))
           .setNumBaseLearners(40).setLearningRate(0.6).setTol(0.05)
           .setValidationIndicatorCol("validation"))
    model = est.fit(sb.Frame(X, y), params={"numRound": 2, "replacement": True,
                                            "subspaceRatio": 0.7}, validation=v)
    w, subs, trees, const = oracle.gbm_regressor_fit(
        X, y, num_base_learners=40, learning_rate=0.6, tol=0.05, num_round=2, replacement=True,
        subspace_ratio=0.7, max_depth=3, validation=v)
    assert 0 < len(w) < 40
    assert model.weights == w and [list(s) for s in model.subspaces] == [list(s) for s in subs]
    pred = model.transform(X)
    np.testing.assert_array_equal(pred, oracle.gbm_predict(w, subs, trees, const, X))
    path = str(tmp_path / "gbm")
    model.save(path)
    back = sb.GBMRegressionModel.load(path)
    assert back.weights == model.weights and back.const == model.const
    np.testing.assert_array_equal(back.transform(X), pred)
    est.save(str(tmp_path / "est"))
    assert sb.GBMRegressor.load(str(tmp_path / "est")).extractParamMap()["learningRate"] == 0.6


def test_gbm_errors(ctx, cpusmall):
    X, y = cpusmall
    with pytest.raises(sb.SparkException):  # optimizedWeights: breeze LBFGS-B not reproduced
        sb.GBMRegressor().setOptimizedWeights(True).fit((X, y))
    with pytest.raises(sb.IllegalArgumentException):
        sb.GBMRegressor().setLoss("logistic")
    with pytest.raises(sb.IllegalArgumentException):  # an empty subspace
        sb.GBMRegressor().fit((X, y), params={"subspaceRatio": 0.0})
    with pytest.raises(sb.SparkException):  # an empty subbag
        ds = nat.DeviceDataset.from_numpy(X, y, ctx)
        try:
            nat.fit_booster(ctx, ds, y, np.zeros(len(y), np.uint8), np.arange(3, dtype=np.int32))
        finally:
            ds.free()


@pytest.fixture(scope="module")
def vehicle():
    X, y = sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))
    return np.asarray(X, np.float64), y


@pytest.mark.parametrize("lr,repl,ratio,sratio", [(0.5, True, 1.0, 0.7), (1.0, False, 0.8, 1.0)])
def test_gbm_classifier_vehicle_bit_exact(ctx, vehicle, tmp_path, lr, repl, ratio, sratio):
    """GBMClassifier (GBMClassifier.scala:190-482) on vehicle (classes 1-4, class 0 empty):
    per iteration one booster per class on 1{label == k} - softmax_k; every booster, weight
    and subspace bit-exact, probabilities and votes equal to the oracle's; save / load."""
    X, y = vehicle
    L = 6
    est = sb.GBMClassifier().setBaseLearner(sb.DecisionTreeRegressor().setMaxDepth(4))
    model = est.fit(sb.Frame(X, y), params={"numBaseLearners": L, "learningRate": lr,
                                            "replacement": repl, "sampleRatio": ratio,
                                            "subspaceRatio": sratio})
    K, w, subs, trees = oracle.gbm_classifier_fit(X, y, num_base_learners=L, learning_rate=lr,
                                                  replacement=repl, sample_ratio=ratio,
                                                  subspace_ratio=sratio, max_depth=4)
    assert model.numClasses == K == 5
    assert model.weights == w and len(model.models) == len(trees)
    for m in range(len(trees)):
        assert list(model.subspaces[m]) == list(subs[m])
        for k in range(K):
            nodes, stats = trees[m][k]
            mn = model.models[m][k]
            for f in ("left", "right", "feature", "threshold", "prediction", "impurity", "gain"):
                assert (mn.nodes[f] == nodes[f]).all(), f"booster {m} class {k} field {f}"
            assert (mn.stats == stats).all(), f"booster {m} class {k} stats"
    prob, votes = oracle.gbm_classifier_predict(K, w, subs, trees, X)
    np.testing.assert_array_equal(model.predict_raw(X), prob)
    np.testing.assert_array_equal(model.transform(X), votes)
    path = str(tmp_path / "gbmc")
    model.save(path)
    back = sb.GBMClassificationModel.load(path)
    np.testing.assert_array_equal(back.transform(X), votes)


def test_gbm_classifier_validation_quirks(ctx, vehicle):
    """With a validation set the reference's recursion replaces numRound by numTry and keeps
    the seed (GBMClassifier.scala:441-462); the mirror stops where the oracle does."""
    X, y = vehicle
    v = np.zeros(len(y), bool)
    v[1::3] = True
    est = (sb.GBMClassifier().setBaseLearner(sb.DecisionTreeRegressor().setMaxDepth(3))
           .setNumBaseLearners(12).setLearningRate(0.8).setTol(0.02)
           .setValidationIndicatorCol("validation"))
    model = est.fit(sb.Frame(X, y), params={"replacement": True, "subspaceRatio": 0.6},
                    validation=v)
    K, w, subs, trees = oracle.gbm_classifier_fit(X, y, num_base_learners=12, learning_rate=0.8,
                                                  tol=0.02, replacement=True, subspace_ratio=0.6,
                                                  max_depth=3, validation=v)
    assert model.weights == w
    assert len({tuple(s) for s in model.subspaces}) == 1  # the same seed every iteration
    np.testing.assert_array_equal(model.transform(X),
                                  oracle.gbm_classifier_predict(K, w, subs, trees, X)[1])
