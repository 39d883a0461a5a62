"""CPU: the GBMRegressor host logic -- params, defaults and validators
(ml/boosting/GBMParams.scala:41-67, ml/regression/GBMRegressor.scala:46-118), the loss and
gradient functions, terminate / terminateVal (GBMParams.scala:308-326,
BoostingParams.scala:150-177) and the on-disk layout of the model's data-$idx rows
(GBMRegressor.scala:538-556).  The GPU fit itself is tested in test_gpu_gbm.py."""
import numpy as np
import pytest

import oracle

import spark_bagging_amd as sb
from spark_bagging_amd import gbm
from spark_bagging_amd import persistence as sp


def test_defaults_and_seed():
    est = sb.GBMRegressor()
    pm = est.extractParamMap()
    assert pm["learningRate"] == 1.0 and pm["numBaseLearners"] == 10 and pm["tol"] == 1e-3
    assert pm["maxIter"] == 10 and pm["optimizedWeights"] is False and pm["loss"] == "squared"
    assert pm["alpha"] == 0.9 and pm["numRound"] == 5
    # HasSeed: "org.apache.spark.ml.regression.GBMRegressor".hashCode
    assert est.getSeed() == sb.java_string_hash("org.apache.spark.ml.regression.GBMRegressor")
    assert est.getSeed() == oracle.DEFAULT_SEED_GBM_REGRESSOR


@pytest.mark.parametrize("name,value", [("learningRate", 0.0), ("numBaseLearners", 0),
                                        ("tol", -1.0), ("numRound", 0), ("loss", "hinge"),
                                        ("sampleRatio", 1.5), ("subspaceRatio", -0.1)])
def test_validators(name, value):
    with pytest.raises(sb.IllegalArgumentException):
        sb.GBMRegressor().set(name, value)


def test_loss_is_case_insensitive():
    assert sb.GBMRegressor().setLoss("HuBeR").getLoss() == "huber"


def test_base_learner_must_be_a_regressor():
    with pytest.raises(sb.IllegalArgumentException):
        sb.GBMRegressor().setBaseLearner(sb.DecisionTreeClassifier())


@pytest.mark.parametrize("loss", gbm.SUPPORTED_LOSSES)
def test_grad_and_loss_match_the_oracle_restatement(loss):
    rng = np.random.default_rng(0)
    y = rng.normal(size=1000) * 10
    p = y + rng.normal(size=1000)
    p[:5] = y[:5]  # zero residuals (signum of +-0.0)
    for a in (0.9, 0.3):
        np.testing.assert_array_equal(gbm.grad_function(loss, a)(y, p), oracle._gbm_grad(loss, a)(y, p))
        np.testing.assert_array_equal(gbm.loss_function(loss, a)(y, p), oracle._gbm_loss(loss, a)(y, p))


def test_absolute_grad_keeps_signed_zero():
    g = gbm.grad_function("absolute", 0.9)(np.array([1.0, 0.0]), np.array([1.0, -0.0]))
    # -Math.signum(+0.0) = -0.0; -Math.signum(0.0 - (-0.0) = +0.0) = -0.0
    assert np.signbit(g).all()


def test_terminate():
    # weight below tol * learningRate: stop and drop that booster
    assert gbm.terminate(1e-5, 1.0, False, 0, 0, 1e-3, 5, 0, 7) == (0, 0.0, 1)
    # no validation: one iteration down
    assert gbm.terminate(0.5, 0.5, False, 3.0, 2.0, 1e-3, 5, 0, 7) == (6, 0.0, 0)
    # validation improved / not improved / out of rounds
    assert gbm.terminate_val(True, 10.0, 9.0, 0.05, 3, 1, 7) == (6, 9.0, 0)
    assert gbm.terminate_val(True, 10.0, 9.8, 0.05, 3, 1, 7) == (6, 10.0, 2)
    assert gbm.terminate_val(True, 10.0, 9.8, 0.05, 3, 2, 7) == (0, 0.0, 3)


def test_seq_sum_is_left_to_right():
    v = np.array([1e16, 1.0, -1e16, 1.0])
    assert gbm.seq_sum(v) == ((1e16 + 1.0) + -1e16) + 1.0


def test_model_data_rows_round_trip(tmp_path):
    row = {"weight": 0.1, "subspace": [0, 2, 5], "const": 0.0}
    sp.write_json_row(str(tmp_path / "data-0"), row)
    assert sp.read_json_row(str(tmp_path / "data-0")) == row


def test_oracle_gbm_small_cpu():
    """The oracle restatement itself: squared loss with learningRate 1 on a one-feature
    set reaches the training labels' leaf means after one booster of unbounded depth."""
    X = np.arange(40, dtype=np.float64)[:, None] % 5
    y = (X[:, 0] * 2.0 + 1.0)
    w, subs, trees, const = oracle.gbm_regressor_fit(X, y, num_base_learners=2, max_depth=5)
    assert w == [1.0, 1.0] and const == 0.0
    np.testing.assert_array_equal(oracle.gbm_predict(w, subs, trees, const, X), y)


def test_classifier_defaults_and_validation():
    est = sb.GBMClassifier()
    assert est.getLoss() == "divergence"
    assert est.getSeed() == oracle.DEFAULT_SEED_GBM_CLASSIFIER
    with pytest.raises(sb.IllegalArgumentException):
        est.setLoss("squared")  # GBMClassifierParams.supportedLossTypes = divergence only
    X = np.zeros((4, 2))
    with pytest.raises(sb.IllegalArgumentException):  # validateLabel: integers in [0, K)
        est.fit((X, np.array([0.0, 1.0, 1.5, 2.0])))


def test_softmax_class_sum_left_to_right():
    res = np.array([[700.0, 0.0, -700.0], [1.0, 2.0, 3.0]])
    e = np.exp(res)
    np.testing.assert_array_equal(gbm.softmax_rows(res), e / (((0.0 + e[:, 0]) + e[:, 1]) + e[:, 2])[:, None])
    np.testing.assert_array_equal(gbm.softmax_rows(res), oracle._softmax_rows(res))
