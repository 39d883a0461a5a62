"""CPU: Spark 2.4.3 on-disk format of the bagging models.

The reference's only assertion on models is a save/load round trip that keeps
the metric (BaggingRegressorSuite.scala:60-69, BaggingClassifierSuite.scala:45-52).
Here the forests come from the CPU oracle (no GPU), are written in Spark's MLWriter
layout (metadata JSON, learner/, model-$i parquet NodeData, data-$i subspace
JSON), read back, and must predict identically.  The layout details are Spark
2.4.3's [verify: no JVM here]; parity with a real Spark reader is unpinned.
"""
import json
import os

import numpy as np
import pyarrow.parquet as pq
import pytest

import oracle
from conftest import DATA

import spark_bagging_amd as sb
from spark_bagging_amd import persistence as sp


def _model(cls, X, y, L, classification, ratio=0.7):
    seed = oracle.DEFAULT_SEED_CLASSIFIER if classification else oracle.DEFAULT_SEED_REGRESSOR
    counts = oracle.bag(True, ratio, 0, L, seed, [0, len(y)], len(y))
    subs = [oracle.subspace(ratio, X.shape[1], seed + i) for i in range(L)]
    orf = oracle.fit(X, y, counts, subs, max_depth=4, max_bins=32, classification=classification)
    imp = sb._native.IMPURITY_GINI if classification else sb._native.IMPURITY_VARIANCE
    models = [sb.DecisionTreeModel(*orf.tree(t), imp) for t in range(L)]
    m = cls(subs, models)
    est = (sb.BaggingClassifier() if classification else sb.BaggingRegressor())
    bl = (sb.DecisionTreeClassifier() if classification else sb.DecisionTreeRegressor()).setMaxDepth(4)
    est.setBaseLearner(bl).setNumBaseLearners(L).setReplacement(True).setSampleRatio(ratio)
    m._copy_params_from(est)
    return m, orf


def _py_predict(m, X, classification):
    votes = np.array([[t.predict(X[i, s]) for i in range(len(X))]
                      for t, s in zip(m.models, m.subspaces)])
    if not classification:
        return votes.sum(axis=0) / len(m.models)
    out = []
    for col in votes.T:  # breeze mode: first value to reach the final max count
        cnt, best, mode = {}, 0, 0.0
        for v in col:
            cnt[v] = cnt.get(v, 0) + 1
            if cnt[v] > best:
                best, mode = cnt[v], v
        out.append(mode)
    return np.array(out)


@pytest.fixture(scope="module")
def cpusmall():
    X, y = sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))
    return X[:1500], y[:1500]


@pytest.fixture(scope="module")
def vehicle():
    return sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))


def test_regression_round_trip_spark_layout(tmp_path, cpusmall):
    X, y = cpusmall
    m, orf = _model(sb.BaggingRegressionModel, X, y, 4, False)
    path = str(tmp_path / "bagging")
    m.save(path)
    for d in ("metadata", "learner/metadata", "model-0/metadata", "model-0/data", "data-0"):
        assert os.path.exists(os.path.join(path, d, "_SUCCESS")), d
    meta = sp.load_metadata(path)
    assert meta["class"] == "org.apache.spark.ml.regression.BaggingRegressionModel"
    assert meta["sparkVersion"] == "2.4.3" and meta["numBaseModels"] == 4
    assert "baseLearner" not in meta["paramMap"]
    assert meta["paramMap"]["numBaseLearners"] == 4 and meta["paramMap"]["replacement"] is True
    assert meta["defaultParamMap"]["seed"] == -1395689524
    lm = sp.load_metadata(os.path.join(path, "learner"))
    assert lm["class"] == sp.DTR_CLASS and lm["paramMap"] == {"maxDepth": 4}
    tm = sp.load_metadata(os.path.join(path, "model-1"))
    assert tm["class"] == sp.DTR_MODEL_CLASS and tm["numFeatures"] == len(m.subspaces[1])
    assert tm["uid"] == lm["uid"]  # trees keep the estimator's uid
    assert {"labelCol", "featuresCol", "predictionCol", "maxDepth"} <= set(tm["paramMap"])

    back = sb.BaggingRegressionModel.load(path)
    assert back.uid == m.uid and back.numBaseModels == 4
    for a, b, sa, sb_ in zip(m.models, back.models, m.subspaces, back.subspaces):
        assert list(sa) == list(sb_)
        for f in ("id", "left", "right", "feature", "prediction", "impurity"):
            assert (a.nodes[f] == b.nodes[f]).all(), f
        internal = a.nodes["left"] >= 0
        assert (a.nodes["threshold"][internal] == b.nodes["threshold"][internal]).all()
        assert (a.nodes["gain"][internal] == b.nodes["gain"][internal]).all()
        assert (b.nodes["gain"][~internal] == -1.0).all()  # NodeData.build: leaf gain
        assert (a.stats == b.stats).all()
    assert back.getBaseLearner().getMaxDepth() == 4
    want = oracle.predict(orf, X)
    np.testing.assert_array_equal(_py_predict(m, X, False), want)
    np.testing.assert_array_equal(_py_predict(back, X, False), want)


def test_node_data_parquet_schema(tmp_path, cpusmall):
    X, y = cpusmall
    m, _ = _model(sb.BaggingRegressionModel, X, y, 1, False)
    path = str(tmp_path / "m")
    m.save(path)
    f = [x for x in os.listdir(os.path.join(path, "model-0", "data")) if x.endswith(".parquet")]
    assert len(f) == 1 and f[0].startswith("part-00000-")
    t = pq.read_table(os.path.join(path, "model-0", "data", f[0]))
    assert t.schema.names == ["id", "prediction", "impurity", "impurityStats", "gain", "leftChild",
                              "rightChild", "split"]
    row_meta = json.loads(t.schema.metadata[b"org.apache.spark.sql.parquet.row.metadata"])
    assert [fl["name"] for fl in row_meta["fields"]] == t.schema.names
    d = t.to_pydict()
    root = d["split"][0]
    assert root["numCategories"] == -1 and len(root["leftCategoriesOrThreshold"]) == 1
    leaves = [i for i, l in enumerate(d["leftChild"]) if l < 0]
    assert all(d["split"][i] == {"featureIndex": -1, "leftCategoriesOrThreshold": [],
                                 "numCategories": -1} for i in leaves)
    assert all(len(s) == 3 for s in d["impurityStats"])  # Variance: count, sum, sumSq
    sub = json.loads(open([os.path.join(path, "data-0", x) for x in os.listdir(os.path.join(path, "data-0"))
                           if x.endswith(".json")][0]).read())
    assert sub == {"subspace": [int(v) for v in m.subspaces[0]]}


def test_classification_round_trip_and_reader_asymmetry(tmp_path, vehicle):
    X, y = vehicle
    m, orf = _model(sb.BaggingClassificationModel, X, y, 5, True)
    path = str(tmp_path / "bc")
    m.save(path)
    tm = sp.load_metadata(os.path.join(path, "model-0"))
    assert tm["class"] == sp.DTC_MODEL_CLASS and tm["numClasses"] == m.models[0].stats.shape[1]
    back = sb.BaggingClassificationModel.load(path)
    np.testing.assert_array_equal(_py_predict(back, X, True), oracle.predict(orf, X, classification=True))
    # H14: the classifier reader counts models from numBaseModels, the regressor's
    # from param numBaseLearners
    mp = os.path.join(path, "metadata", "part-00000")
    meta = json.loads(open(mp).read())
    meta["paramMap"]["numBaseLearners"] = 2
    open(mp, "w").write(json.dumps(meta) + "\n")
    assert sb.BaggingClassificationModel.load(path).numBaseModels == 5


def test_regression_reader_counts_num_base_learners(tmp_path, cpusmall):
    X, y = cpusmall
    m, _ = _model(sb.BaggingRegressionModel, X, y, 3, False)
    path = str(tmp_path / "br")
    m.save(path)
    mp = os.path.join(path, "metadata", "part-00000")
    meta = json.loads(open(mp).read())
    meta["paramMap"]["numBaseLearners"] = 2
    open(mp, "w").write(json.dumps(meta) + "\n")
    assert sb.BaggingRegressionModel.load(path).numBaseModels == 2


def test_load_wrong_class_and_existing_path(tmp_path, cpusmall):
    X, y = cpusmall
    m, _ = _model(sb.BaggingRegressionModel, X, y, 1, False)
    path = str(tmp_path / "x")
    m.save(path)
    with pytest.raises(sb.IllegalArgumentException, match="Expected class name"):
        sb.BaggingClassificationModel.load(path)
    with pytest.raises(sb.IllegalArgumentException, match="already exists"):
        m.save(path)


def test_estimator_round_trip(tmp_path):
    est = (sb.BaggingClassifier().setBaseLearner(sb.DecisionTreeClassifier().setMaxBins(16))
           .setNumBaseLearners(7).setSubspaceRatio(0.5))
    path = str(tmp_path / "est")
    est.save(path)
    meta = sp.load_metadata(path)
    assert meta["class"] == "org.apache.spark.ml.classification.BaggingClassifier"
    back = sb.BaggingClassifier.load(path)
    assert back.uid == est.uid
    assert (back.getNumBaseLearners(), back.getSubspaceRatio()) == (7, 0.5)
    assert back.getBaseLearner().getMaxBins() == 16 and back.getBaseLearner().uid == est.getBaseLearner().uid
