"""Host-side mirror of spark-ensemble's bagging Estimator/Model API.

Same names, parameters, defaults, validation and error behaviour as the
reference (paths relative to /root/reference/core/src/main/scala/org/apache/spark/):

  BaggingRegressor          ml/regression/BaggingRegressor.scala:81-203
  BaggingRegressionModel    ml/regression/BaggingRegressor.scala:235-265
  BaggingClassifier         ml/classification/BaggingClassifier.scala:81-203
  BaggingClassificationModel ml/classification/BaggingClassifier.scala:235-267
  params                    ml/bagging/BaggingParams.scala:23-33, ml/ensemble/HasSubBag.scala:39-79,
                            ml/ensemble/ensembleParams.scala:64-117

`fit` and `transform` run on the MI355X through libsbag (include/sbag.h); there is
no CPU fallback.  Base learners are the two the engine accelerates:
DecisionTreeRegressor and DecisionTreeClassifier (param holders with Spark's
names and defaults; their fit only happens inside the ensemble).
"""
import json
import os
import threading
import uuid
import warnings

import numpy as np

from . import _native as nat


def java_string_hash(s):
    """java.lang.String.hashCode (HasSeed default seed = getClass.getName.hashCode.toLong)."""
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


def _uid(prefix):
    return f"{prefix}_{uuid.uuid4().hex[-12:]}"


class Params:
    """Minimal Spark ML Params: defaults, explicit values, validators, copy(extra)."""

    _defaults = {}
    _validators = {}

    def __init__(self, uid=None):
        self.uid = uid or _uid(type(self).__name__)
        self._values = {}

    def set(self, name, value):
        if name not in self._defaults:
            raise nat.IllegalArgumentException(nat.SBAG_EINVAL, f"{self.uid} has no param {name}")
        v = self._validators.get(name)
        if v is not None and not v(value):
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"{self.uid} parameter {name} given invalid value {value}.")
        self._values[name] = value
        return self

    def get(self, name):
        return self._values.get(name, self._defaults[name])

    def isSet(self, name):
        return name in self._values

    def isDefined(self, name):
        return name in self._values or self._defaults.get(name) is not None

    def extractParamMap(self):
        return {k: self.get(k) for k in self._defaults}

    def copy(self, extra=None):
        other = type(self).__new__(type(self))
        other.__dict__.update(self.__dict__)
        other._values = dict(self._values)
        for k, v in (extra or {}).items():
            other.set(k, v)
        return other


def _in_range01(x):
    return 0.0 <= float(x) <= 1.0


class _DecisionTreeParams(Params):
    _defaults = {"maxDepth": 5, "maxBins": 32, "minInstancesPerNode": 1, "minInfoGain": 0.0,
                 "labelCol": "label", "featuresCol": "features", "predictionCol": "prediction",
                 "seed": None, "impurity": None}
    _validators = {"maxDepth": lambda x: 0 <= int(x) <= 30, "maxBins": lambda x: int(x) >= 2,
                   "minInstancesPerNode": lambda x: int(x) >= 1,
                   "minInfoGain": lambda x: float(x) >= 0.0}

    def setMaxDepth(self, v):
        return self.set("maxDepth", int(v))

    def setMaxBins(self, v):
        return self.set("maxBins", int(v))

    def setMinInstancesPerNode(self, v):
        return self.set("minInstancesPerNode", int(v))

    def setMinInfoGain(self, v):
        return self.set("minInfoGain", float(v))

    def setSeed(self, v):
        # DecisionTree's seed only drives split-finding sampling for subbags larger
        # than max(maxBins^2, 10000) rows, which the engine replaces.
        return self.set("seed", int(v))

    def getMaxDepth(self):
        return self.get("maxDepth")

    def getMaxBins(self):
        return self.get("maxBins")

    def getMinInstancesPerNode(self):
        return self.get("minInstancesPerNode")

    def getMinInfoGain(self):
        return self.get("minInfoGain")

    def getImpurity(self):
        return self.get("impurity")


class DecisionTreeRegressor(_DecisionTreeParams):
    _defaults = dict(_DecisionTreeParams._defaults, impurity="variance",
                     seed=java_string_hash("org.apache.spark.ml.regression.DecisionTreeRegressor"))
    _validators = dict(_DecisionTreeParams._validators, impurity=lambda x: x == "variance")
    impurity_code = nat.IMPURITY_VARIANCE

    def setImpurity(self, v):
        return self.set("impurity", v)


class DecisionTreeClassifier(_DecisionTreeParams):
    _defaults = dict(_DecisionTreeParams._defaults, impurity="gini",
                     seed=java_string_hash("org.apache.spark.ml.classification.DecisionTreeClassifier"))
    _validators = dict(_DecisionTreeParams._validators, impurity=lambda x: x == "gini")
    impurity_code = nat.IMPURITY_GINI

    def setImpurity(self, v):
        return self.set("impurity", v)


class Frame:
    """The (label, features) columns of a DataFrame plus its partitioning.

    Row j of partition p is the j-th row the bag's per-partition generators
    see (sql/catalyst/expressions/Poisson.scala:53-56), so partitioning is part
    of the input, exactly as in Spark.
    """

    def __init__(self, features, label, partition_offsets=None, weight=None):
        self.features = np.ascontiguousarray(features, np.float64)
        self.label = np.ascontiguousarray(label, np.float64)
        n = self.features.shape[0]
        if self.label.shape[0] != n:
            raise nat.IllegalArgumentException(nat.SBAG_EINVAL, "label and features differ in length")
        self.partition_offsets = None if partition_offsets is None else [int(x) for x in partition_offsets]
        self.weight = weight

    @classmethod
    def from_libsvm(cls, path, num_partitions=1):
        from .libsvm import load_libsvm

        X, y = load_libsvm(path)
        return cls(X, y, partition_offsets=even_partitions(len(y), num_partitions))

    @property
    def num_rows(self):
        return self.features.shape[0]

    @property
    def num_features(self):
        return self.features.shape[1]


def even_partitions(n, p):
    return [int(round(i * n / p)) for i in range(p + 1)]


class DecisionTreeModel:
    """A fitted base learner: Spark's NodeData rows in pre-order
    (DecisionTreeModelReadWrite), `feature` in subspace coordinates."""

    def __init__(self, nodes, stats, impurity):
        self.nodes = nodes
        self.stats = stats
        self.impurity = impurity

    @property
    def numNodes(self):
        return len(self.nodes)

    @property
    def depth(self):
        def d(i):
            n = self.nodes[i]
            return 0 if n["left"] < 0 else 1 + max(d(n["left"]), d(n["right"]))
        return d(0)

    def predict(self, sliced):
        """Node.predictImpl on an already-sliced feature vector."""
        i = 0
        while self.nodes[i]["left"] >= 0:
            n = self.nodes[i]
            i = n["left"] if sliced[n["feature"]] <= n["threshold"] else n["right"]
        return float(self.nodes[i]["prediction"])


class _BaggingParams(Params):
    _defaults = {"numBaseLearners": 10, "replacement": False, "sampleRatio": 1.0,
                 "subspaceRatio": 1.0, "parallelism": 1, "weightCol": None, "baseLearner": None,
                 "labelCol": "label", "featuresCol": "features", "predictionCol": "prediction",
                 "seed": None}
    _validators = {"numBaseLearners": lambda x: int(x) >= 1, "sampleRatio": _in_range01,
                   "subspaceRatio": _in_range01, "parallelism": lambda x: int(x) >= 1}

    def getNumBaseLearners(self):
        return self.get("numBaseLearners")

    def getReplacement(self):
        return self.get("replacement")

    def getSampleRatio(self):
        return self.get("sampleRatio")

    def getSubspaceRatio(self):
        return self.get("subspaceRatio")

    def getParallelism(self):
        return self.get("parallelism")

    def getSeed(self):
        return self.get("seed")

    def getBaseLearner(self):
        return self.get("baseLearner")


class _BaggingEstimator(_BaggingParams):
    _model_cls = None
    _agg = None

    def __init__(self, uid=None, devices=None):
        super().__init__(uid)
        # learners can be sharded over several local devices (one context each);
        # results do not depend on the sharding (learners are independent)
        self.devices = devices

    # setters (BaggingRegressor.scala:88-113; no setSeed in the reference, H3)
    def setBaseLearner(self, value):
        if not isinstance(value, (DecisionTreeRegressor, DecisionTreeClassifier)):
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, "the MI355X engine accelerates DecisionTree{Regressor,Classifier} "
                                 f"base learners only, got {type(value).__name__}")
        return self.set("baseLearner", value)

    def setWeightCol(self, value):
        return self.set("weightCol", value)

    def setReplacement(self, value):
        return self.set("replacement", bool(value))

    def setSampleRatio(self, value):
        return self.set("sampleRatio", float(value))

    def setSubspaceRatio(self, value):
        return self.set("subspaceRatio", float(value))

    def setNumBaseLearners(self, value):
        return self.set("numBaseLearners", int(value))

    def setParallelism(self, value):
        return self.set("parallelism", int(value))

    def copy(self, extra=None):
        other = super().copy(extra)
        if other.get("baseLearner") is not None:
            other._values["baseLearner"] = other.get("baseLearner").copy()
        return other

    def _base(self):
        bl = self.get("baseLearner")
        if bl is None:
            raise nat.IllegalArgumentException(nat.SBAG_EINVAL, "baseLearner must be set")
        return bl

    def fit(self, dataset, params=None, bug_compat=True):
        """Predictor.fit -> train (BaggingRegressor.scala:121-199).

        bug_compat=True reproduces the reference exactly, including
        mkSubspace(getSampleRatio, ...); False uses subspaceRatio."""
        est = self.copy(params) if params else self
        return est._train(dataset, bug_compat)

    def fit_range(self, dataset, learner_begin, learner_end, bug_compat=True, devices=None):
        """Train only learners [learner_begin, learner_end) of the ensemble (one
        shard of a multi-process fit, see distributed.py); learner i still uses
        seed + i, so shards concatenate to exactly the single-process model."""
        est = self.copy()
        if devices is not None:
            est.devices = devices
        return est._train(dataset, bug_compat, (learner_begin, learner_end))

    def _train(self, dataset, bug_compat, learner_range=None):
        bl = self._base()
        if self.get("weightCol"):
            # DecisionTree has no HasWeightCol in Spark 2.4 (BaggingRegressor.scala:137-144, H10)
            warnings.warn(f"weightCol is ignored, as it is not supported by {type(bl).__name__} now.")
        L = self.get("numBaseLearners")
        lb0, le0 = learner_range if learner_range is not None else (0, L)
        if not (0 <= lb0 < le0 <= L):
            raise nat.IllegalArgumentException(nat.SBAG_EINVAL, f"bad learner range {learner_range}")
        seed = self.get("seed")
        devices = self.devices or [0]
        if isinstance(dataset, Frame):
            part = dataset.partition_offsets
            make_ds = [lambda ctx, d=dataset: nat.DeviceDataset.from_numpy(d.features, d.label, ctx)]
        elif isinstance(dataset, nat.DeviceDataset):
            part = None
            if len(devices) > 1:
                raise nat.IllegalArgumentException(nat.SBAG_EINVAL,
                                                   "a DeviceDataset lives on one device")
            make_ds = [lambda ctx, d=dataset: d]
        else:
            X, y = dataset
            return self._train(Frame(X, y), bug_compat, learner_range)
        shards = [(lb0 + a, lb0 + b) for a, b in _learner_shards(le0 - lb0, len(devices))]
        results = [None] * len(devices)
        errors = []

        def work(k):
            try:
                ctx = nat.default_context(devices[k])
                ds = make_ds[0](ctx)
                lb, le = shards[k]
                results[k] = nat.fit(
                    ctx, ds, replacement=self.get("replacement"),
                    sample_ratio=self.get("sampleRatio"), seed=seed, learner_begin=lb,
                    learner_end=le, subspace_ratio=self.get("subspaceRatio"),
                    subspace_bug_compat=bug_compat, partition_offsets=part,
                    max_depth=bl.getMaxDepth(), max_bins=bl.getMaxBins(),
                    min_instances_per_node=bl.getMinInstancesPerNode(),
                    min_info_gain=bl.getMinInfoGain(), impurity=bl.impurity_code)
            except Exception as e:  # surfaced like ThreadUtils.awaitResult (BaggingRegressor.scala:191)
                errors.append(e)

        threads = [threading.Thread(target=work, args=(k,)) for k in range(len(devices))
                   if shards[k][1] > shards[k][0]]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        subspaces, models, timings = [], [], []
        for f in results:
            if f is None:
                continue
            timings.append(f.timing())
            for t in range(len(f)):
                nodes, stats = f.tree(t)
                subspaces.append(f.subspace(t))
                models.append(DecisionTreeModel(nodes, stats, bl.impurity_code))
        model = self._model_cls(subspaces, models)
        model._copy_params_from(self)
        model.fit_timing = timings
        return model


def _learner_shards(L, k):
    return [(i * L // k, (i + 1) * L // k) for i in range(k)]


class _BaggingModel(_BaggingParams):
    _agg = None

    def __init__(self, subspaces, models, uid=None):
        super().__init__(uid)
        self.subspaces = [np.asarray(s, np.int32) for s in subspaces]
        self.models = list(models)
        self._forest = None
        self.fit_timing = []

    @property
    def numBaseModels(self):
        return len(self.models)

    def _copy_params_from(self, est):
        # Params.copyValues: explicit values and the estimator's defaults
        for k in est._defaults:
            if k in self._defaults:
                self._values[k] = est.get(k)

    def native_forest(self):
        if self._forest is None:
            imp = self.models[0].impurity if self.models else nat.IMPURITY_VARIANCE
            self._forest = nat.NativeForest.from_trees([m.nodes for m in self.models],
                                                       self.subspaces, imp)
        return self._forest

    def transform(self, dataset, device=0, per_tree=False):
        """PredictionModel.transform: one prediction per row (HIP kernel)."""
        ctx = nat.default_context(device)
        if isinstance(dataset, nat.DeviceDataset):
            return nat.predict_dataset(ctx, self.native_forest(), dataset, self._agg)
        X = dataset.features if isinstance(dataset, Frame) else np.asarray(dataset, np.float64)
        if X.ndim == 1:
            X = X[None, :]
        return nat.predict(ctx, self.native_forest(), X, self._agg, per_tree=per_tree)

    def predict(self, features):
        """Single-vector predict (BaggingRegressor.scala:248-256 / BaggingClassifier.scala:248-257)."""
        return float(self.transform(np.asarray(features, np.float64)[None, :])[0])

    # ---- persistence (MLWritable / MLReadable), Spark directory layout -------------
    def save(self, path):
        """metadata (params + numBaseModels), learner/ (base learner params),
        model-$idx (nodes), data-$idx (subspace) -- BaggingRegressor.scala:273-295."""
        os.makedirs(path, exist_ok=False)
        params = {k: v for k, v in self.extractParamMap().items() if k != "baseLearner"}
        meta = {"class": self._spark_class, "uid": self.uid, "paramMap": params,
                "numBaseModels": self.numBaseModels, "sparkVersion": "2.4.3"}
        with open(os.path.join(path, "metadata.json"), "w") as fh:
            json.dump(meta, fh)
        bl = self.get("baseLearner")
        os.makedirs(os.path.join(path, "learner"))
        with open(os.path.join(path, "learner", "metadata.json"), "w") as fh:
            json.dump({"class": type(bl).__name__ if bl else None,
                       "paramMap": bl.extractParamMap() if bl else {}}, fh)
        for i, (m, s) in enumerate(zip(self.models, self.subspaces)):
            os.makedirs(os.path.join(path, f"model-{i}"))
            np.savez(os.path.join(path, f"model-{i}", "nodes.npz"), nodes=m.nodes, stats=m.stats,
                     impurity=np.int32(m.impurity))
            os.makedirs(os.path.join(path, f"data-{i}"))
            with open(os.path.join(path, f"data-{i}", "part-00000.json"), "w") as fh:
                json.dump({"subspace": [int(x) for x in s]}, fh)

    @classmethod
    def load(cls, path):
        with open(os.path.join(path, "metadata.json")) as fh:
            meta = json.load(fh)
        if meta["class"] != cls._spark_class:
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"Error loading metadata: Expected class name {cls._spark_class} "
                                 f"but found class name {meta['class']}")
        models, subs = [], []
        for i in range(meta["numBaseModels"]):
            z = np.load(os.path.join(path, f"model-{i}", "nodes.npz"), allow_pickle=False)
            models.append(DecisionTreeModel(z["nodes"], z["stats"], int(z["impurity"])))
            with open(os.path.join(path, f"data-{i}", "part-00000.json")) as fh:
                subs.append(json.load(fh)["subspace"])
        m = cls(subs, models, uid=meta["uid"])
        for k, v in meta["paramMap"].items():
            if v is not None:
                m._values[k] = v
        with open(os.path.join(path, "learner", "metadata.json")) as fh:
            lm = json.load(fh)
        if lm["class"]:
            bl = {"DecisionTreeRegressor": DecisionTreeRegressor,
                  "DecisionTreeClassifier": DecisionTreeClassifier}[lm["class"]]()
            for k, v in lm["paramMap"].items():
                if v is not None:
                    bl._values[k] = v
            m._values["baseLearner"] = bl
        return m


class BaggingRegressionModel(_BaggingModel):
    _agg = nat.AGG_MEAN
    _spark_class = "org.apache.spark.ml.regression.BaggingRegressionModel"
    _defaults = dict(_BaggingParams._defaults,
                     seed=java_string_hash("org.apache.spark.ml.regression.BaggingRegressionModel"))


class BaggingClassificationModel(_BaggingModel):
    _agg = nat.AGG_MODE
    _spark_class = "org.apache.spark.ml.classification.BaggingClassificationModel"
    _defaults = dict(_BaggingParams._defaults,
                     seed=java_string_hash("org.apache.spark.ml.classification.BaggingClassificationModel"))


class BaggingRegressor(_BaggingEstimator):
    _model_cls = BaggingRegressionModel
    _defaults = dict(_BaggingParams._defaults,
                     seed=java_string_hash("org.apache.spark.ml.regression.BaggingRegressor"))


class BaggingClassifier(_BaggingEstimator):
    _model_cls = BaggingClassificationModel
    _defaults = dict(_BaggingParams._defaults,
                     seed=java_string_hash("org.apache.spark.ml.classification.BaggingClassifier"))
