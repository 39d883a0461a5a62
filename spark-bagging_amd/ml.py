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
import logging
import os
import threading
import uuid
import warnings

import numpy as np

from . import _native as nat
from . import persistence as sp
from .libsvm import is_sparse, load_libsvm


def java_string_hash(s):
    """java.lang.String.hashCode (HasSeed default seed = getClass.getName.hashCode.toLong)."""
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


_log = logging.getLogger("spark_bagging_amd")

# Instrumentation.logParams list of BaggingRegressor/-Classifier.train
# (ml/regression/BaggingRegressor.scala:121-135, ml/classification/BaggingClassifier.scala:121-135)
_LOGGED_PARAMS = ("labelCol", "weightCol", "featuresCol", "predictionCol", "numBaseLearners",
                  "sampleRatio", "replacement", "subspaceRatio", "seed")


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
        # DecisionTree's seed drives RandomForest.findSplits' split-finding sample of
        # subbags larger than max(maxBins^2, 10000) rows (k_split_sample).
        return self.set("seed", int(v))

    def getSeed(self):
        return self.get("seed")

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


class _DecisionTreeEstimator(_DecisionTreeParams):
    _spark_class = None
    _spark_model_class = None
    _spark_defaults = None
    _uid_prefix = None

    def __init__(self, uid=None):
        super().__init__(uid or f"{self._uid_prefix}_{uuid.uuid4().hex[-12:]}")
        self._other_params = {}  # Spark params the engine does not use (round-tripped)

    def setImpurity(self, v):
        return self.set("impurity", v)

    def save(self, path):
        """DefaultParamsWritable: metadata only (explicitly set params)."""
        sp.save_metadata(path, self._spark_class, self.uid, dict(self._other_params, **self._values),
                         self._spark_defaults)

    @staticmethod
    def load(path):
        meta = sp.load_metadata(path)
        cls = {sp.DTR_CLASS: DecisionTreeRegressor, sp.DTC_CLASS: DecisionTreeClassifier}.get(meta["class"])
        if cls is None:
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"the MI355X engine accelerates DecisionTree base learners only, "
                                 f"found {meta['class']}")
        bl = cls(uid=meta["uid"])
        for k, v in meta["paramMap"].items():
            if k in bl._defaults:
                bl.set(k, v)
            else:
                bl._other_params[k] = v
        return bl

    def copy(self, extra=None):
        other = super().copy(extra)
        other._other_params = dict(self._other_params)
        return other


class DecisionTreeRegressor(_DecisionTreeEstimator):
    _defaults = dict(_DecisionTreeParams._defaults, impurity="variance",
                     seed=java_string_hash("org.apache.spark.ml.regression.DecisionTreeRegressor"))
    _validators = dict(_DecisionTreeParams._validators, impurity=lambda x: x == "variance")
    impurity_code = nat.IMPURITY_VARIANCE
    _spark_class = sp.DTR_CLASS
    _spark_model_class = sp.DTR_MODEL_CLASS
    _spark_defaults = sp.DTR_DEFAULTS
    _uid_prefix = "dtr"


class DecisionTreeClassifier(_DecisionTreeEstimator):
    _defaults = dict(_DecisionTreeParams._defaults, impurity="gini",
                     seed=java_string_hash("org.apache.spark.ml.classification.DecisionTreeClassifier"))
    _validators = dict(_DecisionTreeParams._validators, impurity=lambda x: x == "gini")
    impurity_code = nat.IMPURITY_GINI
    _spark_class = sp.DTC_CLASS
    _spark_model_class = sp.DTC_MODEL_CLASS
    _spark_defaults = sp.DTC_DEFAULTS
    _uid_prefix = "dtc"


class Frame:
    """The (label, features) columns of a DataFrame plus its partitioning.

    Row j of partition p is the j-th row the bag's per-partition generators
    see (sql/catalyst/expressions/Poisson.scala:53-56), so partitioning is part
    of the input, exactly as in Spark.
    """

    def __init__(self, features, label, partition_offsets=None, weight=None):
        # DenseVector rows (an [N x F] array) or SparseVector rows (libsvm.SparseRows /
        # scipy CSR), kept sparse all the way to the device
        self.features = features if is_sparse(features) else np.ascontiguousarray(features, np.float64)
        self.label = np.ascontiguousarray(label, np.float64)
        n = self.features.shape[0]
        if self.label.shape[0] != n:
            raise nat.IllegalArgumentException(nat.SBAG_EINVAL, "label and features differ in length")
        self.partition_offsets = None if partition_offsets is None else [int(x) for x in partition_offsets]
        self.weight = weight

    @classmethod
    def from_libsvm(cls, path, num_partitions=1, sparse=True):
        X, y = load_libsvm(path, sparse=sparse)
        return cls(X, y, partition_offsets=even_partitions(len(y), num_partitions))

    def device_dataset(self, ctx):
        if is_sparse(self.features):
            return nat.DeviceDataset.from_csr(self.features, self.label, ctx)
        return nat.DeviceDataset.from_numpy(self.features, self.label, ctx)

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

    # ---- persistence: BaggingRegressor.write (BaggingRegressorParams.saveImpl,
    # BaggingRegressor.scala:50-66): metadata without baseLearner + learner/
    def save(self, path):
        if os.path.exists(path):
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"Path {path} already exists. To overwrite it, please use "
                                 "write.overwrite().save(path) for Scala and use "
                                 "write().overwrite().save(path) for Java and Python.")
        params = {k: v for k, v in self.extractParamMap().items() if k != "baseLearner"}
        defaults = {k: v for k, v in self._defaults.items() if v is not None and k != "baseLearner"}
        sp.save_metadata(path, self._spark_class, self.uid, params, defaults)
        self._base().save(os.path.join(path, "learner"))

    @classmethod
    def load(cls, path):
        meta = sp.load_metadata(path, cls._spark_class)
        est = cls(uid=meta["uid"])
        for k, v in meta["paramMap"].items():
            if k in est._defaults:
                est._values[k] = v
        est._values["baseLearner"] = _DecisionTreeEstimator.load(os.path.join(path, "learner"))
        return est

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

    def _instrument(self, dataset):
        """Instrumentation.instrumented's records (BaggingRegressor.scala:121-135):
        logPipelineStage, logDataset, logParams -- logged at INFO on the
        "spark_bagging_amd" logger with Spark's "<uid>: " prefix, and returned."""
        part = getattr(dataset, "partition_offsets", None)
        rec = {"stage": type(self).__name__, "uid": self.uid,
               "numPartitions": (len(part) - 1) if part is not None else 1,
               "params": {k: self.get(k) for k in _LOGGED_PARAMS if self.isDefined(k)}}
        _log.info("%s: Stage class: %s", self.uid, rec["stage"])
        _log.info("%s: Stage uid: %s", self.uid, self.uid)
        _log.info("%s: training: numPartitions=%d", self.uid, rec["numPartitions"])
        _log.info("%s: %s", self.uid, json.dumps(rec["params"], sort_keys=True, default=str))
        return rec

    def _train(self, dataset, bug_compat, learner_range=None):
        bl = self._base()
        if not isinstance(dataset, (Frame, nat.DeviceDataset)):
            X, y = dataset
            return self._train(Frame(X, y), bug_compat, learner_range)
        train_log = self._instrument(dataset)
        if self.get("weightCol"):
            # DecisionTree has no HasWeightCol in Spark 2.4 (BaggingRegressor.scala:137-144, H10)
            msg = f"weightCol is ignored, as it is not supported by {type(bl).__name__} now."
            _log.warning("%s: %s", self.uid, msg)
            warnings.warn(msg)
        L = self.get("numBaseLearners")
        lb0, le0 = learner_range if learner_range is not None else (0, L)
        if not (0 <= lb0 < le0 <= L):
            raise nat.IllegalArgumentException(nat.SBAG_EINVAL, f"bad learner range {learner_range}")
        seed = self.get("seed")
        devices = list(self.devices or [0])
        if len(set(devices)) != len(devices):
            # one context per device: two shards on one context would only serialize
            raise nat.IllegalArgumentException(nat.SBAG_EINVAL, f"duplicate device ids {devices}")
        if isinstance(dataset, Frame):
            part = dataset.partition_offsets
            make_ds = [lambda ctx, d=dataset: d.device_dataset(ctx)]
        elif isinstance(dataset, nat.DeviceDataset):
            part = None
            if len(devices) > 1 or (self.devices and devices[0] != dataset.ctx.device):
                raise nat.IllegalArgumentException(
                    nat.SBAG_EINVAL, f"a DeviceDataset lives on device {dataset.ctx.device} only")
            devices = [dataset.ctx.device]
            make_ds = [lambda ctx, d=dataset: d]
        shards = [(lb0 + a, lb0 + b) for a, b in _learner_shards(le0 - lb0, len(devices))]
        results = [None] * len(devices)
        errors = []

        def work(k):
            try:
                ds0 = dataset if isinstance(dataset, nat.DeviceDataset) else None
                ctx = ds0.ctx if ds0 is not None else nat.default_context(devices[k])
                ds = make_ds[0](ctx)
                lb, le = shards[k]
                results[k] = nat.fit(
                    ctx, ds, replacement=self.get("replacement"),
                    sample_ratio=self.get("sampleRatio"), seed=seed, learner_begin=lb,
                    learner_end=le, subspace_ratio=self.get("subspaceRatio"),
                    subspace_bug_compat=bug_compat, partition_offsets=part,
                    max_depth=bl.getMaxDepth(), max_bins=bl.getMaxBins(),
                    min_instances_per_node=bl.getMinInstancesPerNode(),
                    min_info_gain=bl.getMinInfoGain(), impurity=bl.impurity_code,
                    tree_seed=bl.getSeed())
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
        model.train_log = train_log
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
        self.train_log = None

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
        if isinstance(dataset, nat.DeviceDataset):  # on the dataset's own device
            return self._transform_dataset(dataset, per_tree)
        ctx = nat.default_context(device)
        X = dataset.features if isinstance(dataset, Frame) else dataset
        if is_sparse(X):  # SparseVector rows: binned on the device from CSR, no dense copy
            ds = nat.DeviceDataset.from_csr(X, np.zeros(X.shape[0]), ctx)
            try:
                return self._transform_dataset(ds, per_tree)
            finally:
                ds.free()
        X = np.asarray(X, np.float64)
        if X.ndim == 1:
            X = X[None, :]
        return nat.predict(ctx, self.native_forest(), X, self._agg, per_tree=per_tree)

    def _transform_dataset(self, ds, per_tree):
        """Predictions of a device dataset; with per_tree also every tree's prediction
        [L x N] (fp64, learner order), as the host-row path returns them."""
        forest = self.native_forest()
        pred = nat.predict_dataset(ds.ctx, forest, ds, self._agg)
        if not per_tree:
            return pred
        import torch

        dev = torch.device("cuda", ds.ctx.device)
        buf = torch.empty((len(self.models), ds.shape[0]), dtype=torch.float64, device=dev)
        torch.cuda.synchronize(dev)  # the allocation is complete before the library's stream writes
        nat.predict_dataset_device(ds.ctx, forest, ds, nat.OUT_VOTES, 8, buf.data_ptr())
        torch.cuda.synchronize(dev)
        return pred, buf.cpu().numpy()

    def predict(self, features):
        """Single-vector predict (BaggingRegressor.scala:248-256 / BaggingClassifier.scala:248-257)."""
        return float(self.transform(np.asarray(features, np.float64)[None, :])[0])

    # ---- persistence (MLWritable / MLReadable), Spark 2.4.3 directory layout -------
    def _bagging_defaults(self):
        d = {k: v for k, v in _BaggingParams._defaults.items() if v is not None}
        d["seed"] = self._estimator_seed_default
        return d

    def save(self, path):
        """BaggingRegressionModelWriter.saveImpl (BaggingRegressor.scala:273-295):
        metadata (+ numBaseModels), learner/, model-$idx (tree), data-$idx (subspace)."""
        if os.path.exists(path):
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"Path {path} already exists. To overwrite it, please use "
                                 "write.overwrite().save(path) for Scala and use "
                                 "write().overwrite().save(path) for Java and Python.")
        params = {k: v for k, v in self.extractParamMap().items() if k != "baseLearner"}
        sp.save_metadata(path, self._spark_class, self.uid, params, self._bagging_defaults(),
                         {"numBaseModels": self.numBaseModels})
        bl = self.get("baseLearner")
        if bl is None:
            bl = (DecisionTreeClassifier() if self._agg == nat.AGG_MODE else DecisionTreeRegressor())
        bl.save(os.path.join(path, "learner"))
        # fitBaseLearner sets labelCol / featuresCol / predictionCol explicitly
        # (ensembleParams.scala:105-108); the tree model keeps the estimator's uid
        tree_params = dict(bl._other_params, **bl._values)
        tree_params.update(labelCol=self.get("labelCol"), featuresCol=self.get("featuresCol"),
                           predictionCol=self.get("predictionCol"))
        for i, (m, s) in enumerate(zip(self.models, self.subspaces)):
            mp = os.path.join(path, f"model-{i}")
            extra = {"numFeatures": int(len(s))}
            if m.impurity == nat.IMPURITY_GINI:
                extra["numClasses"] = int(m.stats.shape[1])
            sp.save_metadata(mp, bl._spark_model_class, bl.uid, tree_params, bl._spark_defaults,
                             extra)
            sp.write_tree_data(mp, m.nodes, m.stats)
            sp.write_subspace(os.path.join(path, f"data-{i}"), s)

    @classmethod
    def load(cls, path):
        """Bagging*ModelReader.load (BaggingRegressor.scala:297-318; classifier: the
        model count comes from metadata numBaseModels, BaggingClassifier.scala:307)."""
        meta = sp.load_metadata(path, cls._spark_class)
        bl = _DecisionTreeEstimator.load(os.path.join(path, "learner"))
        if cls._agg == nat.AGG_MEAN:
            n = int(meta["paramMap"]["numBaseLearners"])
        else:
            n = int(meta["numBaseModels"])
        models, subs = [], []
        for i in range(n):
            mp = os.path.join(path, f"model-{i}")
            mm = sp.load_metadata(mp)
            imp = nat.IMPURITY_GINI if mm["class"] == sp.DTC_MODEL_CLASS else nat.IMPURITY_VARIANCE
            nodes, stats = sp.read_tree_data(mp)
            models.append(DecisionTreeModel(nodes, stats, imp))
            subs.append(sp.read_subspace(os.path.join(path, f"data-{i}")))
        m = cls(subs, models, uid=meta["uid"])
        for k, v in meta["paramMap"].items():  # DefaultParamsReader.getAndSetParams
            if k in m._defaults:
                m._values[k] = v
        m._values["baseLearner"] = bl
        return m


class BaggingRegressionModel(_BaggingModel):
    _agg = nat.AGG_MEAN
    _spark_class = "org.apache.spark.ml.regression.BaggingRegressionModel"
    _estimator_seed_default = java_string_hash("org.apache.spark.ml.regression.BaggingRegressor")
    _defaults = dict(_BaggingParams._defaults,
                     seed=java_string_hash("org.apache.spark.ml.regression.BaggingRegressionModel"))


class BaggingClassificationModel(_BaggingModel):
    _agg = nat.AGG_MODE
    _spark_class = "org.apache.spark.ml.classification.BaggingClassificationModel"
    _estimator_seed_default = java_string_hash("org.apache.spark.ml.classification.BaggingClassifier")
    _defaults = dict(_BaggingParams._defaults,
                     seed=java_string_hash("org.apache.spark.ml.classification.BaggingClassificationModel"))


class BaggingRegressor(_BaggingEstimator):
    _model_cls = BaggingRegressionModel
    _spark_class = "org.apache.spark.ml.regression.BaggingRegressor"
    _defaults = dict(_BaggingParams._defaults,
                     seed=java_string_hash("org.apache.spark.ml.regression.BaggingRegressor"))


class BaggingClassifier(_BaggingEstimator):
    _model_cls = BaggingClassificationModel
    _spark_class = "org.apache.spark.ml.classification.BaggingClassifier"
    _defaults = dict(_BaggingParams._defaults,
                     seed=java_string_hash("org.apache.spark.ml.classification.BaggingClassifier"))
