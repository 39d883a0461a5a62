"""GBMRegressor / GBMRegressionModel: SURVEY §8(f) rank 3, the reference's GBM reusing
the bagging path's sampler, subspaces and tree engine.

Mirror of (paths relative to /root/reference/core/src/main/scala/org/apache/spark/):

  GBMRegressor.train         ml/regression/GBMRegressor.scala:196-456
  trainBoosters              ml/regression/GBMRegressor.scala:255-399
  GBMRegressionModel.predict ml/regression/GBMRegressor.scala:511-516
  loss / grad functions      ml/regression/GBMRegressor.scala:88-118
  params                     ml/boosting/GBMParams.scala:41-67, ml/boosting/BoostingParams.scala:34-46,
                             ml/ensemble/ensembleParams.scala:26-61, ml/ensemble/HasSubBag.scala:39-79
  terminate / terminateVal   ml/boosting/GBMParams.scala:308-326, ml/boosting/BoostingParams.scala:150-177
  persistence                ml/regression/GBMRegressor.scala:120-146,535-593

Per boosting iteration m (GBMRegressor.scala:286-397):
  * the bags of all learners come from one withBag (sbag_sample, k_poisson3 / k_bernoulli:
    the bagging sampler) over the training rows, seed = getSeed;
  * subspace = mkSubspace(subspaceRatio, numFeatures, seed_m), seed_0 = getSeed and
    seed_{m+1} = seed_m + iter_m (the recursion's `seed + iter`);
  * labels = -grad(label, current prediction) in fp64;
  * the booster is DecisionTreeRegressor on extractSubBag(bag m): sbag_fit_booster, whose
    split statistics are fp64 sums in Spark's row order (k_bt_hist / k_bt_partition);
  * weight = learningRate (optimizedWeights = false; the breeze LBFGS-B line search of
    optimizedWeights = true is not reproduced and is refused);
  * current prediction = BLAS.dot(booster predictions, weights) + const: F2J ddot is a
    left-to-right sum of rounded products, kept here as a running sum in booster order.
"""
import os

import numpy as np

from . import _native as nat
from . import persistence as sp
from .libsvm import is_sparse
from .ml import (DecisionTreeModel, DecisionTreeRegressor, Frame, Params, _DecisionTreeEstimator,
                 _in_range01, java_string_hash)

SUPPORTED_LOSSES = ("squared", "absolute", "huber", "quantile")
DOUBLE_MAX = np.finfo(np.float64).max


def loss_function(loss, alpha):
    """GBMRegressorParams.lossFunction (GBMRegressor.scala:93-105), elementwise fp64."""
    if loss == "squared":
        return lambda y, p: (y - p) * (y - p) / 2.0
    if loss == "absolute":
        return lambda y, p: np.abs(y - p)
    if loss == "huber":
        return lambda y, p: (alpha * alpha) * (np.sqrt(1.0 + ((y - p) / alpha) * ((y - p) / alpha)) - 1.0)
    if loss == "quantile":
        return lambda y, p: np.where(p > y, (alpha - 1.0) * (y - p), alpha * (y - p))
    raise RuntimeError(f"Boosting was given bad loss type: {loss}")


def grad_function(loss, alpha):
    """GBMRegressorParams.gradFunction (GBMRegressor.scala:107-118), elementwise fp64."""
    if loss == "squared":
        return lambda y, p: -(y - p)
    if loss == "absolute":  # breeze signum = Math.signum: +-0.0 map to themselves
        return lambda y, p: -np.where((y - p) == 0, y - p, np.sign(y - p))
    if loss == "huber":
        return lambda y, p: -(y - p) / np.sqrt(1.0 + ((y - p) / alpha) * ((y - p) / alpha))
    if loss == "quantile":
        return lambda y, p: np.where(p > y, -(alpha - 1.0), -alpha)
    raise RuntimeError(f"Boosting was given bad loss type: {loss}")


def seq_sum(v):
    """Spark SQL sum() over one partition: a left-to-right fp64 sum (not pairwise)."""
    v = np.asarray(v, np.float64)
    return float(np.cumsum(v)[-1]) if len(v) else 0.0


def terminate_val(with_validation, error, verror, tol, num_round, num_try, it):
    """BoostingParams.terminateVal (BoostingParams.scala:150-177)."""
    if with_validation:
        if verror < error * (1 - tol):
            return it - 1, verror, 0
        if num_try == num_round - 1:
            return 0, 0.0, num_try + 1
        return it - 1, error, num_try + 1
    return it - 1, 0.0, 0


def terminate(weight, learning_rate, with_validation, error, verror, tol, num_round, num_try, it):
    """GBMParams.terminate(weight: Double, ...) (GBMParams.scala:308-326)."""
    if weight < tol * learning_rate:
        return 0, 0.0, 1
    return terminate_val(with_validation, error, verror, tol, num_round, num_try, it)


class _GBMParams(Params):
    _defaults = {"numBaseLearners": 10, "learningRate": 1.0, "tol": 1e-3, "maxIter": 10,
                 "optimizedWeights": False, "loss": "squared", "alpha": 0.9, "numRound": 5,
                 "replacement": False, "sampleRatio": 1.0, "subspaceRatio": 1.0,
                 "validationIndicatorCol": None, "weightCol": None, "baseLearner": None,
                 "labelCol": "label", "featuresCol": "features", "predictionCol": "prediction",
                 "seed": java_string_hash("org.apache.spark.ml.regression.GBMRegressor")}
    _validators = {"numBaseLearners": lambda x: int(x) >= 1,
                   "learningRate": lambda x: float(x) > 0.0,
                   "tol": lambda x: float(x) >= 0.0, "maxIter": lambda x: int(x) >= 0,
                   "numRound": lambda x: int(x) >= 1,
                   "loss": lambda x: str(x).lower() in SUPPORTED_LOSSES,
                   "sampleRatio": _in_range01, "subspaceRatio": _in_range01}

    def getLoss(self):
        return str(self.get("loss")).lower()

    def getAlpha(self):
        return self.get("alpha")

    def getLearningRate(self):
        return self.get("learningRate")

    def getNumBaseLearners(self):
        return self.get("numBaseLearners")

    def getOptimizedWeights(self):
        return self.get("optimizedWeights")

    def getTol(self):
        return self.get("tol")

    def getMaxIter(self):
        return self.get("maxIter")

    def getNumRound(self):
        return self.get("numRound")

    def getSeed(self):
        return self.get("seed")

    def getReplacement(self):
        return self.get("replacement")

    def getSampleRatio(self):
        return self.get("sampleRatio")

    def getSubspaceRatio(self):
        return self.get("subspaceRatio")

    def getBaseLearner(self):
        return self.get("baseLearner")


class GBMRegressionModel(_GBMParams):
    """GBMRegressionModel (GBMRegressor.scala:492-526): weights, subspaces, models, const."""

    _spark_class = "org.apache.spark.ml.regression.GBMRegressionModel"

    def __init__(self, weights, subspaces, models, const, uid=None):
        super().__init__(uid)
        self.weights = [float(w) for w in weights]
        self.subspaces = [np.asarray(s, np.int32) for s in subspaces]
        self.models = list(models)
        self.const = float(const)
        self._forest = None

    @property
    def numBaseModels(self):
        return len(self.models)

    def native_forest(self):
        if self._forest is None:
            self._forest = nat.NativeForest.from_trees([m.nodes for m in self.models],
                                                       self.subspaces, nat.IMPURITY_VARIANCE)
        return self._forest

    def transform(self, dataset, device=0):
        """predict = BLAS.dot(booster predictions, weights) + const per row: the trees are
        walked on the device (k_predict_tiled, per-tree outputs), the dot is F2J ddot's
        left-to-right sum of rounded products."""
        if not self.models:
            n = dataset.shape[0] if isinstance(dataset, nat.DeviceDataset) else len(dataset)
            return np.full(n, 0.0 + self.const)
        if isinstance(dataset, nat.DeviceDataset):
            X = dataset.features()
            ctx = dataset.ctx
        else:
            X = dataset.features if isinstance(dataset, Frame) else dataset
            ctx = nat.default_context(device)
        if is_sparse(X):
            X = X.toarray() if hasattr(X, "toarray") else X.to_dense()
        X = np.asarray(X, np.float64)
        if X.ndim == 1:
            X = X[None, :]
        _, per_tree = nat.predict(ctx, self.native_forest(), X, nat.AGG_MEAN, per_tree=True)
        s = np.zeros(X.shape[0])
        for p, w in zip(per_tree, self.weights):
            s = s + p * w
        return s + self.const

    def predict(self, features):
        return float(self.transform(np.asarray(features, np.float64)[None, :])[0])

    # ---- persistence: GBMRegressionModelWriter (GBMRegressor.scala:535-559)
    def save(self, path):
        if os.path.exists(path):
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"Path {path} already exists. To overwrite it, please use "
                                 "write.overwrite().save(path) for Scala and use "
                                 "write().overwrite().save(path) for Java and Python.")
        params = {k: v for k, v in self.extractParamMap().items()
                  if k != "baseLearner" and v is not None}
        defaults = {k: v for k, v in self._defaults.items() if v is not None and k != "baseLearner"}
        sp.save_metadata(path, self._spark_class, self.uid, params, defaults,
                         {"numBaseModels": self.numBaseModels})
        bl = self.get("baseLearner") or DecisionTreeRegressor()
        bl.save(os.path.join(path, "learner"))
        tree_params = dict(bl._other_params, **bl._values)
        tree_params.update(labelCol=self.get("labelCol"), featuresCol=self.get("featuresCol"),
                           predictionCol=self.get("predictionCol"))
        for i, (m, s, w) in enumerate(zip(self.models, self.subspaces, self.weights)):
            mp = os.path.join(path, f"model-{i}")
            sp.save_metadata(mp, bl._spark_model_class, bl.uid, tree_params, bl._spark_defaults,
                             {"numFeatures": int(len(s))})
            sp.write_tree_data(mp, m.nodes, m.stats)
            sp.write_json_row(os.path.join(path, f"data-{i}"),
                              {"weight": w, "subspace": [int(x) for x in s], "const": self.const})

    @classmethod
    def load(cls, path):
        """GBMRegressionModelReader (GBMRegressor.scala:561-592)."""
        meta = sp.load_metadata(path, cls._spark_class)
        bl = _DecisionTreeEstimator.load(os.path.join(path, "learner"))
        n = int(meta["numBaseModels"])
        models, subs, weights, consts = [], [], [], []
        for i in range(n):
            mp = os.path.join(path, f"model-{i}")
            nodes, stats = sp.read_tree_data(mp)
            models.append(DecisionTreeModel(nodes, stats, nat.IMPURITY_VARIANCE))
            row = sp.read_json_row(os.path.join(path, f"data-{i}"))
            weights.append(float(row["weight"]))
            subs.append(np.asarray(row["subspace"], np.int32))
            consts.append(float(row["const"]))
        m = cls(weights, subs, models, consts[0] if consts else 0.0, uid=meta["uid"])
        for k, v in meta["paramMap"].items():
            if k in m._defaults:
                m._values[k] = v
        m._values["baseLearner"] = bl
        return m


class GBMRegressor(_GBMParams):
    """GBMRegressor (GBMRegressor.scala:150-461) with a DecisionTreeRegressor base learner."""

    _spark_class = "org.apache.spark.ml.regression.GBMRegressor"

    # setters (GBMRegressor.scala:155-186)
    def setWeightCol(self, v):
        return self.set("weightCol", v)

    def setBaseLearner(self, v):
        if not isinstance(v, DecisionTreeRegressor):
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, "the MI355X booster engine fits DecisionTreeRegressor base "
                                 f"learners, got {type(v).__name__}")
        return self.set("baseLearner", v)

    def setNumBaseLearners(self, v):
        return self.set("numBaseLearners", int(v))

    def setLoss(self, v):
        return self.set("loss", v)

    def setAlpha(self, v):
        return self.set("alpha", float(v))

    def setLearningRate(self, v):
        return self.set("learningRate", float(v))

    def setOptimizedWeights(self, v):
        return self.set("optimizedWeights", bool(v))

    def setValidationIndicatorCol(self, v):
        return self.set("validationIndicatorCol", v)

    def setMaxIter(self, v):
        return self.set("maxIter", int(v))

    def setTol(self, v):
        return self.set("tol", float(v))

    def setSeed(self, v):
        return self.set("seed", int(v))

    def copy(self, extra=None):
        other = super().copy(extra)
        if other.get("baseLearner") is not None:
            other._values["baseLearner"] = other.get("baseLearner").copy()
        return other

    def save(self, path):
        """GBMRegressorWriter (GBMRegressorParams.saveImpl, GBMRegressor.scala:120-136)."""
        if os.path.exists(path):
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"Path {path} already exists. To overwrite it, please use "
                                 "write.overwrite().save(path) for Scala and use "
                                 "write().overwrite().save(path) for Java and Python.")
        params = {k: v for k, v in self.extractParamMap().items()
                  if k != "baseLearner" and v is not None}
        defaults = {k: v for k, v in self._defaults.items() if v is not None and k != "baseLearner"}
        sp.save_metadata(path, self._spark_class, self.uid, params, defaults)
        (self.get("baseLearner") or DecisionTreeRegressor()).save(os.path.join(path, "learner"))

    @classmethod
    def load(cls, path):
        meta = sp.load_metadata(path, cls._spark_class)
        est = cls(uid=meta["uid"])
        for k, v in meta["paramMap"].items():
            if k in est._defaults:
                est._values[k] = v
        est._values["baseLearner"] = _DecisionTreeEstimator.load(os.path.join(path, "learner"))
        return est

    def fit(self, dataset, params=None, validation=None):
        """Predictor.fit -> train.  `dataset` is a Frame or (X, y); `validation` is the
        boolean validationIndicatorCol per row (rows flagged True form the validation set,
        GBMRegressor.scala:235-241), used when validationIndicatorCol is set."""
        est = self.copy(params) if params else self
        return est._train(dataset, validation)

    def _train(self, dataset, validation):
        bl = self.get("baseLearner") or DecisionTreeRegressor()
        if self.get("weightCol"):
            import warnings
            warnings.warn(f"weightCol is ignored, as it is not supported by {type(bl).__name__} now.")
        if self.getOptimizedWeights():
            raise nat.SparkException(
                nat.SBAG_EUNSUPPORTED, "optimizedWeights = true (breeze LBFGS-B line search of "
                                       "GBMParams.findOptimizedWeight) is not reproduced")
        frame = dataset if isinstance(dataset, Frame) else Frame(*dataset)
        X = frame.features
        if is_sparse(X):
            X = X.toarray() if hasattr(X, "toarray") else X.to_dense()
        X = np.asarray(X, np.float64)
        y = frame.label
        N, F = X.shape
        with_validation = bool(self.get("validationIndicatorCol"))
        vmask = np.zeros(N, bool)
        if with_validation:
            if validation is None:
                raise nat.IllegalArgumentException(
                    nat.SBAG_EINVAL, "validationIndicatorCol is set but no indicator was given")
            vmask = np.asarray(validation, bool)
        part = frame.partition_offsets or [0, N]
        # the training DataFrame keeps its partitions, minus the validation rows
        tr_idx = np.nonzero(~vmask)[0]
        tpart = [0] + [int((~vmask[part[p]:part[p + 1]]).sum()) for p in range(len(part) - 1)]
        tpart = list(np.cumsum(tpart))
        Xt, yt = X[tr_idx], y[tr_idx]
        Xv, yv = X[vmask], y[vmask]
        Nt = len(yt)
        L = self.getNumBaseLearners()
        lr = self.getLearningRate()
        lossf = loss_function(self.getLoss(), self.getAlpha())
        grad = grad_function(self.getLoss(), self.getAlpha())
        ctx = nat.default_context(0)
        ds = nat.DeviceDataset.from_numpy(Xt, yt, ctx)
        try:
            counts = nat.sample(ctx, self.getReplacement(), self.getSampleRatio(), self.getSeed(),
                                0, L, Nt, tpart if len(tpart) > 2 else None)
            const = 0.0  # findOptimizedConst only with optimizedWeights (refused above)
            weights, subspaces, models = [], [], []
            S = np.zeros(Nt)            # BLAS.dot of the current model on the training rows
            SV = np.zeros(len(yv))      # ... on the validation rows
            it, error, num_try, seed = L, DOUBLE_MAX, 0, self.getSeed()
            while it != 0:
                m = L - it
                sub = nat.subspace(self.getSubspaceRatio(), F, seed)
                if len(sub) == 0:
                    raise nat.IllegalArgumentException(
                        nat.SBAG_EINVAL, "requirement failed: VectorSlicer requires that at least "
                                         "one feature be selected.")
                residual = -grad(yt, S + const)
                f = nat.fit_booster(ctx, ds, residual, counts[m], sub,
                                    partition_offsets=tpart if len(tpart) > 2 else None,
                                    max_depth=bl.getMaxDepth(), max_bins=bl.getMaxBins(),
                                    min_instances_per_node=bl.getMinInstancesPerNode(),
                                    min_info_gain=bl.getMinInfoGain(), tree_seed=bl.getSeed())
                try:
                    nodes, stats = f.tree(0)
                    p = nat.predict_dataset(ctx, f, ds, nat.AGG_MEAN)
                    pv = nat.predict(ctx, f, Xv, nat.AGG_MEAN) if len(yv) else np.zeros(0)
                finally:
                    f.free()
                weight = lr * 1.0
                weights.append(weight)
                subspaces.append(sub)
                models.append(DecisionTreeModel(nodes, stats, nat.IMPURITY_VARIANCE))
                S = S + p * weight
                SV = SV + pv * weight
                verror = seq_sum(lossf(yv, SV + const)) if len(yv) else DOUBLE_MAX
                old_it = it
                it, error, num_try = terminate(weight, lr, with_validation, error, verror,
                                               self.getTol(), self.getNumRound(), num_try, it)
                seed = seed + old_it
            keep = len(models) - num_try
        finally:
            ds.free()
        model = GBMRegressionModel(weights[:keep], subspaces[:keep], models[:keep], const)
        for k in self._defaults:
            model._values[k] = self.get(k)
        model._values["baseLearner"] = bl
        return model


# ====================================================================== GBMClassifier
def divergence_loss(y, p):
    """GBMClassifierParams.lossFunction("divergence") (GBMClassifier.scala:77-81)."""
    return -y * np.log(p)


def divergence_grad(y, p):
    """GBMClassifierParams.gradFunction("divergence") (GBMClassifier.scala:83-87)."""
    return -(y - p)


def softmax_rows(res):
    """GBMClassificationModel.predictRaw's exp(res) / sum(exp(res)) per row
    (GBMClassifier.scala:540-548): breeze's sum is a left-to-right loop over the classes."""
    e = np.exp(res)
    tot = np.zeros(res.shape[0])
    for k in range(res.shape[1]):
        tot = tot + e[:, k]
    return e / tot[:, None]


class GBMClassificationModel(_GBMParams):
    """GBMClassificationModel (GBMClassifier.scala:519-637): weights[m][k], subspaces[m],
    models[m][k]; predictRaw = softmax of the per-class weighted tree sums, prediction its
    first argmax."""

    _spark_class = "org.apache.spark.ml.classification.GBMClassificationModel"
    _defaults = dict(_GBMParams._defaults, loss="divergence", rawPredictionCol="rawPrediction",
                     parallelism=1,
                     seed=java_string_hash("org.apache.spark.ml.classification.GBMClassifier"))
    _validators = dict(_GBMParams._validators, loss=lambda x: str(x).lower() == "divergence")

    def __init__(self, num_classes, weights, subspaces, models, uid=None):
        super().__init__(uid)
        self.numClasses = int(num_classes)
        self.weights = [[float(w) for w in ws] for ws in weights]
        self.subspaces = [np.asarray(s, np.int32) for s in subspaces]
        self.models = [list(ms) for ms in models]
        self._forest = None

    @property
    def numBaseModels(self):
        return len(self.models)

    def native_forest(self):
        """All K * M trees, iteration-major (tree m * K + k)."""
        if self._forest is None:
            trees = [t.nodes for ms in self.models for t in ms]
            subs = [s for s, ms in zip(self.subspaces, self.models) for _ in ms]
            self._forest = nat.NativeForest.from_trees(trees, subs, nat.IMPURITY_VARIANCE)
        return self._forest

    def raw_sums(self, X, ctx):
        """res[:, k] = sum over m (in order) of models[m][k].predict * weights[m][k]."""
        res = np.zeros((X.shape[0], self.numClasses))
        if not self.models:
            return res
        _, pt = nat.predict(ctx, self.native_forest(), X, nat.AGG_MEAN, per_tree=True)
        K = self.numClasses
        for m in range(len(self.models)):
            for k in range(K):
                res[:, k] = res[:, k] + pt[m * K + k] * self.weights[m][k]
        return res

    def predict_raw(self, dataset, device=0):
        X, ctx = _rows_and_ctx(dataset, device)
        return softmax_rows(self.raw_sums(X, ctx))

    def transform(self, dataset, device=0):
        """prediction = rawPrediction.argmax (ClassificationModel.raw2prediction)."""
        return np.argmax(self.predict_raw(dataset, device), axis=1).astype(np.float64)

    def predict(self, features):
        return float(self.transform(np.asarray(features, np.float64)[None, :])[0])

    def save(self, path):
        """GBMClassificationModelWriter (GBMClassifier.scala:568-596): model-$k-$idx and
        data-$k-$idx ({weight, subspace}), metadata with numClasses and numBaseModels."""
        if os.path.exists(path):
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"Path {path} already exists. To overwrite it, please use "
                                 "write.overwrite().save(path) for Scala and use "
                                 "write().overwrite().save(path) for Java and Python.")
        params = {k: v for k, v in self.extractParamMap().items()
                  if k != "baseLearner" and v is not None}
        defaults = {k: v for k, v in self._defaults.items() if v is not None and k != "baseLearner"}
        sp.save_metadata(path, self._spark_class, self.uid, params, defaults,
                         {"numClasses": self.numClasses, "numBaseModels": self.numBaseModels})
        bl = self.get("baseLearner") or DecisionTreeRegressor()
        bl.save(os.path.join(path, "learner"))
        tree_params = dict(bl._other_params, **bl._values)
        for idx, (ms, ws, s) in enumerate(zip(self.models, self.weights, self.subspaces)):
            for k, (m, w) in enumerate(zip(ms, ws)):
                mp = os.path.join(path, f"model-{k}-{idx}")
                sp.save_metadata(mp, bl._spark_model_class, bl.uid, tree_params,
                                 bl._spark_defaults, {"numFeatures": int(len(s))})
                sp.write_tree_data(mp, m.nodes, m.stats)
                sp.write_json_row(os.path.join(path, f"data-{k}-{idx}"),
                                  {"weight": w, "subspace": [int(x) for x in s]})

    @classmethod
    def load(cls, path):
        meta = sp.load_metadata(path, cls._spark_class)
        bl = _DecisionTreeEstimator.load(os.path.join(path, "learner"))
        K, M = int(meta["numClasses"]), int(meta["numBaseModels"])
        models, weights, subs = [], [], []
        for idx in range(M):
            ms, ws = [], []
            for k in range(K):
                nodes, stats = sp.read_tree_data(os.path.join(path, f"model-{k}-{idx}"))
                ms.append(DecisionTreeModel(nodes, stats, nat.IMPURITY_VARIANCE))
                row = sp.read_json_row(os.path.join(path, f"data-{k}-{idx}"))
                ws.append(float(row["weight"]))
                if k == 0:
                    subs.append(np.asarray(row["subspace"], np.int32))
            models.append(ms)
            weights.append(ws)
        m = cls(K, weights, subs, models, uid=meta["uid"])
        for k, v in meta["paramMap"].items():
            if k in m._defaults:
                m._values[k] = v
        m._values["baseLearner"] = bl
        return m


def _rows_and_ctx(dataset, device):
    if isinstance(dataset, nat.DeviceDataset):
        return dataset.features(), dataset.ctx
    X = dataset.features if isinstance(dataset, Frame) else dataset
    if is_sparse(X):
        X = X.toarray()
    X = np.asarray(X, np.float64)
    if X.ndim == 1:
        X = X[None, :]
    return X, nat.default_context(device)


class GBMClassifier(GBMRegressor):
    """GBMClassifier (GBMClassifier.scala:122-486): one DecisionTreeRegressor per class and
    iteration on the residuals of the one-vs-rest labels against the softmax of the current
    model.  Reproduced as the reference runs, including two quirks of its recursion
    (GBMClassifier.scala:441-462): it passes `numTry` where `numRound` goes, and the same
    `seed` every iteration (so every iteration draws the same subspace)."""

    _spark_class = "org.apache.spark.ml.classification.GBMClassifier"
    _defaults = GBMClassificationModel._defaults
    _validators = GBMClassificationModel._validators

    def setLoss(self, v):
        return self.set("loss", v)

    def setParallelism(self, v):
        return self.set("parallelism", int(v))

    def _train(self, dataset, validation):
        bl = self.get("baseLearner") or DecisionTreeRegressor()
        if self.get("weightCol"):
            import warnings
            warnings.warn(f"weightCol is ignored, as it is not supported by {type(bl).__name__} now.")
        if self.getOptimizedWeights():
            raise nat.SparkException(
                nat.SBAG_EUNSUPPORTED, "optimizedWeights = true (breeze LBFGS-B line search of "
                                       "GBMParams.findOptimizedWeight) is not reproduced")
        frame = dataset if isinstance(dataset, Frame) else Frame(*dataset)
        X = frame.features.toarray() if is_sparse(frame.features) else np.asarray(frame.features)
        X = np.asarray(X, np.float64)
        y = frame.label
        N, F = X.shape
        K = int(y.max()) + 1 if N else 0  # computeNumClasses: max label + 1
        bad = ~((y == np.floor(y)) & (y >= 0) & (y < K))
        if bad.any():
            raise nat.IllegalArgumentException(
                nat.SBAG_EINVAL, f"Classifier was given dataset with invalid label {y[bad][0]}.  "
                                 f"Labels must be integers in range [0, {K}).")
        with_validation = bool(self.get("validationIndicatorCol"))
        vmask = np.zeros(N, bool)
        if with_validation:
            if validation is None:
                raise nat.IllegalArgumentException(
                    nat.SBAG_EINVAL, "validationIndicatorCol is set but no indicator was given")
            vmask = np.asarray(validation, bool)
        part = frame.partition_offsets or [0, N]
        tpart = [0] + [int((~vmask[part[p]:part[p + 1]]).sum()) for p in range(len(part) - 1)]
        tpart = list(np.cumsum(tpart))
        tr = ~vmask
        Xt, yt, Xv, yv = X[tr], y[tr], X[vmask], y[vmask]
        Nt = len(yt)
        L = self.getNumBaseLearners()
        lr = self.getLearningRate()
        ctx = nat.default_context(0)
        ds = nat.DeviceDataset.from_numpy(Xt, yt, ctx)
        try:
            counts = nat.sample(ctx, self.getReplacement(), self.getSampleRatio(), self.getSeed(),
                                0, L, Nt, tpart if len(tpart) > 2 else None)
            weights, subspaces, models = [], [], []
            res = np.zeros((Nt, K))
            resv = np.zeros((len(yv), K))
            it, error, num_try = L, DOUBLE_MAX, 0
            num_round, seed = self.getNumRound(), self.getSeed()
            while it != 0:
                m = L - it
                sub = nat.subspace(self.getSubspaceRatio(), F, seed)
                if len(sub) == 0:
                    raise nat.IllegalArgumentException(
                        nat.SBAG_EINVAL, "requirement failed: VectorSlicer requires that at least "
                                         "one feature be selected.")
                prob = softmax_rows(res)
                ws, ms, preds, predv = [], [], [], []
                for k in range(K):  # the reference's per-class Futures, joined in class order
                    relabeled = np.where(yt == k, 1.0, 0.0)
                    residual = -divergence_grad(relabeled, prob[:, k])
                    f = nat.fit_booster(ctx, ds, residual, counts[m], sub,
                                        partition_offsets=tpart if len(tpart) > 2 else None,
                                        max_depth=bl.getMaxDepth(), max_bins=bl.getMaxBins(),
                                        min_instances_per_node=bl.getMinInstancesPerNode(),
                                        min_info_gain=bl.getMinInfoGain(), tree_seed=bl.getSeed())
                    try:
                        nodes, stats = f.tree(0)
                        preds.append(nat.predict_dataset(ctx, f, ds, nat.AGG_MEAN))
                        predv.append(nat.predict(ctx, f, Xv, nat.AGG_MEAN) if len(yv) else np.zeros(0))
                    finally:
                        f.free()
                    ws.append(lr * 1.0)
                    ms.append(DecisionTreeModel(nodes, stats, nat.IMPURITY_VARIANCE))
                weights.append(ws)
                subspaces.append(sub)
                models.append(ms)
                for k in range(K):
                    res[:, k] = res[:, k] + preds[k] * ws[k]
                    resv[:, k] = resv[:, k] + predv[k] * ws[k]
                if len(yv):  # evaluateOnValidation: per class SQL sum, then Array.sum
                    pv = softmax_rows(resv)
                    verror = 0.0
                    for k in range(K):
                        verror = verror + seq_sum(divergence_loss(np.where(yv == k, 1.0, 0.0), pv[:, k]))
                else:
                    verror = DOUBLE_MAX
                # GBMParams.terminate(weights: Array[Double], ...)
                if all(w < self.getTol() * lr for w in ws):
                    nxt = (0, 0.0, 1)
                else:
                    nxt = terminate_val(with_validation, error, verror, self.getTol(), num_round,
                                        num_try, it)
                num_round = num_try  # the recursion passes numTry as numRound
                it, error, num_try = nxt
            keep = len(models) - num_try
        finally:
            ds.free()
        model = GBMClassificationModel(K, weights[:keep], subspaces[:keep], models[:keep])
        for k in self._defaults:
            model._values[k] = self.get(k)
        model._values["baseLearner"] = bl
        return model
