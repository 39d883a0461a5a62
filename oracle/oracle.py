"""ctypes front-end to the C oracle (oracle/lib/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product (spark-bagging_amd/).
PARITY UNPINNED (see oracle/sbag_oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "liboracle.so")

DEFAULT_SEED_REGRESSOR = -1395689524   # "org.apache.spark.ml.regression.BaggingRegressor".hashCode
DEFAULT_SEED_CLASSIFIER = 42087812     # "org.apache.spark.ml.classification.BaggingClassifier".hashCode
# base learners' HasSeed defaults (class-name hashCode): seed of the split-finding sample
DT_SEED_REGRESSOR = 926680331          # "org.apache.spark.ml.regression.DecisionTreeRegressor"
DT_SEED_CLASSIFIER = 159147643         # "org.apache.spark.ml.classification.DecisionTreeClassifier"


class TreeParams(ctypes.Structure):
    _fields_ = [("max_depth", ctypes.c_int32), ("max_bins", ctypes.c_int32),
                ("min_instances_per_node", ctypes.c_int32), ("impurity", ctypes.c_int32),
                ("min_info_gain", ctypes.c_double), ("seed", ctypes.c_int64),
                ("part_off", ctypes.c_void_p), ("num_partitions", ctypes.c_int32),
                ("pad_", ctypes.c_int32)]


NODE_DTYPE = np.dtype([("id", "<i4"), ("left", "<i4"), ("right", "<i4"), ("feature", "<i4"),
                       ("split_bin", "<i4"), ("pad", "<i4"), ("threshold", "<f8"),
                       ("prediction", "<f8"), ("impurity", "<f8"), ("gain", "<f8")])

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i32, i64, dbl = ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        L.or_hash_seed.restype = ctypes.c_uint64
        L.or_hash_seed.argtypes = [i64]
        L.or_xorshift_next.argtypes = [i64, i32, i32, P]
        L.or_xorshift_doubles.argtypes = [i64, i32, P]
        L.or_well_next.argtypes = [i64, i32, i32, P]
        L.or_well_doubles.argtypes = [i64, i32, P]
        L.or_poisson.argtypes = [dbl, i64, i32, P]
        L.or_bag.argtypes = [i32, dbl, i32, i32, i64, P, i32, i64, P]
        L.or_subspace.argtypes = [dbl, i32, i64, P, P]
        L.or_find_splits.argtypes = [P, i64, i32, i32, P, i32, P, P]
        L.or_fit.argtypes = [P, P, i64, i32, P, i32, P, P, ctypes.POINTER(TreeParams), i32,
                             P, i32, P, i32, P, P, P]
        L.or_predict.argtypes = [P, i64, i32, i32, P, P, P, i32, i32, P, P]
        L.or_split_sample_fraction.restype = dbl
        L.or_split_sample_fraction.argtypes = [i64, i32]
        L.or_split_sample_seeds.argtypes = [i64, i32, P]
        L.or_split_sample.restype = i64
        L.or_split_sample.argtypes = [P, P, i32, i64, dbl, P]
        L.or_fit_x.argtypes = [P, i32, P, i64, i32, P, i32, P, P, ctypes.POINTER(TreeParams), i32,
                               P, i32, P, i32, P, P, P]
        L.or_synth.argtypes = [i64, i64, i32, ctypes.c_uint64, i32, i32, P, P]
        L.or_fastmath_exp_neg.restype = dbl
        L.or_fastmath_exp_neg.argtypes = [dbl]
        L.or_mm3_bytes_hash.restype = ctypes.c_uint32
        L.or_mm3_bytes_hash.argtypes = [P, i32, ctypes.c_uint32]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def hash_seed(seed):
    return int(lib().or_hash_seed(seed))


def xorshift_next(seed, bits, n):
    out = np.zeros(n, np.int32)
    lib().or_xorshift_next(seed, bits, n, _p(out))
    return out


def xorshift_doubles(seed, n):
    out = np.zeros(n, np.float64)
    lib().or_xorshift_doubles(seed, n, _p(out))
    return out


def well_next(seed, bits, n):
    out = np.zeros(n, np.int32)
    lib().or_well_next(seed, bits, n, _p(out))
    return out


def well_doubles(seed, n):
    out = np.zeros(n, np.float64)
    lib().or_well_doubles(seed, n, _p(out))
    return out


def poisson(lam, seed, n):
    out = np.zeros(n, np.int32)
    lib().or_poisson(lam, seed, n, _p(out))
    return out


def bag(replacement, ratio, learner_begin, learner_end, seed, part_off, n):
    part_off = np.ascontiguousarray(part_off, dtype=np.int64)
    out = np.zeros((learner_end - learner_begin, n), np.uint8)
    rc = lib().or_bag(int(replacement), float(ratio), learner_begin, learner_end, seed,
                      _p(part_off), len(part_off) - 1, n, _p(out))
    if rc:
        raise ValueError(f"or_bag failed rc={rc}")
    return out


def subspace(ratio, nfeat, seed):
    idx = np.zeros(max(nfeat, 1), np.int32)
    n = np.zeros(1, np.int32)
    lib().or_subspace(float(ratio), nfeat, seed, _p(idx), _p(n))
    return idx[: n[0]].copy()


def find_splits(X, counts, feature, max_bins):
    X = np.ascontiguousarray(X, np.float64)
    counts = np.ascontiguousarray(counts, np.uint8)
    thr = np.zeros(max_bins, np.float64)
    ex = np.zeros(1, np.int32)
    nt = lib().or_find_splits(_p(X), X.shape[0], X.shape[1], feature, _p(counts), max_bins,
                              _p(thr), _p(ex))
    return thr[:nt].copy(), bool(ex[0])


class Forest:
    """Oracle forest: per-learner pre-order node arrays (NodeData layout)."""

    def __init__(self, nodes, stats, num_nodes, num_stats, subspaces, exact):
        self.nodes, self.stats = nodes, stats
        self.num_nodes, self.num_stats = num_nodes, num_stats
        self.subspaces, self.exact = subspaces, exact

    def tree(self, l):
        n = int(self.num_nodes[l])
        return self.nodes[l, :n], self.stats[l, :n, : int(self.num_stats[l])]


def split_sample_fraction(num_examples, max_bins):
    return lib().or_split_sample_fraction(int(num_examples), int(max_bins))


def split_sample_seeds(dt_seed, P):
    out = np.zeros(P, np.int64)
    lib().or_split_sample_seeds(int(dt_seed), int(P), _p(out))
    return out


def split_sample(counts_row, part_off, dt_seed, fraction):
    """Multiplicity of each row of one replica's subbag in RandomForest.findSplits'
    sample (sbag_oracle.c or_split_sample)."""
    c = np.ascontiguousarray(counts_row, np.uint8)
    off = np.ascontiguousarray(part_off, np.int64)
    mult = np.zeros(len(c), np.uint16)
    lib().or_split_sample(_p(c), _p(off), len(off) - 1, int(dt_seed), float(fraction), _p(mult))
    return mult


def fastmath_exp_neg(x):
    """commons-math3 FastMath.exp(x) for -41 < x < 0 (or_fastmath.h)."""
    return float(lib().or_fastmath_exp_neg(float(x)))


def mm3_bytes_hash(data, seed):
    """scala.util.hashing.MurmurHash3.bytesHash (= MurmurHash3_x86_32) of a bytes object."""
    buf = np.frombuffer(bytes(data), np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
    return int(lib().or_mm3_bytes_hash(_p(buf), len(data), seed & 0xFFFFFFFF))


def synth(num_rows, num_features, seed=20261015, num_classes=0, row_begin=0, nthreads=None):
    """The synthetic bench rows as u8 codes [N][F] + fp64 labels."""
    X = np.empty((num_rows, num_features), np.uint8)
    y = np.empty(num_rows, np.float64)
    lib().or_synth(row_begin, num_rows, num_features, seed, num_classes,
                   nthreads or os.cpu_count() or 1, _p(X), _p(y))
    return X, y


def fit(X, y, counts, subspaces, max_depth=5, max_bins=32, min_instances_per_node=1,
        min_info_gain=0.0, classification=False, nthreads=None, max_stats=None, part=None,
        dt_seed=None):
    """Fit one tree per row of counts.  X is fp64 [N][F], or u8 value codes whose fp64 value
    is the code (the synthetic workload)."""
    xkind = 1 if np.asarray(X).dtype == np.uint8 else 0
    X = np.ascontiguousarray(X, np.uint8 if xkind else np.float64)
    y = np.ascontiguousarray(y, np.float64)
    counts = np.ascontiguousarray(counts, np.uint8)
    L, N = counts.shape
    F = X.shape[1]
    sub = np.zeros((L, F), np.int32)
    nsub = np.zeros(L, np.int32)
    for l, s in enumerate(subspaces):
        sub[l, : len(s)] = s
        nsub[l] = len(s)
    # a leaf holds at least one distinct row: <= 2N - 1 nodes whatever the depth
    max_nodes = min((1 << (max_depth + 1)) - 1, 2 * N + 1)
    if max_stats is None:
        max_stats = 3 if not classification else int(y.max()) + 1
    nodes = np.zeros((L, max_nodes), NODE_DTYPE)
    stats = np.zeros((L, max_nodes, max_stats), np.float64)
    num_nodes = np.zeros(L, np.int32)
    num_stats = np.zeros(L, np.int32)
    exact = np.zeros(L, np.int32)
    if dt_seed is None:
        dt_seed = DT_SEED_CLASSIFIER if classification else DT_SEED_REGRESSOR
    off = np.ascontiguousarray(part if part is not None else [0, N], np.int64)
    p = TreeParams(max_depth, max_bins, min_instances_per_node, 1 if classification else 0,
                   min_info_gain, int(dt_seed), off.ctypes.data, len(off) - 1, 0)
    rc = lib().or_fit_x(_p(X), xkind, _p(y), N, F, _p(counts), L, _p(sub), _p(nsub),
                        ctypes.byref(p), nthreads or os.cpu_count() or 1, _p(nodes), max_nodes,
                        _p(stats), max_stats, _p(num_nodes), _p(num_stats), _p(exact))
    if rc:
        raise ValueError(f"or_fit failed rc={rc}")
    return Forest(nodes, stats, num_nodes, num_stats, [np.asarray(s, np.int32) for s in subspaces],
                  exact.astype(bool))


def predict(forest, X, classification=False, per_tree=False):
    X = np.ascontiguousarray(X, np.float64)
    N, F = X.shape
    L = forest.nodes.shape[0]
    sub = np.zeros((L, F), np.int32)
    nsub = np.zeros(L, np.int32)
    for l, s in enumerate(forest.subspaces):
        sub[l, : len(s)] = s
        nsub[l] = len(s)
    out = np.zeros(N, np.float64)
    pt = np.zeros((L, N), np.float64) if per_tree else None
    lib().or_predict(_p(X), N, F, L, _p(sub), _p(nsub), _p(forest.nodes), forest.nodes.shape[1],
                     1 if classification else 0, _p(out), _p(pt) if per_tree else None)
    return (out, pt) if per_tree else out


# ---------------------------------------------------------------- GBMRegressor
_DOUBLE_MAX = np.finfo(np.float64).max
DEFAULT_SEED_GBM_REGRESSOR = 1243996765  # "org.apache.spark.ml.regression.GBMRegressor".hashCode


def _gbm_grad(loss, alpha):
    """GBMRegressorParams.gradFunction (ml/regression/GBMRegressor.scala:107-118)."""
    def signum(d):  # Math.signum: NaN and +-0.0 map to themselves
        return np.where(d == 0, d, np.sign(d))
    return {
        "squared": lambda y, p: -(y - p),
        "absolute": lambda y, p: -signum(y - p),
        "huber": lambda y, p: -(y - p) / np.sqrt(1 + ((y - p) / alpha) * ((y - p) / alpha)),
        "quantile": lambda y, p: np.where(p > y, -(alpha - 1.0), -alpha),
    }[loss]


def _gbm_loss(loss, alpha):
    """GBMRegressorParams.lossFunction (ml/regression/GBMRegressor.scala:93-105)."""
    return {
        "squared": lambda y, p: (y - p) * (y - p) / 2.0,
        "absolute": lambda y, p: np.abs(y - p),
        "huber": lambda y, p: (alpha * alpha) * (np.sqrt(1.0 + ((y - p) / alpha) * ((y - p) / alpha)) - 1.0),
        "quantile": lambda y, p: np.where(p > y, (alpha - 1.0) * (y - p), alpha * (y - p)),
    }[loss]


def gbm_regressor_fit(X, y, *, num_base_learners=10, learning_rate=1.0, loss="squared",
                      alpha=0.9, replacement=False, sample_ratio=1.0, subspace_ratio=1.0,
                      seed=DEFAULT_SEED_GBM_REGRESSOR, tol=1e-3, num_round=5, max_depth=5,
                      max_bins=32, min_instances_per_node=1, min_info_gain=0.0, dt_seed=None,
                      validation=None, nthreads=None):
    """GBMRegressor.train with optimizedWeights = false (ml/regression/GBMRegressor.scala:
    196-456): withBag over the training rows (seed), then per iteration m mkSubspace(
    subspaceRatio, F, seed_m) with seed_{m+1} = seed_m + iter_m, residuals -grad(label,
    dot(predictions, weights) + const), DecisionTreeRegressor on extractSubBag(bag m)
    (this oracle's fit, fp64 sums in row order), weight = learningRate, and
    terminate / terminateVal (ml/boosting/GBMParams.scala:308-326,
    ml/boosting/BoostingParams.scala:150-177).  One partition.
    Returns (weights, subspaces, trees [(nodes, stats)], const)."""
    X = np.ascontiguousarray(X, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    vmask = np.zeros(len(y), bool) if validation is None else np.asarray(validation, bool)
    with_validation = validation is not None
    Xt, yt, Xv, yv = X[~vmask], y[~vmask], X[vmask], y[vmask]
    Nt, F = Xt.shape
    grad, lossf = _gbm_grad(loss, alpha), _gbm_loss(loss, alpha)
    counts = bag(replacement, sample_ratio, 0, num_base_learners, seed, [0, Nt], Nt)
    const = 0.0
    weights, subs, trees = [], [], []
    S, SV = np.zeros(Nt), np.zeros(len(yv))
    it, error, num_try, s = num_base_learners, _DOUBLE_MAX, 0, seed
    while it != 0:
        m = num_base_learners - it
        sub = subspace(subspace_ratio, F, s)
        r = -grad(yt, S + const)
        f = fit(Xt, r, counts[m:m + 1], [sub], max_depth=max_depth, max_bins=max_bins,
                min_instances_per_node=min_instances_per_node, min_info_gain=min_info_gain,
                nthreads=nthreads, dt_seed=dt_seed)
        w = learning_rate * 1.0
        _, p = predict(f, Xt, per_tree=True)
        S = S + p[0] * w
        if len(yv):
            _, pv = predict(f, Xv, per_tree=True)
            SV = SV + pv[0] * w
            verror = float(np.cumsum(lossf(yv, SV + const))[-1])  # SQL sum, left to right
        else:
            verror = _DOUBLE_MAX
        weights.append(w)
        subs.append(sub)
        trees.append(f.tree(0))
        old = it
        if w < tol * learning_rate:
            it, error, num_try = 0, 0.0, 1
        elif with_validation:
            if verror < error * (1 - tol):
                it, error, num_try = it - 1, verror, 0
            elif num_try == num_round - 1:
                it, error, num_try = 0, 0.0, num_try + 1
            else:
                it, num_try = it - 1, num_try + 1
        else:
            it, error, num_try = it - 1, 0.0, 0
        s = s + old
    keep = len(trees) - num_try
    return weights[:keep], subs[:keep], trees[:keep], const


def gbm_predict(weights, subspaces, trees, const, X):
    """GBMRegressionModel.predict: BLAS.dot(tree predictions, weights) + const, the dot a
    left-to-right sum of rounded products (F2J ddot)."""
    X = np.ascontiguousarray(X, np.float64)
    L = len(trees)
    if L == 0:
        return np.full(X.shape[0], 0.0 + const)
    width = max(len(t[0]) for t in trees)
    nodes = np.zeros((L, width), NODE_DTYPE)
    for l, (n, _) in enumerate(trees):
        nodes[l, : len(n)] = n
    f = Forest(nodes, np.zeros((L, width, 3)), np.array([len(t[0]) for t in trees], np.int32),
               np.full(L, 3, np.int32), [np.asarray(s, np.int32) for s in subspaces], np.ones(L, bool))
    _, pt = predict(f, X, per_tree=True)
    acc = np.zeros(X.shape[0])
    for p, w in zip(pt, weights):
        acc = acc + p * w
    return acc + const


DEFAULT_SEED_GBM_CLASSIFIER = -1593632877  # "org.apache.spark.ml.classification.GBMClassifier".hashCode


def _softmax_rows(res):
    """exp(res) / breeze sum(exp(res)) (GBMClassificationModel.predictRaw,
    ml/classification/GBMClassifier.scala:540-548); the class sum left to right."""
    e = np.exp(res)
    tot = np.zeros(res.shape[0])
    for k in range(res.shape[1]):
        tot = tot + e[:, k]
    return e / tot[:, None]


def gbm_classifier_fit(X, y, *, num_base_learners=10, learning_rate=1.0, replacement=False,
                       sample_ratio=1.0, subspace_ratio=1.0, seed=DEFAULT_SEED_GBM_CLASSIFIER,
                       tol=1e-3, num_round=5, max_depth=5, max_bins=32, min_instances_per_node=1,
                       min_info_gain=0.0, dt_seed=None, validation=None, nthreads=None):
    """GBMClassifier.train, loss "divergence", optimizedWeights = false
    (ml/classification/GBMClassifier.scala:190-482): per iteration and class k, residuals
    -grad(1{label == k}, softmax(res)_k) = 1{label == k} - p_k, one DecisionTreeRegressor
    on extractSubBag(bag m), weight learningRate; res_k += tree * weight.  The recursion
    (:441-462) keeps `seed` fixed and passes numTry as numRound; terminate on all K weights
    (ml/boosting/GBMParams.scala:288-306).  Returns (numClasses, weights[m][k],
    subspaces[m], trees[m][k])."""
    X = np.ascontiguousarray(X, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    K = int(y.max()) + 1
    vmask = np.zeros(len(y), bool) if validation is None else np.asarray(validation, bool)
    with_validation = validation is not None
    Xt, yt, Xv, yv = X[~vmask], y[~vmask], X[vmask], y[vmask]
    Nt, F = Xt.shape
    counts = bag(replacement, sample_ratio, 0, num_base_learners, seed, [0, Nt], Nt)
    weights, subs, trees = [], [], []
    res, resv = np.zeros((Nt, K)), np.zeros((len(yv), K))
    it, error, num_try, nround = num_base_learners, _DOUBLE_MAX, 0, num_round
    while it != 0:
        m = num_base_learners - it
        sub = subspace(subspace_ratio, F, seed)
        prob = _softmax_rows(res)
        ws, ts, p_tr, p_v = [], [], [], []
        for k in range(K):
            lab = np.where(yt == k, 1.0, 0.0)
            r = -(-(lab - prob[:, k]))
            f = fit(Xt, r, counts[m:m + 1], [sub], max_depth=max_depth, max_bins=max_bins,
                    min_instances_per_node=min_instances_per_node, min_info_gain=min_info_gain,
                    nthreads=nthreads, dt_seed=dt_seed)
            p_tr.append(predict(f, Xt, per_tree=True)[1][0])
            p_v.append(predict(f, Xv, per_tree=True)[1][0] if len(yv) else np.zeros(0))
            ws.append(learning_rate * 1.0)
            ts.append(f.tree(0))
        for k in range(K):
            res[:, k] = res[:, k] + p_tr[k] * ws[k]
            resv[:, k] = resv[:, k] + p_v[k] * ws[k]
        weights.append(ws)
        subs.append(sub)
        trees.append(ts)
        if len(yv):
            pv = _softmax_rows(resv)
            verror = 0.0
            for k in range(K):
                lab = np.where(yv == k, 1.0, 0.0)
                verror = verror + float(np.cumsum(-lab * np.log(pv[:, k]))[-1])
        else:
            verror = _DOUBLE_MAX
        if all(w < tol * learning_rate for w in ws):
            nxt = (0, 0.0, 1)
        elif with_validation:
            if verror < error * (1 - tol):
                nxt = (it - 1, verror, 0)
            elif num_try == nround - 1:
                nxt = (0, 0.0, num_try + 1)
            else:
                nxt = (it - 1, error, num_try + 1)
        else:
            nxt = (it - 1, 0.0, 0)
        nround = num_try
        it, error, num_try = nxt
    keep = len(trees) - num_try
    return K, weights[:keep], subs[:keep], trees[:keep]


def gbm_classifier_predict(K, weights, subspaces, trees, X):
    """(softmax probabilities [N, K], predictions = first argmax)."""
    X = np.ascontiguousarray(X, np.float64)
    res = np.zeros((X.shape[0], K))
    for ws, s, ts in zip(weights, subspaces, trees):
        for k in range(K):
            p = gbm_predict([1.0], [s], [ts[k]], 0.0, X)  # 0 + p * 1.0 + 0.0 == p
            res[:, k] = res[:, k] + p * ws[k]
    prob = _softmax_rows(res)
    return prob, np.argmax(prob, axis=1).astype(np.float64)
