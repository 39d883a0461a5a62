"""GPU: sparse (CSR) and columnar ingest (sbag_dataset_create_csr / _columns).

The reference trains on SparseVector rows -- spark.read.format("libsvm") yields them,
and HasSubBag.slicer slices them (ml/ensemble/HasSubBag.scala:128-131) -- so the engine
takes CSR without a dense copy.  A dataset built from CSR or from columns must be the
same dataset as the dense one: same value codes, and fits / predictions bit-exact
against the dense path and the oracle, including explicit zeros, -0.0, empty rows,
negative values (0.0 not the smallest code) and features absent from every row."""
import os

import numpy as np
import pytest

import oracle
from conftest import DATA

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = nat.Context(0)
    yield c
    c.close()


def _csr(X, drop_zeros=True, explicit_zero_frac=0.0, rng=None):
    """CSR of X; optionally keep some zeros explicit (as 0.0 or -0.0)."""
    indptr, indices, values = [0], [], []
    for row in X:
        for j, v in enumerate(row):
            keep = v != 0.0 or (rng is not None and rng.random() < explicit_zero_frac)
            if keep or not drop_zeros:
                indices.append(j)
                values.append(v if v != 0.0 or rng is None or rng.random() < 0.5 else -0.0)
        indptr.append(len(indices))
    return sb.SparseRows(indptr, indices, values, X.shape)


def _fit(ctx, ds, cls, L=5, ratio=0.8, part=None):
    seed = oracle.DEFAULT_SEED_CLASSIFIER if cls else oracle.DEFAULT_SEED_REGRESSOR
    return nat.fit(ctx, ds, replacement=True, sample_ratio=ratio, seed=seed, learner_begin=0,
                   learner_end=L, partition_offsets=part, max_depth=6, max_bins=32,
                   impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)


def _same_forest(a, b):
    assert len(a) == len(b)
    for t in range(len(a)):
        (na, sa), (nb, sb_) = a.tree(t), b.tree(t)
        assert na.tobytes() == nb.tobytes(), f"tree {t}"
        assert (sa == sb_).all()


def test_vehicle_libsvm_as_csr(ctx):
    """vehicle.svm read as Spark reads it (SparseVector rows) fits bit-exact against the
    dense path and the oracle; transform of the sparse rows equals the oracle's votes."""
    X, y = sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))
    S, _ = sb.load_libsvm(os.path.join(DATA, "vehicle.svm"), sparse=True)
    dd = nat.DeviceDataset.from_numpy(X, y, ctx)
    ds = nat.DeviceDataset.from_csr(S, y, ctx)
    np.testing.assert_array_equal(ds.features(), X)
    fd, fs = _fit(ctx, dd, True), _fit(ctx, ds, True)
    _same_forest(fd, fs)
    seed = oracle.DEFAULT_SEED_CLASSIFIER
    counts = oracle.bag(True, 0.8, 0, 5, seed, [0, len(y)], len(y))
    subs = [oracle.subspace(0.8, X.shape[1], seed + i) for i in range(5)]
    orf = oracle.fit(X, y, counts, subs, max_depth=6, max_bins=32, classification=True)
    for t in range(5):
        assert fs.tree(t)[0]["threshold"].tobytes() == orf.tree(t)[0]["threshold"].tobytes()
    want = oracle.predict(orf, X, classification=True)
    np.testing.assert_array_equal(nat.predict_dataset(ctx, fs, ds, nat.AGG_MODE), want)
    # the Spark-API mirror keeps the rows sparse end to end
    est = (sb.BaggingClassifier().setBaseLearner(sb.DecisionTreeClassifier().setMaxDepth(6))
           .setNumBaseLearners(5).setReplacement(True).setSampleRatio(0.8))
    model = est.fit(sb.Frame(S, y))
    np.testing.assert_array_equal(model.transform(S), want)
    np.testing.assert_array_equal(model.transform(X), want)
    for f in (fd, fs):
        f.free()
    dd.free()
    ds.free()


@pytest.mark.parametrize("cls", [False, True])
def test_sparse_edge_cases_match_dense(ctx, cls):
    rng = np.random.default_rng(11 + cls)
    N, F = 5000, 14
    X = np.round(rng.normal(size=(N, F)), 1)
    X[rng.random((N, F)) < 0.7] = 0.0       # mostly sparse
    X[:, 3] = np.abs(X[:, 3])                # 0.0 is code 0 here
    X[:, 9] = 0.0                            # never present
    X[:, 11] = rng.integers(1, 4, N)         # never zero: dense column in CSR
    X[100:140] = 0.0                         # empty rows
    y = (rng.integers(0, 5, N) if cls else rng.integers(-64, 64, N) / 8).astype(np.float64)
    S = _csr(X, explicit_zero_frac=0.05, rng=rng)  # some explicit 0.0 / -0.0 entries
    assert (S.toarray() == X).all()
    dd = nat.DeviceDataset.from_numpy(X, y, ctx)
    ds = nat.DeviceDataset.from_csr(S, y, ctx)
    np.testing.assert_array_equal(ds.features(), dd.features())
    part = [0, 1700, 5000]
    fd, fs = _fit(ctx, dd, cls, part=part), _fit(ctx, ds, cls, part=part)
    _same_forest(fd, fs)
    seed = oracle.DEFAULT_SEED_CLASSIFIER if cls else oracle.DEFAULT_SEED_REGRESSOR
    counts = oracle.bag(True, 0.8, 0, 5, seed, part, N)
    subs = [oracle.subspace(0.8, F, seed + i) for i in range(5)]
    orf = oracle.fit(X, y, counts, subs, max_depth=6, max_bins=32, classification=cls, part=part)
    for t in range(5):
        on, _ = orf.tree(t)
        nn, _ = fs.tree(t)
        for k in ("left", "right", "feature", "threshold", "prediction", "impurity", "gain"):
            assert (nn[k] == on[k]).all(), (t, k)
    agg = nat.AGG_MODE if cls else nat.AGG_MEAN
    np.testing.assert_array_equal(nat.predict_dataset(ctx, fs, ds, agg),
                                  oracle.predict(orf, X, classification=cls))
    for f in (fd, fs):
        f.free()
    dd.free()
    ds.free()


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.uint8])
def test_columnar_ingest_matches_dense(ctx, dtype):
    rng = np.random.default_rng(5)
    N, F = 4000, 9
    if dtype == np.uint8:
        Xc = rng.integers(0, 40, size=(N, F)).astype(np.uint8)
    else:
        Xc = np.round(rng.normal(size=(N, F)), 2).astype(dtype)
    X = Xc.astype(np.float64)
    y = rng.integers(0, 3, N).astype(np.float64)
    cols = [np.ascontiguousarray(Xc[:, f]) for f in range(F)]
    dc = nat.DeviceDataset.from_columns(cols, y, ctx)
    dd = nat.DeviceDataset.from_numpy(X, y, ctx)
    np.testing.assert_array_equal(dc.features(), X)
    _same_forest(_fit(ctx, dd, True), _fit(ctx, dc, True))
    dc.free()
    dd.free()


def test_bad_sparse_input_is_illegal_argument(ctx):
    y = np.zeros(2)
    for ind in ([1, 0], [0, 0], [0, 7]):  # decreasing, repeated, out of range
        S = sb.SparseRows([0, 2, 2], ind, [1.0, 2.0], (2, 5))
        with pytest.raises(sb.IllegalArgumentException):
            nat.DeviceDataset.from_csr(S, y, ctx)
    S = sb.SparseRows([0, 1, 1], [0], [float("nan")], (2, 5))
    with pytest.raises(sb.IllegalArgumentException):
        nat.DeviceDataset.from_csr(S, y, ctx)
    with pytest.raises(sb.IllegalArgumentException):
        nat.DeviceDataset.from_columns([np.zeros(2), np.zeros(2, np.float32)], y, ctx)
