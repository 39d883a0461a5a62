"""GPU parity at the benchmarked configurations (BASELINE.json configs[2..4]).

bench.py times C3 (10M x 100, 128 partitions, 128 learners, depth 8) and one GPU's shard
of C4 / C5.  These tests run exactly those fits through the C ABI and compare chosen
learners bit-exact against oracle fits of just those learners: learners are independent
(ml/regression/BaggingRegressor.scala:163-191 fits each from its own bag column and
subspace), so the oracle can fit a subset.  Every other tree of the fit is checked through
size-independent properties (pre-order links, parent stats = left + right, leaf
predictions from their stats, root count = the learner's bag size).

Data: the synthetic workload of SURVEY.md §8d, generated on the device by the product
(k_synth) and on the host by oracle.synth; the two are compared first.
"""
import os

import numpy as np
import pytest

import oracle
from parity_utils import assert_tree_equal

from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu

SEED_REG = oracle.DEFAULT_SEED_REGRESSOR
SEED_CLS = oracle.DEFAULT_SEED_CLASSIFIER
DATA_SEED = 20261015  # bench.py --seed
P = 128               # bench.py --partitions
NTHREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def ctx():
    c = nat.Context(0)
    yield c
    c.close()


def _partitions(n, p=P):
    return [int(round(i * n / p)) for i in range(p + 1)]


def _dataset(ctx, n, f, classes):
    """Device synthetic rows + the oracle's host copy; the product's generator must agree."""
    ds = nat.DeviceDataset.synthetic(n, f, seed=DATA_SEED, num_classes=classes, ctx=ctx)
    X, y = oracle.synth(n, f, DATA_SEED, classes, nthreads=NTHREADS)
    np.testing.assert_array_equal(ds.labels(), y)
    for r0 in (0, n // 2, n - 1000):
        np.testing.assert_array_equal(ds.features(r0, r0 + 1000), X[r0:r0 + 1000].astype(np.float64))
    return ds, X, y


def check_tree_invariants(nodes, stats, gini, max_depth, bag_size):
    """Size-independent properties of one Spark tree (DecisionTreeModel NodeData, pre-order)."""
    n = len(nodes)
    assert (nodes["id"] == np.arange(n)).all()
    internal = nodes["left"] >= 0
    assert ((nodes["left"] < 0) == (nodes["right"] < 0)).all()
    ids = np.arange(n)
    assert (nodes["left"][internal] == ids[internal] + 1).all()  # pre-order: left child next
    assert (nodes["right"][internal] > nodes["left"][internal]).all()
    assert (nodes["feature"][~internal] == -1).all()
    # parent stats are the sum of its children's (integer / dyadic: exact)
    li, ri = nodes["left"][internal], nodes["right"][internal]
    np.testing.assert_array_equal(stats[internal], stats[li] + stats[ri])
    count = stats.sum(axis=1) if gini else stats[:, 0]
    assert count[0] == bag_size
    if gini:
        np.testing.assert_array_equal(nodes["prediction"], np.argmax(stats, axis=1).astype(np.float64))
    else:
        np.testing.assert_array_equal(nodes["prediction"], stats[:, 1] / stats[:, 0])
    assert (nodes["gain"][internal] > 0).all()
    # depth of every node <= maxDepth
    depth = np.zeros(n, np.int64)
    for i in np.nonzero(internal)[0]:
        depth[nodes["left"][i]] = depth[i] + 1
        depth[nodes["right"][i]] = depth[i] + 1
    assert depth.max() <= max_depth


def _run_config(ctx, *, n, f, classes, replacement, ratio, seed, lb, le, depth, check):
    """Fit learners [lb, le) exactly as bench.py does, then compare learners `check`
    (global indices) against the oracle and every tree against the invariants."""
    cls = classes > 0
    ds, X, y = _dataset(ctx, n, f, classes)
    part = _partitions(n)
    forest = nat.fit(ctx, ds, replacement=replacement, sample_ratio=ratio, seed=seed,
                     learner_begin=lb, learner_end=le, partition_offsets=part, max_depth=depth,
                     max_bins=32, impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
    assert len(forest) == le - lb
    counts = nat.sample(ctx, replacement, ratio, seed, lb, le, n, part)
    for t in range(le - lb):
        nodes, stats = forest.tree(t)
        check_tree_invariants(nodes, stats, cls, depth, int(counts[t].sum(dtype=np.int64)))
    ocounts = np.stack([oracle.bag(replacement, ratio, i, i + 1, seed, part, n)[0] for i in check])
    for k, i in enumerate(check):
        np.testing.assert_array_equal(counts[i - lb], ocounts[k], err_msg=f"bag of learner {i}")
    subs = [oracle.subspace(ratio, f, seed + i) for i in check]
    orf = oracle.fit(X, y, ocounts, subs, max_depth=depth, max_bins=32, classification=cls,
                     nthreads=NTHREADS, part=part)
    for k, i in enumerate(check):
        assert_tree_equal(forest, i - lb, orf, k)
    return ds, X, forest, orf, counts


def test_c3_as_benched(ctx):
    """C3 (BASELINE configs[2]) exactly as bench.py times it: 10M x 100, P=128, all 128
    learners, depth 8.  Learners {0, 1, 127} bit-exact against the oracle; transform of a
    row sample per tree bit-exact; the ensemble mean is breeze's in-order sum / L."""
    n, L = 10_000_000, 128
    ds, X, forest, orf, _ = _run_config(ctx, n=n, f=100, classes=0, replacement=True, ratio=1.0,
                                        seed=SEED_REG, lb=0, le=L, depth=8, check=[0, 1, 127])
    rows = np.random.default_rng(0).choice(n, 100_000, replace=False)
    Xs = X[rows].astype(np.float64)
    mean, per_tree = nat.predict(ctx, forest, Xs, nat.AGG_MEAN, per_tree=True)
    _, opt = oracle.predict(orf, Xs, per_tree=True)
    np.testing.assert_array_equal(per_tree[[0, 1, 127]], opt)
    acc = np.zeros(len(rows))
    for t in range(L):
        acc = acc + per_tree[t]
    np.testing.assert_array_equal(mean, acc / L)
    full = nat.predict_dataset(ctx, forest, ds, nat.AGG_MEAN)
    np.testing.assert_array_equal(full[rows], mean)
    forest.free()
    ds.free()


def test_c4_shard_wide_rows_64bit_offsets(ctx):
    """C4 (BASELINE configs[3]) shard shape: 2^24 + 4097 rows x 256 features (k_hist with
    four 64-feature lane groups, row offsets past 32 bits), P=128, depth 8, learners
    [448, 450) -- rank 7's first two of 512 learners over 8 GPUs.  Learner 449 is
    checked against the oracle (a CPU fit of this size takes about a minute), 448
    through the tree invariants."""
    n = (1 << 24) + 4097
    ds, X, forest, orf, _ = _run_config(ctx, n=n, f=256, classes=0, replacement=True, ratio=1.0,
                                        seed=SEED_REG, lb=448, le=450, depth=8, check=[449])
    forest.free()
    ds.free()


def test_c3_rows_past_2_24_row_lanes(ctx):
    """The row-lane histogram (k_hist_rl, F=100) with 64-bit row addresses: 2^24 + 4097 rows."""
    n = (1 << 24) + 4097
    ds, X, forest, orf, _ = _run_config(ctx, n=n, f=100, classes=0, replacement=True, ratio=1.0,
                                        seed=SEED_REG, lb=5, le=6, depth=5, check=[5])
    forest.free()
    ds.free()


def test_c5_shard(ctx):
    """C5 (BASELINE configs[4]) shard shape: 2M rows x 100 features, 64 classes, Bernoulli 0.5
    without replacement (XORShift streams), depth 12, P=128, learners [112, 114) -- rank 7's
    first two of 128 learners over 8 GPUs; votes of a row sample equal the oracle's."""
    n = 2_000_000
    ds, X, forest, orf, _ = _run_config(ctx, n=n, f=100, classes=64, replacement=False, ratio=0.5,
                                        seed=SEED_CLS, lb=112, le=114, depth=12,
                                        check=[112, 113])
    rows = np.random.default_rng(1).choice(n, 50_000, replace=False)
    Xs = X[rows].astype(np.float64)
    np.testing.assert_array_equal(nat.predict(ctx, forest, Xs, nat.AGG_MODE),
                                  oracle.predict(orf, Xs, classification=True))
    forest.free()
    ds.free()


def _full_shard(ctx, *, n, f, classes, replacement, ratio, seed, lb, le, depth, check):
    """One GPU's whole learner shard of a multi-GPU config at its full size, fitted exactly as
    bench.py --workload c4 / c5 times it.  The data are checked against the oracle's
    generator on row slices (the full host copy would be 25.6 GB for C4); every tree
    through the size-independent invariants, with its root count against its bag; the bags
    of the `check` learners bit-exact against oracle.bag at full length."""
    cls = classes > 0
    ds = nat.DeviceDataset.synthetic(n, f, seed=DATA_SEED, num_classes=classes, ctx=ctx)
    yall = ds.labels()
    for r0 in (0, n // 3, n - 1000):
        Xs, ys = oracle.synth(1000, f, DATA_SEED, classes, row_begin=r0, nthreads=1)
        np.testing.assert_array_equal(ds.features(r0, r0 + 1000), Xs.astype(np.float64))
        np.testing.assert_array_equal(yall[r0:r0 + 1000], ys)
    del yall
    part = _partitions(n)
    forest = nat.fit(ctx, ds, replacement=replacement, sample_ratio=ratio, seed=seed,
                     learner_begin=lb, learner_end=le, partition_offsets=part, max_depth=depth,
                     max_bins=32, impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
    assert len(forest) == le - lb
    step = 8
    for b0 in range(lb, le, step):
        b1 = min(le, b0 + step)
        counts = nat.sample(ctx, replacement, ratio, seed, b0, b1, n, part)
        for i in range(b0, b1):
            nodes, stats = forest.tree(i - lb)
            check_tree_invariants(nodes, stats, cls, depth, int(counts[i - b0].sum(dtype=np.int64)))
            if i in check:
                want = oracle.bag(replacement, ratio, i, i + 1, seed, part, n)[0]
                np.testing.assert_array_equal(counts[i - b0], want, err_msg=f"bag of learner {i}")
        del counts
    forest.free()
    ds.free()


def test_c4_full_shard(ctx):
    """C4 (BASELINE configs[3]) at full size on one GPU: 100M rows x 256 features, rank 7's
    learners [448, 512) of 512, P=128, depth 8 -- the shard bench.py --workload c4 times."""
    _full_shard(ctx, n=100_000_000, f=256, classes=0, replacement=True, ratio=1.0, seed=SEED_REG,
                lb=448, le=512, depth=8, check=(448, 511))


def test_c5_full_shard(ctx):
    """C5 (BASELINE configs[4]) at full size on one GPU: 50M rows x 100 features, 64 classes,
    Bernoulli 0.5 without replacement, depth 12, rank 7's learners [112, 128) of 128."""
    _full_shard(ctx, n=50_000_000, f=100, classes=64, replacement=False, ratio=0.5, seed=SEED_CLS,
                lb=112, le=128, depth=12, check=(112, 127))


def test_c3_nondyadic_as_benched(ctx):
    """bench.py's nondyadic_labels line: C3 (10M x 100, P=128, 128 learners, depth 8) on the
    real-valued labels 1.1 y + 0.3, through the screened fp64 engine.  Learners {0, 127}
    bit-exact against the oracle's row-order fp64 fit; every tree's structure sound."""
    n, L = 10_000_000, 128
    ds, X, y = _dataset(ctx, n, 100, 0)
    y2 = y * 1.1 + 0.3
    ds.set_labels(y2)
    part = _partitions(n)
    forest = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                     learner_end=L, partition_offsets=part, max_depth=8, max_bins=32,
                     impurity=nat.IMPURITY_VARIANCE)
    assert len(forest) == L
    t = forest.timing()
    for i in range(L):
        nodes, _ = forest.tree(i)
        internal = nodes["left"] >= 0
        assert (nodes["left"][internal] == np.nonzero(internal)[0] + 1).all()
        assert (nodes["gain"][internal] > 0).all()
    check = [0, 127]
    ocounts = np.stack([oracle.bag(True, 1.0, i, i + 1, SEED_REG, part, n)[0] for i in check])
    subs = [oracle.subspace(1.0, 100, SEED_REG + i) for i in check]
    orf = oracle.fit(X, y2, ocounts, subs, max_depth=8, max_bins=32, nthreads=NTHREADS, part=part)
    for k, i in enumerate(check):
        assert_tree_equal(forest, i, orf, k)
    print("c3 nondyadic: fit ms", t["total_ms"], "exact_fallbacks", t["exact_fallbacks"])
    forest.free()
    ds.free()
