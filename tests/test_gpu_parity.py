"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact: bag counts, subspaces, thresholds, tree structure, impurities, gains,
node stats and classification votes.  Regression predictions: within 1e-5
relative (north_star tolerance); they come out bit-exact for the dyadic labels used.
Reference workloads: data/cpusmall (BaggingRegressorSuite.scala:12) and
data/vehicle (BaggingClassifierSuite.scala:12), copied under tests/golden/data.
"""
import os

import numpy as np
import pytest

import oracle
from conftest import DATA
from parity_utils import assert_forest_equal, oracle_forest

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu

SEED_REG = oracle.DEFAULT_SEED_REGRESSOR
SEED_CLS = oracle.DEFAULT_SEED_CLASSIFIER


@pytest.fixture(scope="module")
def ctx():
    return sb.default_context(0)


@pytest.fixture(scope="module")
def cpusmall():
    return sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))


@pytest.fixture(scope="module")
def vehicle():
    return sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))


# ---------------------------------------------------------------- sampler
@pytest.mark.parametrize("seed", [SEED_REG, SEED_CLS, 0, 7, 2**40 + 3, -5])
@pytest.mark.parametrize("ratio", [1.0, 0.7, 0.05])
def test_poisson_bag_bit_exact(ctx, seed, ratio):
    N = 5000
    off = [0, 1234, 1234, 4000, 5000]  # includes an empty partition
    got = nat.sample(ctx, True, ratio, seed, 3, 11, N, off)
    want = oracle.bag(True, ratio, 3, 11, seed, off, N)
    assert (got == want).all()


@pytest.mark.parametrize("lanes", ["0", "8", "16", "4"])
@pytest.mark.parametrize("ratio", [1.0, 0.2, 0.001])
def test_poisson_sampler_variants_many_streams(ctx, monkeypatch, lanes, ratio):
    # k_poisson4 with lanes by stream count (0), 8, 16 and 4 lanes per stream (capped parse for
    # ratio <= 0.255, where nextPoisson's n < 1000 * mean can end a row), on 38 learners x 7
    # ragged partitions (266 streams: idle slots in the last block) with streams long enough to
    # run round the 624-word ring many times.  (Rounds 1-3's k_poisson / k_poisson2 /
    # k_poisson3 were removed in round 6.)
    monkeypatch.setenv("SBAG_POISSON_LANES", lanes)
    N = 120_000
    off = [0, 1, 17_000, 17_000, 50_001, 77_777, 100_000, N]
    got = nat.sample(ctx, True, ratio, SEED_REG, 5, 43, N, off)
    want = oracle.bag(True, ratio, 5, 43, SEED_REG, off, N)
    assert (got == want).all()


@pytest.mark.parametrize("lanes", ["0", "4", "8", "16"])
def test_poisson4_many_draws(ctx, monkeypatch, lanes):
    # 32M draws per layout: a wrong low mantissa bit of nextDouble() moves a draw only when
    # the running product lands within ~2^-27 of exp(-mean) (one draw in ~10^7), which the
    # small cases above cannot see
    monkeypatch.setenv("SBAG_POISSON_LANES", lanes)
    N, L = 2_000_000, 16
    off = [int(round(i * N / 64)) for i in range(65)]
    got = nat.sample(ctx, True, 1.0, SEED_REG, 100, 100 + L, N, off)
    want = oracle.bag(True, 1.0, 100, 100 + L, SEED_REG, off, N)
    assert (got == want).all()


@pytest.mark.parametrize("seed", [SEED_REG, SEED_CLS, 2**31 - 3, -2**31 + 1, 2**40 + 3])
@pytest.mark.parametrize("ratio", [0.5, 0.3, 0.999])
def test_bernoulli_bag_bit_exact(ctx, seed, ratio):
    N = 70000
    off = [0, 300, 30000, 30001, 70000]
    got = nat.sample(ctx, False, ratio, seed, 0, 6, N, off)
    want = oracle.bag(False, ratio, 0, 6, seed, off, N)
    assert (got == want).all()


def test_spark2_hash_seed_anchor_through_c_abi(ctx):
    """Spark 2.4.3's XORShiftRandom(0).nextDouble() is 0.8446490682263027 (64-byte
    hashSeed). rand(seed + i) on partition 0 row 0 and mkSubspace both take that draw with a
    strict `<`: ratio == u gives 0 / [], the next double up 1 / [0]."""
    u = 0.8446490682263027
    up = float(np.nextafter(u, 1.0))
    assert list(nat.subspace(u, 1, 0)) == []
    assert list(nat.subspace(up, 1, 0)) == [0]
    assert nat.sample(ctx, False, u, 0, 0, 1, 1, [0, 1])[0, 0] == 0
    assert nat.sample(ctx, False, up, 0, 0, 1, 1, [0, 1])[0, 0] == 1
    # the other two published anchors: seed 30 and 5419823303878592871 (SQL Int wrap does not
    # apply above Int range; learner 0, partition 0)
    for seed, v in [(30, 0.31429268272540556), (5419823303878592871, 0.2304755080444375)]:
        assert nat.sample(ctx, False, v, seed, 0, 1, 1, [0, 1])[0, 0] == 0
        assert nat.sample(ctx, False, float(np.nextafter(v, 1.0)), seed, 0, 1, 1, [0, 1])[0, 0] == 1


def test_all_ones_bag(ctx):
    got = nat.sample(ctx, False, 1.0, SEED_REG, 0, 4, 1000)
    assert (got == 1).all()


def test_sampler_rejects_bad_ratio(ctx):
    with pytest.raises(sb.IllegalArgumentException):
        nat.sample(ctx, True, 0.0, 1, 0, 2, 10)
    with pytest.raises(sb.IllegalArgumentException):
        nat.sample(ctx, False, 1.5, 1, 0, 2, 10)


# ---------------------------------------------------------------- fit
def _fit_both(ctx, X, y, L, *, replacement, ratio, seed, depth, bins, cls, subspace_ratio=1.0,
              bug_compat=True, part=None, min_inst=1, min_gain=0.0):
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    forest = nat.fit(ctx, ds, replacement=replacement, sample_ratio=ratio, seed=seed,
                     learner_begin=0, learner_end=L, subspace_ratio=subspace_ratio,
                     subspace_bug_compat=bug_compat, partition_offsets=part, max_depth=depth,
                     max_bins=bins, min_instances_per_node=min_inst, min_info_gain=min_gain,
                     impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
    N, F = X.shape
    off = part if part is not None else [0, N]
    counts = oracle.bag(replacement, ratio, 0, L, seed, off, N)
    sratio = ratio if bug_compat else subspace_ratio
    subs = [oracle.subspace(sratio, F, seed + i) for i in range(L)]
    orf = oracle_forest(X, y, counts, subs, depth, bins, cls, min_inst, min_gain)
    return forest, orf, ds


def test_cpusmall_c1_parity(ctx, cpusmall):
    """BASELINE config 1: BaggingRegressor(DecisionTreeRegressor) on cpusmall, 10 learners."""
    X, y = cpusmall
    forest, orf, _ = _fit_both(ctx, X, y, 10, replacement=True, ratio=1.0, seed=SEED_REG,
                               depth=5, bins=32, cls=False)
    assert_forest_equal(forest, orf)
    pred = nat.predict(ctx, forest, X, nat.AGG_MEAN)
    np.testing.assert_allclose(pred, oracle.predict(orf, X), rtol=1e-5, atol=0)


@pytest.mark.parametrize("budget_mb", ["1.0", "0.2"])
def test_per_replica_bins_over_budget_split_learner_range(ctx, cpusmall, monkeypatch, budget_mb):
    """cpusmall's thresholds differ across replicas, so bins are per replica (≈150 KB each for
    the in-bag rows); over the device budget (SBAG_BINS_BUDGET_MB) the learner range is fitted
    in parts (down to one learner per fit at 0.2 MB) and the trees concatenated in learner
    order."""
    X, y = cpusmall
    whole, _, _ = _fit_both(ctx, X, y, 10, replacement=True, ratio=1.0, seed=SEED_REG,
                            depth=5, bins=32, cls=False)
    monkeypatch.setenv("SBAG_BINS_BUDGET_MB", budget_mb)
    forest, orf, _ = _fit_both(ctx, X, y, 10, replacement=True, ratio=1.0, seed=SEED_REG,
                               depth=5, bins=32, cls=False)
    assert len(forest) == 10
    # every sub-range ran its own level loop
    assert forest.timing()["hist_launches"] > whole.timing()["hist_launches"]
    assert_forest_equal(forest, orf)
    np.testing.assert_allclose(nat.predict(ctx, forest, X, nat.AGG_MEAN), oracle.predict(orf, X),
                               rtol=1e-5, atol=0)


def test_cpusmall_reference_grid_point(ctx, cpusmall):
    """One CV grid point of BaggingRegressorSuite.scala:30-38 (depth 10, bins 30, ratio 0.7)."""
    X, y = cpusmall
    forest, orf, _ = _fit_both(ctx, X, y, 10, replacement=True, ratio=0.7, seed=SEED_REG,
                               depth=10, bins=30, cls=False)
    assert_forest_equal(forest, orf)
    np.testing.assert_allclose(nat.predict(ctx, forest, X, nat.AGG_MEAN), oracle.predict(orf, X),
                               rtol=1e-5, atol=0)


@pytest.mark.parametrize("cls,depth", [(False, 30), (True, 30), (False, 26)])
def test_max_depth_up_to_30(ctx, cpusmall, vehicle, cls, depth):
    """Spark's DecisionTree allows maxDepth <= 30 (fitBaseLearner passes it through,
    ml/ensemble/ensembleParams.scala:99-117). cpusmall / vehicle grown without a depth
    bound in practice (cpusmall's trees reach levels 25-27, vehicle's 15-16), bit-exact
    against the oracle."""
    X, y = vehicle if cls else cpusmall
    forest, orf, _ = _fit_both(ctx, X, y, 3, replacement=True, ratio=1.0,
                               seed=SEED_CLS if cls else SEED_REG, depth=depth, bins=64, cls=cls)
    assert_forest_equal(forest, orf)

    def tree_depth(nodes, i=0):
        n = nodes[i]
        return 0 if n["left"] < 0 else 1 + max(tree_depth(nodes, n["left"]),
                                               tree_depth(nodes, n["right"]))
    deepest = max(tree_depth(forest.tree(t)[0]) for t in range(3))
    assert deepest <= depth and (cls or deepest > 24)
    agg = nat.AGG_MODE if cls else nat.AGG_MEAN
    got = nat.predict(ctx, forest, X, agg)
    want = oracle.predict(orf, X, classification=cls)
    assert (got == want).all() if cls else np.allclose(got, want, rtol=1e-5, atol=0)


def test_vehicle_c2_parity(ctx, vehicle):
    """BASELINE config 2: BaggingClassifier on vehicle, 32 learners, subspaceRatio 0.7 (H1: no-op)."""
    X, y = vehicle
    forest, orf, _ = _fit_both(ctx, X, y, 32, replacement=False, ratio=1.0, seed=SEED_CLS,
                               depth=5, bins=32, cls=True, subspace_ratio=0.7)
    assert_forest_equal(forest, orf)
    got = nat.predict(ctx, forest, X, nat.AGG_MODE)
    assert (got == oracle.predict(orf, X, classification=True)).all()


def test_vehicle_replacement_ratio07(ctx, vehicle):
    X, y = vehicle
    forest, orf, _ = _fit_both(ctx, X, y, 32, replacement=True, ratio=0.7, seed=SEED_CLS,
                               depth=6, bins=32, cls=True)
    assert_forest_equal(forest, orf)
    assert (nat.predict(ctx, forest, X, nat.AGG_MODE) ==
            oracle.predict(orf, X, classification=True)).all()


def test_vehicle_bernoulli_min_instances(ctx, vehicle):
    X, y = vehicle
    forest, orf, _ = _fit_both(ctx, X, y, 8, replacement=False, ratio=0.6, seed=SEED_CLS,
                               depth=7, bins=16, cls=True, min_inst=5, min_gain=0.01)
    assert_forest_equal(forest, orf)


def test_synthetic_partitions_regression(ctx):
    """Device-generated synthetic data, P=3 partitions (pins per-partition seeding, H4)."""
    ds = nat.DeviceDataset.synthetic(30000, 20, seed=5, num_classes=0, ctx=ctx)
    X, y = ds.features(), ds.labels()
    part = [0, 10000, 17000, 30000]
    forest = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                     learner_end=6, partition_offsets=part, max_depth=6, max_bins=32)
    counts = oracle.bag(True, 1.0, 0, 6, SEED_REG, part, 30000)
    subs = [oracle.subspace(1.0, 20, SEED_REG + i) for i in range(6)]
    orf = oracle_forest(X, y, counts, subs, 6, 32, False)
    assert_forest_equal(forest, orf)
    np.testing.assert_allclose(nat.predict_dataset(ctx, forest, ds, nat.AGG_MEAN),
                               oracle.predict(orf, X), rtol=1e-5, atol=0)


def test_synthetic_classification_subspace(ctx):
    ds = nat.DeviceDataset.synthetic(20000, 24, seed=11, num_classes=7, ctx=ctx)
    X, y = ds.features(), ds.labels()
    forest = nat.fit(ctx, ds, replacement=False, sample_ratio=0.5, seed=SEED_CLS, learner_begin=0,
                     learner_end=5, max_depth=8, max_bins=32, impurity=nat.IMPURITY_GINI)
    counts = oracle.bag(False, 0.5, 0, 5, SEED_CLS, [0, 20000], 20000)
    subs = [oracle.subspace(0.5, 24, SEED_CLS + i) for i in range(5)]
    orf = oracle_forest(X, y, counts, subs, 8, 32, True)
    assert_forest_equal(forest, orf)
    assert (nat.predict_dataset(ctx, forest, ds, nat.AGG_MODE) ==
            oracle.predict(orf, X, classification=True)).all()


def test_variance_screen_fallback_on_exact_ties(ctx, cpusmall):
    """Duplicated feature columns make every split on column 0 tie exactly with its
    copy: the (count, sum) screen must flag those nodes, and the exact fallback (sums
    of squares histogram + Spark-order k_split) must pick the first feature like
    RandomForest.binsToBestSplit's maxBy.  Checked bit-exact against the oracle."""
    X, y = cpusmall
    X = np.ascontiguousarray(np.concatenate([X, X[:, :3]], axis=1))
    forest, orf, _ = _fit_both(ctx, X, y, 4, replacement=True, ratio=1.0, seed=SEED_REG,
                               depth=6, bins=32, cls=False)
    assert forest.timing()["exact_fallbacks"] > 0
    assert_forest_equal(forest, orf)


@pytest.mark.parametrize("min_gain", [0.0, 0.5, 25.0])
def test_variance_min_info_gain(ctx, cpusmall, min_gain):
    """minInfoGain decides leaves through Spark's fp64 gain: screened nodes near the
    threshold fall back to the exact split."""
    X, y = cpusmall
    forest, orf, _ = _fit_both(ctx, X, y, 4, replacement=True, ratio=0.8, seed=SEED_REG + 3,
                               depth=8, bins=24, cls=False, min_gain=min_gain, min_inst=3)
    assert_forest_equal(forest, orf)


def _synthetic_cls(ctx, N, F, C, L, depth, seed_data, ratio=0.5, replacement=False):
    ds = nat.DeviceDataset.synthetic(N, F, seed=seed_data, num_classes=C, ctx=ctx)
    X, y = ds.features(), ds.labels()
    forest = nat.fit(ctx, ds, replacement=replacement, sample_ratio=ratio, seed=SEED_CLS,
                     learner_begin=0, learner_end=L, max_depth=depth, max_bins=32,
                     impurity=nat.IMPURITY_GINI)
    counts = oracle.bag(replacement, ratio, 0, L, SEED_CLS, [0, N], N)
    subs = [oracle.subspace(ratio, F, SEED_CLS + i) for i in range(L)]
    orf = oracle_forest(X, y, counts, subs, depth, 32, True)
    return ds, X, forest, orf


def test_many_classes_c5_shape(ctx):
    """BASELINE config 5 in miniature: 64 classes, without-replacement subsample 0.5,
    depth 12.  64 class planes do not fit in LDS, so k_hist runs class tiles."""
    ds, X, forest, orf = _synthetic_cls(ctx, 24000, 100, 64, 3, 12, seed_data=17)
    assert_forest_equal(forest, orf)
    assert (nat.predict_dataset(ctx, forest, ds, nat.AGG_MODE) ==
            oracle.predict(orf, X, classification=True)).all()


def test_many_classes_known_tile_cursors_checked(ctx, monkeypatch):
    """Without-replacement bags (every draw count 1) group class tiles from the split's known
    class counts (k_tile_scatter_known: atomic (segment, tile) cursors placed by host sizes).
    SBAG_TILE_CHECK=1 copies every cursor back and fails the fit unless each ends exactly at
    its tile's end (no test had run the check); trees bit-exact."""
    monkeypatch.setenv("SBAG_TILE_CHECK", "1")
    ds, X, forest, orf = _synthetic_cls(ctx, 30000, 100, 64, 3, 12, seed_data=29)
    assert_forest_equal(forest, orf)


@pytest.mark.parametrize("replacement", [False, True])
def test_tile_resident_entries_opt_in(ctx, monkeypatch, replacement):
    """SBAG_TILE_RESIDENT=1: the root's class-tile grouping kept for the whole fit, the
    partition splitting every (node, tile) sub-segment in place -- same trees (the option
    is off by default: slower on the C5 shard)."""
    monkeypatch.setenv("SBAG_TILE_RESIDENT", "1")
    ds, X, forest, orf = _synthetic_cls(ctx, 24000, 100, 64, 3, 12, seed_data=19,
                                        replacement=replacement, ratio=0.6)
    assert_forest_equal(forest, orf)


def test_gini_class_tiles_forced(ctx, monkeypatch):
    """A tiny LDS budget forces one-class tiles on a 7-class problem (k_hist class
    tiling + per-wave entry staging), bit-exact against the oracle."""
    monkeypatch.setenv("SBAG_HIST_LDS_KB", "12")
    ds, X, forest, orf = _synthetic_cls(ctx, 15000, 80, 7, 4, 7, seed_data=23, ratio=0.8,
                                        replacement=True)
    assert_forest_equal(forest, orf)


@pytest.mark.parametrize("min_gain", [0.0, 0.02])
def test_gini_screen_exact_ties_and_min_gain(ctx, min_gain):
    """The gini split screen (cheap 1 - sum l^2/lt^2 against the block's best exact gain of
    earlier feature groups) must keep Spark's choice: duplicated columns in later feature
    groups tie the earlier ones exactly (first feature wins), and minInfoGain near the
    gains decides leaves on the exact fp64 gain.  64 classes: grouped class tiles and the
    class-tile-major histogram layout."""
    ds0 = nat.DeviceDataset.synthetic(20000, 40, seed=29, num_classes=64, ctx=ctx)
    X0, y = ds0.features(), ds0.labels()
    X = np.ascontiguousarray(np.concatenate([X0, X0[:, :12], X0[:, 5:9]], axis=1))
    forest, orf, _ = _fit_both(ctx, X, y, 3, replacement=False, ratio=1.0, seed=SEED_CLS,
                               depth=9, bins=32, cls=True, min_gain=min_gain, min_inst=2)
    assert_forest_equal(forest, orf)


@pytest.mark.parametrize("classes,lds_kb,layout", [(64, None, "1"), (10, "29", None),
                                                   (12, "29", None), (12, "12", None)])
def test_gini_tile_layouts(ctx, monkeypatch, classes, lds_kb, layout):
    """Class tiles that divide the classes store the histogram class-tile-major (12 classes
    in tiles of 3: scalar flush and staging paths; tiles of 1); tiles that do not (10
    classes in tiles of 3) keep the [f][b][NS] layout; SBAG_NO_TILE_LAYOUT=1 forces the
    plain layout.  Every case bit-exact against the oracle."""
    if lds_kb:
        monkeypatch.setenv("SBAG_HIST_GROUPED_LDS_KB", lds_kb)
    if layout:
        monkeypatch.setenv("SBAG_NO_TILE_LAYOUT", layout)
    ds, X, forest, orf = _synthetic_cls(ctx, 16000, 60, classes, 3, 9, seed_data=31)
    assert_forest_equal(forest, orf)


def test_transform_batches_nan_and_signed_zero(ctx, cpusmall, monkeypatch):
    """Batched host-row transform (rows binned on the device against the forest's
    thresholds): several upload batches, NaN (Spark: `NaN <= t` is false -> right),
    -0.0 == 0.0 and +-inf, bit-exact against the oracle's tree walk."""
    X, y = cpusmall
    forest, orf, _ = _fit_both(ctx, X, y, 7, replacement=True, ratio=0.9, seed=SEED_REG,
                               depth=7, bins=32, cls=False)
    Z = X.copy()
    rng = np.random.default_rng(3)
    Z[rng.random(Z.shape) < 0.05] = np.nan
    Z[rng.random(Z.shape) < 0.05] = -0.0
    Z[rng.random(Z.shape) < 0.01] = np.inf
    Z[rng.random(Z.shape) < 0.01] = -np.inf
    monkeypatch.setenv("SBAG_PREDICT_BATCH_ROWS", "1000")
    got = nat.predict(ctx, forest, Z, nat.AGG_MEAN)
    np.testing.assert_array_equal(got, oracle.predict(orf, Z))


def test_wide_rows_four_lane_groups(ctx):
    """200 features: 256-byte rows and four 64-feature lane groups in k_hist (the C4
    shape has 256), with a partial last group and a 0.6 feature subspace."""
    ds = nat.DeviceDataset.synthetic(12000, 200, seed=29, num_classes=0, ctx=ctx)
    X, y = ds.features(), ds.labels()
    forest = nat.fit(ctx, ds, replacement=True, sample_ratio=0.6, seed=SEED_REG, learner_begin=0,
                     learner_end=3, max_depth=6, max_bins=32)
    counts = oracle.bag(True, 0.6, 0, 3, SEED_REG, [0, 12000], 12000)
    subs = [oracle.subspace(0.6, 200, SEED_REG + i) for i in range(3)]
    orf = oracle_forest(X, y, counts, subs, 6, 32, False)
    assert_forest_equal(forest, orf)
    np.testing.assert_array_equal(nat.predict_dataset(ctx, forest, ds, nat.AGG_MEAN),
                                  oracle.predict(orf, X))


@pytest.mark.parametrize("rl", ["0", "1", "auto"])
def test_row_lane_histogram_modes(ctx, cpusmall, monkeypatch, rl):
    """k_hist_rl (16 lanes per entry, 4 entries per LDS atomic) against k_hist: off,
    forced 64-bit row addresses, and the automatic choice (32-bit offsets here), on
    variance (with the exact-tie Sq fallback), gini and a 100-feature tail tile."""
    if rl != "auto":
        monkeypatch.setenv("SBAG_HIST_RL", rl)
    X, y = cpusmall
    X2 = np.ascontiguousarray(np.concatenate([X, X[:, :3]], axis=1))
    forest, orf, _ = _fit_both(ctx, X2, y, 3, replacement=True, ratio=1.0, seed=SEED_REG,
                               depth=6, bins=32, cls=False)
    assert forest.timing()["exact_fallbacks"] > 0
    assert_forest_equal(forest, orf)
    ds, Xs, forest, orf = _synthetic_cls(ctx, 12000, 100, 9, 3, 8, seed_data=29, ratio=1.0,
                                         replacement=True)
    assert_forest_equal(forest, orf)
    ds = nat.DeviceDataset.synthetic(16000, 100, seed=31, num_classes=0, ctx=ctx)
    Xr, yr = ds.features(), ds.labels()
    forest = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                     learner_end=3, max_depth=7, max_bins=32)
    counts = oracle.bag(True, 1.0, 0, 3, SEED_REG, [0, 16000], 16000)
    subs = [oracle.subspace(1.0, 100, SEED_REG + i) for i in range(3)]
    assert_forest_equal(forest, oracle_forest(Xr, yr, counts, subs, 7, 32, False))


@pytest.mark.parametrize("n_rows,cls,P", [(30000, False, 3), (16000, True, 2), (40000, False, 1),
                                           (400000, False, 7), (250000, True, 5)])
def test_sampled_split_finding(ctx, n_rows, cls, P):
    """Subbags larger than max(maxBins^2, 10^4) rows: thresholds from RandomForest.findSplits'
    RDD.sample (k_split_sample: per-partition BernoulliSampler seeded through
    java.util.Random, GapSampling at fraction <= 0.4, per-item draws above), continuous
    features with zeros, bit-exact against the oracle's restatement."""
    rng = np.random.default_rng(n_rows + P)
    F = 5
    X = np.round(rng.normal(size=(n_rows, F)), 2)
    X[rng.random((n_rows, F)) < 0.15] = 0.0
    y = (rng.integers(0, 5, n_rows) if cls else rng.integers(-256, 256, n_rows) / 16).astype(np.float64)
    part = [int(round(i * n_rows / P)) for i in range(P + 1)]
    L = 3
    seed = SEED_CLS if cls else SEED_REG
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    forest = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=seed, learner_begin=0,
                     learner_end=L, partition_offsets=part, max_depth=6, max_bins=32,
                     impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
    counts = oracle.bag(True, 1.0, 0, L, seed, part, n_rows)
    assert oracle.split_sample_fraction(int(counts[0].sum()), 32) < 1.0
    subs = [oracle.subspace(1.0, F, seed + i) for i in range(L)]
    orf = oracle_forest(X, y, counts, subs, 6, 32, cls, part=part)
    assert_forest_equal(forest, orf)


@pytest.mark.parametrize("cls", [False, True])
def test_device_split_finding_edge_features(ctx, monkeypatch, capfd, cls):
    """findSplitsForContinuousFeature on the device (k_find_splits, a wave per (replica,
    feature)) on the cases its walk branches on: 0.0 in the dictionary or only implied by a
    sample short of numSamples (inserted first, last or in the middle), at most numSplits + 1
    values (midpoints), just above it (stride walk), a constant and an all-zero feature, mostly
    zeros.  Bit-exact against the oracle, as is the host walk over the value counts copied back
    (SBAG_SPLITS_HOST=1)."""
    rng = np.random.default_rng(11 + int(cls))
    n, P, L = 60000, 4, 4
    c0 = np.round(rng.normal(size=n), 3)
    c0[rng.random(n) < 0.1] = 0.0
    c3 = np.round(rng.normal(size=n), 3)
    c3[c3 == 0.0] = 0.5
    c7 = np.where(rng.random(n) < 0.97, 0.0, np.round(rng.normal(size=n), 2))
    X = np.stack([c0,
                  np.round(rng.uniform(1, 2, n), 4),        # positive only: 0.0 implied first
                  -np.round(rng.uniform(1, 2, n), 4),       # negative only: 0.0 implied last
                  c3,                                       # both signs, no 0.0: in the middle
                  rng.integers(0, 10, n).astype(np.float64),  # midpoints
                  np.full(n, 3.0),                          # constant
                  np.zeros(n),                              # all zeros
                  c7,
                  rng.choice(np.round(rng.normal(size=40), 3), n)], axis=1)  # stride, few values
    y = (rng.integers(0, 4, n) if cls else rng.integers(-256, 256, n) / 16).astype(np.float64)
    part = [int(round(i * n / P)) for i in range(P + 1)]
    seed = SEED_CLS if cls else SEED_REG
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    kw = dict(replacement=True, sample_ratio=1.0, seed=seed, learner_begin=0, learner_end=L,
              partition_offsets=part, max_depth=6, max_bins=32, subspace_ratio=1.0,
              subspace_bug_compat=False, impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
    monkeypatch.setenv("SBAG_DEBUG_BINS", "1")
    forest = nat.fit(ctx, ds, **kw)
    # a sample above numSamples passes a 32nd target: 32 cuts fill the 32-slot table, whose last
    # slot k_bin_cuts counts apart from its binary search
    assert "maxcuts 32 ncp 32" in capfd.readouterr().err
    monkeypatch.delenv("SBAG_DEBUG_BINS")
    counts = oracle.bag(True, 1.0, 0, L, seed, part, n)
    assert oracle.split_sample_fraction(int(counts[0].sum()), 32) < 1.0
    subs = [oracle.subspace(1.0, X.shape[1], seed + i) for i in range(L)]
    orf = oracle_forest(X, y, counts, subs, 6, 32, cls, part=part)
    assert_forest_equal(forest, orf)
    monkeypatch.setenv("SBAG_SPLITS_HOST", "1")
    assert_forest_equal(nat.fit(ctx, ds, **kw), orf)


@pytest.mark.parametrize("cls,replacement,ratio", [(False, True, 1.0), (True, True, 1.0),
                                                  (False, False, 0.1)])
def test_wide_features_more_than_65536_values(ctx, cls, replacement, ratio):
    """Features with more than 65536 distinct values (u32 value codes): split finding
    counts the sampled rows' (or, for small subbags, the in-bag rows') values sparsely,
    bins are materialized per replica from code cuts; trees, predictions on host rows and
    on the device dataset bit-exact against the oracle."""
    rng = np.random.default_rng(7 + int(cls) + int(replacement))
    n_rows, F, P, L = 90000, 3, 3, 3
    X = np.round(rng.normal(size=(n_rows, F)), 6)
    X[:, 1] = np.round(X[:, 1], 1)  # one narrow feature next to the wide ones
    X[rng.random((n_rows, F)) < 0.05] = 0.0
    assert len(np.unique(X[:, 0])) > 65536
    y = (rng.integers(0, 4, n_rows) if cls else rng.integers(-512, 512, n_rows) / 8).astype(np.float64)
    part = [int(round(i * n_rows / P)) for i in range(P + 1)]
    seed = SEED_CLS if cls else SEED_REG
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    # subspaceRatio 1 (not the sample ratio of H1): a 0.1 subspace of 3 features is empty
    forest = nat.fit(ctx, ds, replacement=replacement, sample_ratio=ratio, seed=seed,
                     learner_begin=0, learner_end=L, partition_offsets=part, max_depth=5,
                     max_bins=32, subspace_ratio=1.0, subspace_bug_compat=False,
                     impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
    counts = oracle.bag(replacement, ratio, 0, L, seed, part, n_rows)
    assert (counts.sum(axis=1) > 10000).all() == replacement  # sampled / whole-subbag paths
    subs = [oracle.subspace(1.0, F, seed + i) for i in range(L)]
    orf = oracle_forest(X, y, counts, subs, 5, 32, cls, part=part)
    assert_forest_equal(forest, orf)
    agg = nat.AGG_MODE if cls else nat.AGG_MEAN
    want = oracle.predict(orf, X, classification=cls)
    np.testing.assert_array_equal(nat.predict(ctx, forest, X, agg), want)
    np.testing.assert_array_equal(nat.predict_dataset(ctx, forest, ds, agg), want)
    np.testing.assert_array_equal(ds.features(0, 1000), np.where(X[:1000] == 0.0, 0.0, X[:1000]))


def test_layout_cache_shared_by_fits(ctx, monkeypatch):
    """The column copy and side-bit planes of a codes-as-bins dataset are built by its
    first fit and reused (sbag_dataset.d_cols / d_planes): fits with other impurities,
    subspaces and depths on the same dataset, a fit without the cache, and learner
    halves on two contexts racing to build it are all bit-exact against the oracle.
    Depth 10 on 3-4 learners reaches >= 1024 parents, where the partition reads planes."""
    N, F = 60000, 40

    def check(ds, X, y, L, cls, ratio, depth):
        forest = nat.fit(ctx, ds, replacement=True, sample_ratio=ratio, seed=SEED_CLS,
                         learner_begin=0, learner_end=L, max_depth=depth, max_bins=32,
                         impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
        counts = oracle.bag(True, ratio, 0, L, SEED_CLS, [0, N], N)
        subs = [oracle.subspace(ratio, F, SEED_CLS + i) for i in range(L)]
        assert_forest_equal(forest, oracle_forest(X, y, counts, subs, depth, 32, cls))

    ds = nat.DeviceDataset.synthetic(N, F, seed=5, num_classes=5, ctx=ctx)
    X, y = ds.features(), ds.labels()
    check(ds, X, y, 3, True, 1.0, 10)
    check(ds, X, y, 3, False, 0.6, 9)
    monkeypatch.setenv("SBAG_NO_LAYOUT_CACHE", "1")
    check(ds, X, y, 3, True, 1.0, 10)
    monkeypatch.delenv("SBAG_NO_LAYOUT_CACHE")
    monkeypatch.setenv("SBAG_OVERLAP", "2")
    ds2 = nat.DeviceDataset.synthetic(N, F, seed=6, num_classes=5, ctx=ctx)
    check(ds2, ds2.features(), ds2.labels(), 4, True, 1.0, 10)
