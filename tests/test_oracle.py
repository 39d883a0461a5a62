"""CPU: the C oracle against the independent pure-Python restatement, known
answers and the committed golden fixtures (no GPU)."""
import json
import os

import numpy as np
import pytest

import oracle
import pyoracle as po
from conftest import DATA, GOLDEN

import spark_bagging_amd as sb
from spark_bagging_amd import synthetic


def test_default_seeds_are_java_string_hashes():
    # HasSeed default = getClass.getName.hashCode.toLong
    assert sb.java_string_hash("org.apache.spark.ml.regression.BaggingRegressor") == -1395689524
    assert sb.java_string_hash("org.apache.spark.ml.classification.BaggingClassifier") == 42087812
    assert sb.java_string_hash("org.apache.spark.ml.regression.DecisionTreeRegressor") == 926680331
    assert sb.java_string_hash("org.apache.spark.ml.classification.DecisionTreeClassifier") == 159147643
    assert oracle.DEFAULT_SEED_REGRESSOR == -1395689524


def test_murmur3_x86_32_smhasher_verification():
    """XORShiftRandom.hashSeed rests on scala.util.hashing.MurmurHash3.bytesHash, which is
    MurmurHash3_x86_32.  SMHasher's VerificationTest: hash {}, {0}, {0,1}, ... {0..254}
    with seed 256-i, hash the 1024-byte array of little-endian results with seed 0; the
    published value for MurmurHash3_x86_32 is 0xB0F57EE3 (an anchor outside this repo)."""
    key = bytes(range(256))
    hashes = b"".join(oracle.mm3_bytes_hash(key[:i], 256 - i).to_bytes(4, "little")
                      for i in range(256))
    assert oracle.mm3_bytes_hash(hashes, 0) == 0xB0F57EE3
    # the Python twin agrees on the same keys (it implements hashSeed independently)
    for i in (0, 1, 3, 4, 7, 8, 255):
        assert po.bytes_hash(key[:i], 256 - i) == oracle.mm3_bytes_hash(key[:i], 256 - i)


SPARK2_XORSHIFT_ANCHORS = [
    # seed, XORShiftRandom(seed).nextDouble() under Spark 2.x (published values):
    (0, 0.8446490682263027),                     # Spark 2.x `rand(0)` docstring example
    (30, 0.31429268272540556),                   # Spark 2.x RandomSuite
    (5419823303878592871, 0.2304755080444375),   # SPARK-9127 test
]


@pytest.mark.parametrize("seed,want", SPARK2_XORSHIFT_ANCHORS)
def test_xorshift_spark2_anchors(seed, want):
    """Spark 2.4.3's hashSeed hashes ByteBuffer.allocate(java.lang.Long.SIZE) = 64 bytes
    (Spark 3.x: 8). These published 2.x values pin that; the 8-byte form gives
    0.7604953758285915 for seed 0."""
    assert oracle.xorshift_doubles(seed, 1)[0] == want
    assert po.XORShiftRandom(seed).next_double() == want


def test_subspace_anchor_boundary():
    """mkSubspace keeps f iff nextDouble() < ratio (strict): with seed 0 the first draw is
    0.8446490682263027, so ratio == that value drops feature 0 and the next double up keeps
    it (ml/ensemble/HasSubBag.scala:97-103)."""
    u = SPARK2_XORSHIFT_ANCHORS[0][1]
    assert list(oracle.subspace(u, 1, 0)) == []
    assert list(oracle.subspace(float(np.nextafter(u, 1.0)), 1, 0)) == [0]
    assert po.subspace(u, 1, 0) == [] and po.subspace(float(np.nextafter(u, 1.0)), 1, 0) == [0]
    # the same draw is row 0 of learner 0's Bernoulli bag on partition 0 (seed + 0 + 0)
    assert oracle.bag(False, u, 0, 1, 0, [0, 1], 1)[0, 0] == 0
    assert oracle.bag(False, float(np.nextafter(u, 1.0)), 0, 1, 0, [0, 1], 1)[0, 0] == 1


@pytest.mark.parametrize("seed", [0, 1, -1, 12345, -1395689524, 2**62 + 11, -(2**63)])
def test_rng_streams_c_vs_python(seed):
    assert oracle.hash_seed(seed) == po.hash_seed(seed)
    r = po.XORShiftRandom(seed)
    assert list(oracle.xorshift_doubles(seed, 40)) == [r.next_double() for _ in range(40)]
    r = po.XORShiftRandom(seed)
    assert list(oracle.xorshift_next(seed, 32, 40)) == [r.next_int() for _ in range(40)]
    w = po.Well19937c(seed)
    assert list(oracle.well_next(seed, 32, 1500)) == [w.next(32) for _ in range(1500)]
    w = po.Well19937c(seed)
    assert list(oracle.well_doubles(seed, 100)) == [w.next_double() for _ in range(100)]


@pytest.mark.parametrize("lam", [1.0, 0.7, 0.25, 0.001, 2.5])
def test_poisson_c_vs_python(lam):
    g = po.poisson_stream(lam, 99)
    assert list(oracle.poisson(lam, 99, 300)) == [next(g) for _ in range(300)]


def test_poisson_small_mean_cap():
    # n < 1000 * mean: at mean 0.0005 the draw is capped at 1
    assert oracle.poisson(0.0005, 3, 20000).max() <= 1


def test_well_doubles_in_unit_interval():
    d = oracle.well_doubles(7, 5000)
    assert d.min() >= 0.0 and d.max() < 1.0
    assert len(np.unique(d)) == 5000


@pytest.mark.parametrize("repl,ratio,seed", [(True, 1.0, -1395689524), (True, 0.7, 5),
                                             (False, 0.5, 42087812), (False, 1.0, 3),
                                             (False, 0.3, 2**31 - 2), (False, 0.3, 2**33)])
def test_bag_c_vs_python(repl, ratio, seed):
    off = [0, 37, 80, 80, 100]
    a = oracle.bag(repl, ratio, 2, 7, seed, off, 100)
    b = po.bag(repl, ratio, range(2, 7), seed, off)
    assert (a == np.array(b)).all()


def test_bag_partition_overlap_h4():
    """(learner i, partition p) uses seed+i+p: learner i+1 on partition p equals
    learner i on partition p+1 for equal-length partitions."""
    off = [0, 50, 100, 150]
    c = oracle.bag(True, 1.0, 0, 3, 77, off, 150)
    assert (c[1, 0:50] == c[0, 50:100]).all()
    assert (c[1, 50:100] == c[0, 100:150]).all()


def test_bag_without_replacement_int_wrap_h15():
    """rand(seed+i) with an Int seed wraps in 32 bits."""
    seed = 2**31 - 1
    a = oracle.bag(False, 0.5, 1, 2, seed, [0, 64], 64)[0]
    r = po.XORShiftRandom(-(2**31))  # Int.MaxValue + 1 wraps to Int.MinValue
    assert list(a) == [1 if r.next_double() < 0.5 else 0 for _ in range(64)]


def test_bag_rejects_nonpositive_ratio():
    with pytest.raises(ValueError):
        oracle.bag(True, 0.0, 0, 1, 1, [0, 10], 10)
    with pytest.raises(ValueError):
        oracle.bag(False, 1.5, 0, 1, 1, [0, 10], 10)


def test_subspace_identity_and_sorted():
    assert list(oracle.subspace(1.0, 18, 5)) == list(range(18))
    for s in range(20):
        idx = oracle.subspace(0.7, 18, s)
        assert list(idx) == sorted(set(idx)) and list(idx) == po.subspace(0.7, 18, s)


def test_subspace_is_rand_stream_of_partition0_h6():
    """mkSubspace uses XORShiftRandom(seed+i): the same stream as learner i's
    rand on partition 0."""
    seed, ratio, F = 42087812, 0.6, 16
    sub = oracle.subspace(ratio, F, seed + 3)
    bag = oracle.bag(False, ratio, 3, 4, seed, [0, F], F)[0]
    assert list(sub) == list(np.nonzero(bag)[0])


def test_find_splits_small_and_stride_cases():
    X = np.array([[0.0], [1.0], [2.0], [2.0], [3.0], [0.0]])
    thr, exact = oracle.find_splits(X, np.array([1, 1, 2, 1, 1, 0], np.uint8), 0, 32)
    assert exact and list(thr) == [0.5, 1.5, 2.5]
    assert po.find_splits({0.0: 1, 1.0: 1, 2.0: 3, 3.0: 1}, 6, 32) == [0.5, 1.5, 2.5]
    rng = np.random.default_rng(0)
    vals = rng.integers(-50, 50, size=(3000, 1)).astype(np.float64)
    cnt = rng.integers(0, 3, size=3000).astype(np.uint8)
    thr, _ = oracle.find_splits(vals, cnt, 0, 16)
    mult = {}
    for v, c in zip(vals[:, 0], cnt):
        if c:
            mult[v] = mult.get(v, 0) + int(c)
    assert list(thr) == po.find_splits(mult, int(cnt.sum()), 16)
    assert len(thr) <= 15


def test_find_splits_all_zero_feature_has_no_splits():
    X = np.zeros((10, 1))
    thr, _ = oracle.find_splits(X, np.ones(10, np.uint8), 0, 32)
    assert len(thr) == 0


@pytest.mark.parametrize("cls", [False, True])
def test_small_forest_c_vs_python(cls):
    Xs, ys = synthetic.generate(700, 9, seed=2, num_classes=5 if cls else 0)
    counts = oracle.bag(True, 0.8, 0, 3, 11, [0, 300, 700], 700)
    subs = [oracle.subspace(0.8, 9, 11 + i) for i in range(3)]
    f = oracle.fit(Xs, ys, counts, subs, max_depth=5, max_bins=8, classification=cls,
                   min_instances_per_node=2)
    for t in range(3):
        nodes, stats = f.tree(t)
        pt = po.fit_tree(Xs.tolist(), ys.tolist(), counts[t].tolist(), list(subs[t]), max_depth=5,
                         max_bins=8, min_inst=2, gini=cls)
        assert len(pt) == len(nodes)
        for a, b in zip(nodes, pt):
            for k in ("left", "right", "feature", "threshold", "prediction", "impurity", "gain"):
                assert a[k] == b[k]
    pred = oracle.predict(f, Xs, classification=cls)
    trees = [po.fit_tree(Xs.tolist(), ys.tolist(), counts[t].tolist(), list(subs[t]), max_depth=5,
                         max_bins=8, min_inst=2, gini=cls) for t in range(3)]
    for i in range(0, 700, 37):
        assert pred[i] == po.predict_ensemble(trees, subs, Xs[i], cls)


def test_mode_tie_break_first_to_reach_max_h11():
    """breeze mode: the class that first reaches the final max count wins."""
    X = np.zeros((1, 1))

    def leaf(pred):
        n = np.zeros(1, oracle.NODE_DTYPE)
        n["left"] = n["right"] = -1
        n["feature"] = -1
        n["prediction"] = pred
        return n

    for votes, want in [([2, 1, 1, 2], 1.0), ([3, 3, 0, 0], 3.0), ([0, 1, 2], 0.0),
                        ([4, 2, 2, 4, 4, 2], 4.0), ([1, 2, 2, 1], 2.0)]:
        L = len(votes)
        nodes = np.zeros((L, 1), oracle.NODE_DTYPE)
        for l, v in enumerate(votes):
            nodes[l] = leaf(float(v))
        f = oracle.Forest(nodes, np.zeros((L, 1, 1)), np.ones(L, np.int32), np.ones(L, np.int32),
                          [np.array([0], np.int32)] * L, np.ones(L, bool))
        assert oracle.predict(f, X, classification=True)[0] == want, votes


def test_golden_rng_fixture():
    g = json.load(open(os.path.join(GOLDEN, "rng.json")))
    for i, s in enumerate(g["seeds"]):
        assert str(oracle.hash_seed(s)) == g["hash_seed"][i]
        assert [float(x).hex() for x in oracle.xorshift_doubles(s, 8)] == g["xorshift_doubles"][i]
        assert [int(x) for x in oracle.xorshift_next(s, 32, 8)] == g["xorshift_int"][i]
        assert [float(x).hex() for x in oracle.well_doubles(s, 8)] == g["well_doubles"][i]
    for lam, per_seed in g["poisson"].items():
        for s, vals in per_seed.items():
            assert [int(x) for x in oracle.poisson(float(lam), int(s), 64)] == vals


def _load(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)


def _data(name):
    if name.startswith("cpusmall"):
        return sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))
    if name.startswith("vehicle"):
        return sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))
    if name == "synth_p3":
        return synthetic.generate(6000, 12, seed=3)
    return synthetic.generate(5000, 10, seed=4, num_classes=6)


@pytest.mark.parametrize("name", ["cpusmall_c1", "vehicle_c2", "vehicle_repl07", "synth_p3",
                                  "synth_bern"])
def test_oracle_matches_golden(name):
    g = _load(name)
    X, y = _data(name)
    L, repl, ratio, seed, depth, bins, cls = g["params"]
    L, depth, bins, seed = int(L), int(depth), int(bins), int(seed)
    part = list(g["partitions"])
    counts = oracle.bag(bool(repl), ratio, 0, L, seed, part, X.shape[0])
    assert (counts == g["counts"]).all()
    subs = [s[s >= 0] for s in g["subspaces"]]
    for i in range(L):
        assert list(oracle.subspace(ratio, X.shape[1], seed + i)) == list(subs[i])
    f = oracle.fit(X, y, counts, subs, max_depth=depth, max_bins=bins, classification=bool(cls))
    nodes = np.concatenate([f.tree(t)[0] for t in range(L)])
    assert (f.num_nodes == g["num_nodes"]).all()
    assert (nodes == g["nodes"]).all()
    assert (oracle.predict(f, X, classification=bool(cls)) == g["prediction"]).all()


def test_libsvm_reader_matches_reference_files():
    X, y = sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))
    assert X.shape == (8192, 12) and y.min() == 0 and y.max() == 99
    assert (y == np.floor(y)).all()
    Xv, yv = sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))
    assert Xv.shape == (846, 18)
    assert sorted(set(yv)) == [1.0, 2.0, 3.0, 4.0]
    # distinct values per feature
    assert [len(np.unique(X[:, f])) for f in range(12)] == [235, 189, 4115, 794, 640, 228, 386,
                                                            7997, 7939, 302, 3165, 7658]


def test_synthetic_generator_shape_and_levels():
    X, y = synthetic.generate(4000, 20, seed=9)
    assert X.min() == 0 and X.max() == 31 and (X == np.floor(X)).all()
    assert (np.ldexp(y, 6) == np.floor(np.ldexp(y, 6))).all()
    Xc, yc = synthetic.generate(4000, 20, seed=9, num_classes=7)
    assert (X == Xc).all() and set(np.unique(yc)) <= set(range(7))


# ---------------------------------------------------------------- split-finding sample
def test_java_random_known_answers():
    """java.util.Random(42): nextLong() = -5025562857975149833, -5843495416241995736."""
    jr = po.JavaRandom(42)
    assert jr.next_long() == -5025562857975149833
    assert jr.next_long() == -5843495416241995736
    seeds = oracle.split_sample_seeds(oracle.DT_SEED_REGRESSOR, 3)
    jr = po.JavaRandom(po.XORShiftRandom(oracle.DT_SEED_REGRESSOR).next_int())
    assert list(seeds) == [jr.next_long() for _ in range(3)]


@pytest.mark.parametrize("n_rows,P", [(30000, 3), (13000, 2)])
def test_split_sample_matches_python_twin(n_rows, P):
    """RandomForest.findSplits' sample (GapSampling at fraction <= 0.4, per-item
    nextDouble above): C oracle == pure-Python twin, row multiplicities exact."""
    rng = np.random.default_rng(n_rows)
    counts = rng.poisson(1.0, n_rows).astype(np.uint8)
    off = [int(round(i * n_rows / P)) for i in range(P + 1)]
    n = int(counts.sum())
    f = oracle.split_sample_fraction(n, 32)
    assert f == po.split_sample_fraction(n, 32) and f < 1.0
    assert (f <= 0.4) == (n_rows == 30000)
    got = oracle.split_sample(counts, off, oracle.DT_SEED_REGRESSOR, f)
    want = po.split_sample(counts, off, oracle.DT_SEED_REGRESSOR, f)
    assert list(got) == want
    assert (got <= counts).all()
    # the expected size is f * n = 10000; a Bernoulli(f) sample lands within a few sigma
    assert abs(int(got.sum()) - 10000) < 500


def test_sampled_split_finding_in_fit():
    """A subbag larger than max(maxBins^2, 10^4) with continuous features: the oracle's
    thresholds are those of findSplitsForContinuousFeature over the sample (zeros implied
    by numSamples = (fraction * n).toInt), not over the whole subbag."""
    rng = np.random.default_rng(5)
    N, F = 24000, 3
    X = np.round(rng.normal(size=(N, F)), 3)
    X[rng.random((N, F)) < 0.2] = 0.0
    y = rng.integers(0, 64, N).astype(np.float64) / 8
    counts = rng.poisson(1.0, (1, N)).astype(np.uint8)
    off = [0, 9000, 24000]
    orf = oracle.fit(X, y, counts, [np.arange(F)], max_depth=2, max_bins=16, part=off)
    n = int(counts.sum())
    frac = po.split_sample_fraction(n, 16)
    mult = po.split_sample(counts[0], off, oracle.DT_SEED_REGRESSOR, frac)
    ns = int(frac * n)
    nodes, _ = orf.tree(0)
    root = nodes[0]
    assert root["feature"] >= 0
    f = int(root["feature"])
    vm = {}
    for r in range(N):
        if mult[r] and X[r, f] != 0.0:
            vm[X[r, f]] = vm.get(X[r, f], 0) + mult[r]
    thr = po.find_splits(vm, n, 16, num_samples=ns)
    assert root["threshold"] in thr


def test_oracle_u8_codes_equal_fp64_rows():
    """oracle.fit over the synthetic u8 codes (value = code, the bench workload's rows as
    tests/test_gpu_bench_configs.py feeds them) equals the same fit over fp64 rows."""
    X, y = oracle.synth(3000, 7, 99, 0, nthreads=2)
    X2, y2 = oracle.synth(3000, 7, 99, 0, row_begin=0, nthreads=1)
    assert (X == X2).all() and (y == y2).all()
    counts = oracle.bag(True, 1.0, 0, 2, 5, [0, 1000, 3000], 3000)
    subs = [oracle.subspace(1.0, 7, 5 + i) for i in range(2)]
    a = oracle.fit(X, y, counts, subs, max_depth=6, max_bins=32, nthreads=4)
    b = oracle.fit(X.astype(np.float64), y, counts, subs, max_depth=6, max_bins=32, nthreads=1)
    for t in range(2):
        (na, sa), (nb, sb_) = a.tree(t), b.tree(t)
        assert na.tobytes() == nb.tobytes() and (sa == sb_).all()
    # rows of a later range are the same rows (row_begin offsets the generator)
    Xt, yt = oracle.synth(1000, 7, 99, 0, row_begin=2000, nthreads=2)
    assert (Xt == X[2000:]).all() and (yt == y[2000:]).all()


def test_nondyadic_labels_c_vs_python():
    """Real-valued labels (the row-order fp64 path): the C oracle's trees equal the
    pure-Python restatement's, every field -- both sum count, y, y*y per exploded row in
    row order (DTStatsAggregator.update)."""
    X, y = synthetic.generate(900, 6, seed=12)
    y = y * np.pi + 0.1
    counts = oracle.bag(True, 1.0, 0, 2, 21, [0, 900], 900)
    subs = [oracle.subspace(1.0, 6, 21 + i) for i in range(2)]
    f = oracle.fit(X, y, counts, subs, max_depth=6, max_bins=8)
    for t in range(2):
        nodes, _ = f.tree(t)
        pt = po.fit_tree(X.tolist(), y.tolist(), counts[t].tolist(), list(subs[t]), max_depth=6,
                         max_bins=8)
        assert len(pt) == len(nodes)
        for a, b in zip(nodes, pt):
            for k in ("left", "right", "feature", "threshold", "prediction", "impurity", "gain"):
                assert a[k] == b[k], (t, k)


def test_nondyadic_labels_per_partition_sums_c_vs_python():
    """Several partitions with real-valued labels: Spark aggregates each partition's rows
    (mapPartitions, DTStatsAggregator.update in row order) and merges the partials with
    reduceByKey(_ merge _) -- here in partition order, one order Spark produces.  The C oracle
    and the pure-Python twin agree on every field, and the fp64 statistics differ from a
    single-partition fit of the same bags (the merge order is visible in the sums)."""
    X, y = synthetic.generate(900, 6, seed=12)
    y = y * np.pi * 1e3 + 0.1
    part = [0, 250, 611, 900]
    counts = oracle.bag(True, 1.0, 0, 2, 21, part, 900)
    subs = [oracle.subspace(1.0, 6, 21 + i) for i in range(2)]
    f = oracle.fit(X, y, counts, subs, max_depth=6, max_bins=8, part=part)
    f1 = oracle.fit(X, y, counts, subs, max_depth=6, max_bins=8)
    differ = False
    for t in range(2):
        nodes, stats = f.tree(t)
        pt = po.fit_tree(X.tolist(), y.tolist(), counts[t].tolist(), list(subs[t]), max_depth=6,
                         max_bins=8, part_off=part)
        assert len(pt) == len(nodes)
        for a, b in zip(nodes, pt):
            for k in ("left", "right", "feature", "threshold", "prediction", "impurity", "gain"):
                assert a[k] == b[k], (t, k)
        n1, s1 = f1.tree(t)
        differ = differ or len(n1) != len(nodes) or not np.array_equal(stats, s1)
    assert differ, "per-partition sums should round differently from one row-order sum"
