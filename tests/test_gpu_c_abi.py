"""GPU: the C ABI driven from plain C in the JNI shim's argument order
(tests/c/abi_driver.c over integration/sbagjni_core.c), bit-exact
against the oracle and against the ctypes path.  Covers the 16th fit argument
(treeSeed = the base learner's seed, which picks the split-finding sample of every
subbag above 10^4 rows) and the exception mapping of a bad parameter."""
import os

import numpy as np
import pytest

import oracle
from c_abi_util import run_driver, run_gbm_driver, run_threads
from conftest import DATA, ROOT

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu

FIELDS = ["id", "left", "right", "feature", "threshold", "prediction", "impurity", "gain"]


def _check_trees(trees, subs, orf):
    assert len(trees) == orf.nodes.shape[0]
    for t, packed in enumerate(trees):
        on, _ = orf.tree(t)
        assert packed.shape[0] == len(on), f"tree {t}"
        for k, f in enumerate(FIELDS):
            assert (packed[:, k] == on[f].astype(np.float64)).all(), f"tree {t} field {f}"
        assert list(subs[t]) == list(orf.subspaces[t])


def test_c_driver_vehicle_classifier(tmp_path):
    X, y = sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))
    seed, L = oracle.DEFAULT_SEED_CLASSIFIER, 6
    part = [0, 300, 846]
    p, st, trees, subs, pred = run_driver(
        tmp_path, X, y, part, replacement=1, ratio=0.7, seed=seed, lb=0, le=L, sub_ratio=0.7,
        bug_compat=1, depth=5, bins=32, min_inst=1, impurity=nat.IMPURITY_GINI, min_gain=0.0,
        tree_seed=nat.DT_SEED_CLASSIFIER, agg=nat.AGG_MODE)
    assert st == 0, p.stdout + p.stderr
    counts = oracle.bag(True, 0.7, 0, L, seed, part, len(y))
    sub = [oracle.subspace(0.7, X.shape[1], seed + i) for i in range(L)]
    orf = oracle.fit(X, y, counts, sub, max_depth=5, max_bins=32, classification=True, part=part)
    _check_trees(trees, subs, orf)
    assert (pred == oracle.predict(orf, X, classification=True)).all()


@pytest.mark.parametrize("tree_seed", [nat.DT_SEED_REGRESSOR, 12345])
def test_c_driver_sampled_split_finding_uses_tree_seed(tmp_path, tree_seed):
    """24k rows: every subbag exceeds 10^4 rows, so thresholds come from Spark's
    split-finding sample seeded by treeSeed -- the argument the old binding dropped."""
    rng = np.random.default_rng(4)
    X = np.round(rng.normal(size=(24000, 6)), 2)  # continuous: the sample decides the thresholds
    X[rng.random(X.shape) < 0.15] = 0.0
    y = rng.integers(-256, 256, 24000) / 16
    seed, L = oracle.DEFAULT_SEED_REGRESSOR, 3
    part = [0, 9000, 24000]
    p, st, trees, subs, pred = run_driver(
        tmp_path, X, y, part, replacement=1, ratio=1.0, seed=seed, lb=0, le=L, sub_ratio=1.0,
        bug_compat=1, depth=4, bins=16, min_inst=1, impurity=nat.IMPURITY_VARIANCE, min_gain=0.0,
        tree_seed=tree_seed, agg=nat.AGG_MEAN)
    assert st == 0, p.stdout + p.stderr
    counts = oracle.bag(True, 1.0, 0, L, seed, part, len(y))
    sub = [oracle.subspace(1.0, X.shape[1], seed + i) for i in range(L)]
    assert oracle.split_sample_fraction(int(counts[0].sum()), 16) < 1.0
    orf = oracle.fit(X, y, counts, sub, max_depth=4, max_bins=16, part=part, dt_seed=tree_seed)
    _check_trees(trees, subs, orf)
    ctx = nat.Context(0)
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    f = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=seed, learner_begin=0,
                learner_end=L, partition_offsets=part, max_depth=4, max_bins=16,
                tree_seed=tree_seed)
    np.testing.assert_array_equal(pred, nat.predict(ctx, f, X, nat.AGG_MEAN))
    f.free()
    ds.free()
    ctx.close()


def test_c_driver_bad_ratio_is_illegal_argument(tmp_path):
    X, y = np.zeros((8, 2)), np.zeros(8)
    p, st, *_ = run_driver(tmp_path, X, y, [0, 8], replacement=1, ratio=1.5, seed=1, lb=0, le=2,
                           sub_ratio=1.0, bug_compat=1, depth=3, bins=8, min_inst=1, impurity=0,
                           min_gain=0.0, tree_seed=1, agg=0)
    assert st == nat.SBAG_EINVAL and p.returncode == 3
    assert "fit" in p.stdout and "java/lang/IllegalArgumentException" in p.stdout


def test_c_driver_under_host_asan(tmp_path):
    """The whole host side (C ABI, orchestration, ingest, predict planning) under
    AddressSanitizer + UBSan (tests/c/abi_driver_asan; device code is not sanitized):
    a classifier fit + transform and a sampled-split regression fit, no reports."""
    from c_abi_util import DRIVER_ASAN

    env = {"ASAN_OPTIONS": "detect_leaks=0:verify_asan_link_order=0:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}
    X, y = sb.load_libsvm(os.path.join(DATA, "vehicle.svm"))
    p, st, trees, subs, pred = run_driver(
        tmp_path, X, y, [0, 300, 846], replacement=1, ratio=0.7, seed=5, lb=0, le=4,
        sub_ratio=0.7, bug_compat=1, depth=5, bins=32, min_inst=1, impurity=nat.IMPURITY_GINI,
        min_gain=0.0, tree_seed=nat.DT_SEED_CLASSIFIER, agg=nat.AGG_MODE, driver=DRIVER_ASAN,
        env=env)
    assert p.returncode == 0 and st == 0, p.stdout + p.stderr[-3000:]
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr
    rng = np.random.default_rng(9)
    Xr = np.round(rng.normal(size=(20000, 5)), 2)
    yr = rng.integers(-100, 100, 20000) / 4
    p, st, *_ = run_driver(
        tmp_path, Xr, yr, [0, 20000], replacement=1, ratio=1.0, seed=3, lb=2, le=4, sub_ratio=1.0,
        bug_compat=1, depth=6, bins=16, min_inst=2, impurity=nat.IMPURITY_VARIANCE, min_gain=0.0,
        tree_seed=nat.DT_SEED_REGRESSOR, agg=nat.AGG_MEAN, driver=DRIVER_ASAN, env=env)
    assert p.returncode == 0 and st == 0, p.stdout + p.stderr[-3000:]
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr


def test_c_gbm_driver_matches_oracle_gbm(tmp_path):
    """GBMRegressor's boosting loop from plain C through the shim core (SbagNative.sample /
    fitBooster / forestNodes / predict) against the oracle's
    restatement of GBMRegressor.train: every booster and F(x) bit-exact."""
    X, y = sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))
    X = np.asarray(X, np.float64)
    L, lr, seed = 5, 0.1, oracle.DEFAULT_SEED_GBM_REGRESSOR
    w, subs, trees, const = oracle.gbm_regressor_fit(X, y, num_base_learners=L, learning_rate=lr,
                                                     replacement=True, subspace_ratio=0.7,
                                                     seed=seed, max_depth=4)
    p, st, ctrees, pred = run_gbm_driver(tmp_path, X, y, subs, L=L, lr=lr, replacement=1,
                                         ratio=1.0, seed=seed, depth=4, bins=32,
                                         tree_seed=nat.DT_SEED_REGRESSOR)
    assert st == 0, p.stdout + p.stderr
    for m, (nodes, _) in enumerate(trees):
        assert ctrees[m].shape[0] == len(nodes), f"booster {m}"
        for k, f in enumerate(FIELDS):
            assert (ctrees[m][:, k] == nodes[f].astype(np.float64)).all(), f"booster {m} {f}"
    np.testing.assert_array_equal(pred, oracle.gbm_predict(w, subs, trees, const, X))


THREAD_CASES = [
    # (data, label transform, partitions, impurity, agg): the gini engine, the integer
    # variance engine (integral labels) and the fp64 engine (labels / 10)
    ("vehicle.svm", None, [0, 300, 846], nat.IMPURITY_GINI, nat.AGG_MODE),
    ("cpusmall.svm", None, [0, 4000, 8192], nat.IMPURITY_VARIANCE, nat.AGG_MEAN),
    ("cpusmall.svm", 10.0, [0, 2000, 5000, 8192], nat.IMPURITY_VARIANCE, nat.AGG_MEAN),
]


@pytest.mark.parametrize("case", range(len(THREAD_CASES)))
def test_c_threads_concurrent_fits_equal_serial(tmp_path, case):
    """CrossValidator.setParallelism(4) (BaggingRegressorSuite.scala:38-43) from plain C:
    four pthreads fit + predict at once on one shared context, then on four contexts, then
    with one thread's SBAG_EINVAL -- every forest and prediction byte-equal to the serial
    run, the error only in the failing thread's sbag_last_error()."""
    name, div, part, imp, agg = THREAD_CASES[case]
    X, y = sb.load_libsvm(os.path.join(DATA, name))
    if div:
        y = y / div
    p = run_threads(tmp_path, X, y, part, seed=7 + case, depth=6, bins=32, impurity=imp, agg=agg)
    assert p.returncode == 0, p.stdout + p.stderr[-3000:]
    for mode in ("shared", "separate", "errors-shared", "errors-separate"):
        assert f"ok {mode}:" in p.stdout, p.stdout
    assert "java/lang/IllegalArgumentException" in p.stdout


def test_c_threads_under_host_asan(tmp_path):
    """The concurrent driver over the host-ASan/UBSan build of libsbag: the per-context
    lock, the thread-local error and the worker pools raced by four threads, no reports."""
    from c_abi_util import THREADS_ASAN

    env = {"ASAN_OPTIONS": "detect_leaks=0:verify_asan_link_order=0:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}
    X, y = sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))
    logdir = os.path.join(ROOT, "gpurun_out", "asan_threads")
    os.makedirs(logdir, exist_ok=True)
    for modes in ("setup-only", "shared,errors-shared", "separate", "errors-separate"):
        p = run_threads(tmp_path, X, y / 10.0, [0, 2000, 5000, 8192], seed=3, depth=5, bins=16,
                        impurity=nat.IMPURITY_VARIANCE, agg=nat.AGG_MEAN, driver=THREADS_ASAN,
                        env=env, modes=modes)
        with open(os.path.join(logdir, modes.replace(",", "+") + ".log"), "w") as f:
            f.write(f"rc {p.returncode}\n--- stdout\n{p.stdout}\n--- stderr\n{p.stderr}")
        assert p.returncode == 0, (modes, p.stdout, p.stderr[:4000], p.stderr[-1500:])
        assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr
        assert p.stdout.count("ok ") == modes.count(",") + 1, p.stdout
