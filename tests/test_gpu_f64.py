"""GPU: bagging regression on arbitrary fp64 labels.

The reference accepts any Double label (ml/regression/BaggingRegressor.scala:146-150 selects
the label column as is; DecisionTreeRegressor sums count, y, y^2 per exploded row in row
order, RandomForest's DTStatsAggregator.update).  Labels that are not dyadic fixed point
take the engine's row-order fp64 path (sbag_f64s.hip).  Spark sums each partition's rows in
row order and merges the partitions' aggregates with reduceByKey (RandomForest.findBestSplits);
the merge order is the shuffle's, and partition order is one order Spark produces.  The
oracle and the engine both follow it (round 6: k_fb_psum / k_fb_pmerge; before, the engine
and the oracle summed a node's rows in one row order, which no Spark run with P > 1 does), so
the trees are bit-exact in every field at every P.
"""
import os

import numpy as np
import pytest

import oracle
from conftest import DATA
from parity_utils import assert_forest_equal, assert_tree_equal, oracle_forest

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu

SEED_REG = oracle.DEFAULT_SEED_REGRESSOR


@pytest.fixture(scope="module")
def ctx():
    return sb.default_context(0)


@pytest.fixture(scope="module")
def cpusmall():
    return sb.load_libsvm(os.path.join(DATA, "cpusmall.svm"))


def _fit_both(ctx, X, y, L, *, replacement=True, ratio=1.0, seed=SEED_REG, depth=5, bins=32,
              part=None, min_inst=1, min_gain=0.0):
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    try:
        forest = nat.fit(ctx, ds, replacement=replacement, sample_ratio=ratio, seed=seed,
                         learner_begin=0, learner_end=L, partition_offsets=part, max_depth=depth,
                         max_bins=bins, min_instances_per_node=min_inst, min_info_gain=min_gain,
                         impurity=nat.IMPURITY_VARIANCE)
    finally:
        ds.free()
    N, F = X.shape
    off = part if part is not None else [0, N]
    counts = oracle.bag(replacement, ratio, 0, L, seed, off, N)
    subs = [oracle.subspace(ratio, F, seed + i) for i in range(L)]
    orf = oracle_forest(X, y, counts, subs, depth, bins, False, min_inst, min_gain, part=part)
    return forest, orf


@pytest.mark.parametrize("label", ["y/10", "y*pi"])
@pytest.mark.parametrize("depth", [5, 10])
def test_cpusmall_nondyadic_labels_bit_exact(ctx, cpusmall, label, depth):
    """cpusmall with labels y/10 and y*pi, 10 learners, P = 1."""
    X, y = cpusmall
    y2 = y / 10 if label == "y/10" else y * np.pi
    forest, orf = _fit_both(ctx, X, y2, 10, depth=depth)
    assert_forest_equal(forest, orf)
    pred = nat.predict(ctx, forest, X, nat.AGG_MEAN)
    want = oracle.predict(orf, X)
    np.testing.assert_allclose(pred, want, rtol=1e-5, atol=0)
    assert (pred == want).all()  # the same sums in the same order: bit-exact in practice


def test_cpusmall_nondyadic_subspace_bernoulli(ctx, cpusmall):
    """Without replacement at ratio 0.7: Bernoulli bags and a 0.7 subspace (H1)."""
    X, y = cpusmall
    forest, orf = _fit_both(ctx, X, y * 0.1 + 1e-3, 6, replacement=False, ratio=0.7, depth=7)
    assert_forest_equal(forest, orf)


def test_min_instances_and_gain_nondyadic(ctx, cpusmall):
    X, y = cpusmall
    y2 = np.sqrt(y + 1.0)
    forest, orf = _fit_both(ctx, X, y2, 4, depth=8, min_inst=5, min_gain=0.01)
    assert_forest_equal(forest, orf)


def test_partitions_p3_bit_exact(ctx):
    """P = 3 partitions: every partition's rows summed in row order, the partials merged in
    partition order (one execution of Spark's reduceByKey) -- bit-exact in every field."""
    rng = np.random.default_rng(7)
    N, F = 9000, 6
    X = np.round(rng.normal(size=(N, F)), 2)
    y = rng.normal(size=N) * 3.7 + 0.1
    part = [0, 2500, 6100, N]
    forest, orf = _fit_both(ctx, X, y, 5, depth=6, part=part)
    assert_forest_equal(forest, orf)


@pytest.mark.parametrize("part", [[0, 1000, 3000, 5000, 8192], [0, 0, 4000, 4000, 8192],
                                  [round(i * 8192 / 64) for i in range(65)]],
                         ids=["p4", "empty-partitions", "p64"])
@pytest.mark.parametrize("depth", [4, 10])
def test_cpusmall_nondyadic_partitions_bit_exact(ctx, cpusmall, part, depth):
    """cpusmall with labels y*pi over several partitions -- uneven, empty ones (their
    partials add +0.0), and 64 of them (most (node, partition) runs of a deep node are empty
    or a few entries long): bit-exact against the oracle's per-partition sums, and the
    predictions equal."""
    X, y = cpusmall
    forest, orf = _fit_both(ctx, X, y * np.pi, 6, depth=depth, part=part)
    assert_forest_equal(forest, orf)
    assert (nat.predict(ctx, forest, X, nat.AGG_MEAN) == oracle.predict(orf, X)).all()


def test_partition_order_is_visible(ctx, cpusmall):
    """The same bags fitted as 1 and as 4 partitions give different fp64 statistics (the
    merge order shows in the sums), each bit-exact against its own oracle run."""
    X, y = cpusmall
    N = len(y)
    y2 = y * np.pi * 1e3 + 0.1
    part = [0, 1000, 3000, 5000, N]
    ds = nat.DeviceDataset.from_numpy(X, y2, ctx)
    try:
        fits = [nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                        learner_end=4, partition_offsets=p, max_depth=8, max_bins=32,
                        impurity=nat.IMPURITY_VARIANCE) for p in (None, part)]
    finally:
        ds.free()
    # Poisson bags depend on the partitions (seed + i + p): draw the P = 4 bags, fit both ways
    counts = oracle.bag(True, 1.0, 0, 4, SEED_REG, part, N)
    subs = [oracle.subspace(1.0, X.shape[1], SEED_REG + i) for i in range(4)]
    assert_forest_equal(fits[1], oracle_forest(X, y2, counts, subs, 8, 32, False, part=part))
    one = oracle_forest(X, y2, counts, subs, 8, 32, False)
    four = oracle_forest(X, y2, counts, subs, 8, 32, False, part=part)
    assert any(not np.array_equal(one.tree(t)[1], four.tree(t)[1]) or len(one.tree(t)[0]) != len(four.tree(t)[0])
               for t in range(4))


def test_sampled_split_finding_nondyadic(ctx):
    """Subbags above max(maxBins^2, 10^4) rows: thresholds from Spark's split-finding
    sample, row-order fp64 sums."""
    rng = np.random.default_rng(11)
    N, F = 26000, 4
    X = np.round(rng.normal(size=(N, F)), 3)
    X[rng.random((N, F)) < 0.15] = 0.0
    y = np.exp(rng.normal(size=N))
    forest, orf = _fit_both(ctx, X, y, 3, depth=6, bins=16, part=[0, 12000, N])
    assert_forest_equal(forest, orf)


def test_forced_f64_path_equals_integer_path_on_dyadic_labels(ctx, cpusmall, monkeypatch):
    """On dyadic labels both engines' sums are exact, so the row-order fp64 path
    (SBAG_F64=1) must give the integer engine's trees bit for bit."""
    X, y = cpusmall
    a, _ = _fit_both(ctx, X, y, 6, depth=9)
    monkeypatch.setenv("SBAG_F64", "1")
    import importlib  # noqa: F401  (the env var is read per process by the library)
    b, orf = _fit_both(ctx, X, y, 6, depth=9)
    assert_forest_equal(b, orf)
    for t in range(6):
        (na, sa), (nb, sb_) = a.tree(t), b.tree(t)
        assert na.tobytes() == nb.tobytes() and (sa == sb_).all()


def test_synthetic_u8_codes_nondyadic(ctx):
    """The bench workload's shape (32-level u8 features, shared bins) with real-valued
    labels, 8 learners over 8 partitions."""
    N, F = 200_000, 20
    X, yk = oracle.synth(N, F, 20261015, 0)
    y = yk * 1.1 + 0.3
    part = [i * N // 8 for i in range(9)]
    forest, orf = _fit_both(ctx, X.astype(np.float64), y, 8, depth=8, part=part)
    assert_forest_equal(forest, orf)


def test_api_accepts_real_labels(cpusmall):
    """BaggingRegressor.fit on a real-valued label column through the Python API."""
    X, y = cpusmall
    y2 = y / 7.0
    model = (sb.BaggingRegressor().setBaseLearner(sb.DecisionTreeRegressor())
             .setNumBaseLearners(4).setReplacement(True)
             .setSampleRatio(0.9)).fit(sb.Frame(X, y2))
    seed = SEED_REG
    counts = oracle.bag(True, 0.9, 0, 4, seed, [0, len(y)], len(y))
    subs = [oracle.subspace(0.9, X.shape[1], seed + i) for i in range(4)]
    orf = oracle.fit(X, y2, counts, subs, max_depth=5, max_bins=32)
    np.testing.assert_allclose(model.transform(X), oracle.predict(orf, X), rtol=1e-5, atol=0)


def test_nonfinite_labels_rejected(ctx, cpusmall):
    X, y = cpusmall
    y2 = y / 10
    y2[5] = np.inf
    ds = nat.DeviceDataset.from_numpy(X, y2, ctx)
    try:
        with pytest.raises(sb.IllegalArgumentException):
            nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=1, learner_begin=0,
                    learner_end=2, max_depth=3, impurity=nat.IMPURITY_VARIANCE)
    finally:
        ds.free()


def _fit(ctx, X, y, L, depth, part=None, **kw):
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    try:
        f = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                    learner_end=L, partition_offsets=part, max_depth=depth, max_bins=32,
                    impurity=nat.IMPURITY_VARIANCE, **kw)
    finally:
        ds.free()
    return f


@pytest.mark.parametrize("case", ["cpusmall_pi", "cpusmall_sqrt", "ties", "tiny_spread",
                                  "cpusmall_pi_p4", "ties_p4"])
def test_screened_engine_equals_unscreened(ctx, cpusmall, monkeypatch, case):
    """The screened fp64 engine (sbag_f64s.hip: splits chosen from the integer histograms
    of the labels' fixed-point image under a rigorous bound, only the chosen feature summed
    in row order) gives the unscreened engine's trees (SBAG_F64_SCREEN=0: every feature of
    every node in row order) byte for byte, including datasets built to defeat the screen:
    duplicated columns (exact ties) and labels whose spread is a few ulps."""
    X, y = cpusmall
    part = [0, 1000, 3000, 5000, len(y)] if case.endswith("_p4") else None
    if case.startswith("cpusmall_pi"):
        y2 = y * np.pi
    elif case == "cpusmall_sqrt":
        y2 = np.sqrt(y + 0.5)
    elif case.startswith("ties"):
        X = np.concatenate([X, X[:, :4]], axis=1)  # every split of the first 4 columns ties
        y2 = y / 3.0
    else:
        y2 = 1.0 + (y - y.mean()) * 1e-13  # gains at the rounding level: the screen must defer
    a = _fit(ctx, X, y2, 6, 9, part)
    ta = a.timing()
    monkeypatch.setenv("SBAG_F64_SCREEN", "0")
    b = _fit(ctx, X, y2, 6, 9, part)
    tb = b.timing()
    # the exact fallback both ways (one partition): every flagged node walked in row order by
    # one wave per (node, feature group) (k_f64_hist), and every flagged node's tasks per
    # (node, feature) (the default splits them by node size, SBAG_F64_WALK_MAX); several
    # partitions always take the per-partition tasks
    monkeypatch.setenv("SBAG_F64_FALLBACK", "hist")
    c = _fit(ctx, X, y2, 6, 9, part)
    monkeypatch.setenv("SBAG_F64_FALLBACK", "chain")
    d = _fit(ctx, X, y2, 6, 9, part)
    # and the scatter gathering y[row] instead of reading the labels carried with the entries
    monkeypatch.delenv("SBAG_F64_SCREEN")
    monkeypatch.delenv("SBAG_F64_FALLBACK")
    monkeypatch.setenv("SBAG_F64_NO_CARRY", "1")
    e = _fit(ctx, X, y2, 6, 9, part)
    for t in range(6):
        (na, sa), (nb, sb_), (nc, sc), (nd, sd), (ne, se) = a.tree(t), b.tree(t), c.tree(t), d.tree(t), e.tree(t)
        assert na.tobytes() == nb.tobytes() == nc.tobytes() == nd.tobytes() == ne.tobytes(), f"tree {t}"
        assert sa.tobytes() == sb_.tobytes() == sc.tobytes() == sd.tobytes() == se.tobytes()
    assert tb["exact_fallbacks"] >= ta["exact_fallbacks"]
    if case in ("cpusmall_pi", "cpusmall_sqrt", "cpusmall_pi_p4"):
        assert ta["exact_fallbacks"] < tb["exact_fallbacks"] / 2  # the screen decides most nodes
    if case.startswith("ties"):
        assert ta["exact_fallbacks"] > 0
    if part is not None:
        N, F = X.shape
        counts = oracle.bag(True, 1.0, 0, 6, SEED_REG, part, N)
        subs = [oracle.subspace(1.0, F, SEED_REG + i) for i in range(6)]
        assert_forest_equal(a, oracle_forest(X, y2, counts, subs, 9, 32, False, part=part))


def test_c3_shape_nondyadic_screened(ctx):
    """The bench's real-valued-label line at 1/10 of its rows: 1M x 100 synthetic u8 codes,
    labels 1.1 y + 0.3, 16 learners, depth 8, P = 128 -- every tree bit-exact against the
    oracle (row-order fp64 sums) and almost every node decided by the screen."""
    N, F, L = 1_000_000, 100, 16
    X, yk = oracle.synth(N, F, 20261015, 0)
    y = yk * 1.1 + 0.3
    part = [round(i * N / 128) for i in range(129)]
    forest, orf = _fit_both(ctx, X.astype(np.float64), y, L, depth=8, part=part)
    assert_forest_equal(forest, orf)
    t = forest.timing()
    nodes = sum(len(forest.tree(i)[0]) for i in range(L))
    assert t["exact_fallbacks"] <= 0.02 * nodes, (t["exact_fallbacks"], nodes)


def test_bucket_budget_chunks_equal_one_launch(ctx, cpusmall, monkeypatch):
    """The decided nodes' bucketing tasks run in chunks when their buckets exceed a budget
    (the C4 shard's root: 73 GB at once); the chunked fit equals the one-launch fit byte for
    byte, and the oracle."""
    X, y = cpusmall
    y2 = y * np.pi
    a = _fit(ctx, X, y2, 4, 7)
    monkeypatch.setenv("SBAG_F64_BUCKET_BUDGET", "3000")  # a few nodes per chunk
    b = _fit(ctx, X, y2, 4, 7)
    for t in range(4):
        (na, sa), (nb, sb_) = a.tree(t), b.tree(t)
        assert na.tobytes() == nb.tobytes(), f"tree {t}"
        assert sa.tobytes() == sb_.tobytes()
    N, F = X.shape
    counts = oracle.bag(True, 1.0, 0, 4, SEED_REG, [0, N], N)
    subs = [oracle.subspace(1.0, F, SEED_REG + i) for i in range(4)]
    assert_forest_equal(b, oracle_forest(X, y2, counts, subs, 7, 32, False))


def test_c3_full_nondyadic_engines_agree(ctx, monkeypatch):
    """The bench's real-valued-label fit at full size (10M x 100, 128 learners, depth 8,
    P = 128), where the oracle cannot follow: the default engine (screen, routing scatter,
    column-ordered and XCD-dispatched tasks, per-partition sums) gives the same trees byte for
    byte as (a) the same screen with tasks in node order and pieces in order and
    (b) the unscreened engine, every feature of every node summed per partition and merged
    (k_fb_psum / k_fb_pmerge over every (node, feature))."""
    N, F, L = 10_000_000, 100, 128
    ds = nat.DeviceDataset.synthetic(N, F, seed=20261015, ctx=ctx)
    try:
        ds.set_labels(ds.labels() * 1.1 + 0.3)
        part = [round(i * N / 128) for i in range(129)]

        def fit():
            return nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=-1395689524,
                           learner_begin=0, learner_end=L, partition_offsets=part, max_depth=8,
                           max_bins=32, impurity=nat.IMPURITY_VARIANCE)

        a = fit()
        for k in ("SBAG_F64_TASK_ORDER", "SBAG_F64_XCD_ORDER"):
            monkeypatch.setenv(k, "0")
        b = fit()
        for k in ("SBAG_F64_TASK_ORDER", "SBAG_F64_XCD_ORDER"):
            monkeypatch.delenv(k)
        monkeypatch.setenv("SBAG_F64_SCREEN", "0")
        c = fit()
    finally:
        ds.free()
    ta, tc = a.timing(), c.timing()
    assert ta["exact_fallbacks"] < tc["exact_fallbacks"] / 20, (ta["exact_fallbacks"], tc["exact_fallbacks"])
    for t in range(L):
        (na, sa), (nb, sb_), (nc, sc) = a.tree(t), b.tree(t), c.tree(t)
        assert na.tobytes() == nb.tobytes() == nc.tobytes(), f"tree {t}"
        assert sa.tobytes() == sb_.tobytes() == sc.tobytes(), f"tree {t} stats"
    for f in (a, b, c):
        f.free()


@pytest.mark.parametrize("part", [None, [0, 7000, 7000, 20_000]], ids=["p1-chains", "p3-psum"])
def test_chain_windows_many_bins_large_counts(ctx, part):
    """Spark's row-order sums with every row drawn 9 times (k_fb_chainx's several draw
    windows per stage at P = 1), maxBins 255 on features with ~1000 distinct values (up to 255
    chains per task; at P > 1, k_fb_psum's one run per wave with four (run, bin) keys per lane
    and 9 draws per entry in its draw loop), fp64 labels, one booster -- bit-exact against the
    oracle."""
    rng = np.random.default_rng(29)
    n, f = 20_000, 6
    X = np.round(rng.normal(size=(n, f)) * 150) / 7
    lab = rng.normal(size=n) * 3.3 + X[:, 2] * 0.01
    counts = np.full(n, 9, np.uint8)
    counts[rng.random(n) < 0.1] = 0
    sub = np.arange(f, dtype=np.int32)
    ds = nat.DeviceDataset.from_numpy(X, np.zeros(n), ctx)
    try:
        fb = nat.fit_booster(ctx, ds, lab, counts, sub, partition_offsets=part, max_depth=6,
                             max_bins=255)
    finally:
        ds.free()
    orf = oracle.fit(X, lab, counts[None, :], [sub], max_depth=6, max_bins=255, part=part)
    assert_tree_equal(fb, 0, orf, 0)


def test_wide_addressing_equals_buffer_path(ctx, cpusmall, monkeypatch):
    """k_fb_scatter's 64-bit-pointer variant (taken from 2^28 rows on; SBAG_F64_WIDE=1 forces
    it) gives the buffer-resource variant's trees byte for byte, and the oracle's."""
    X, y = cpusmall
    y2 = y * np.pi
    a = _fit(ctx, X, y2, 4, 7)
    monkeypatch.setenv("SBAG_F64_WIDE", "1")
    b = _fit(ctx, X, y2, 4, 7)
    monkeypatch.setenv("SBAG_F64_NO_CARRY", "1")  # the labels gathered by row, 64-bit
    c = _fit(ctx, X, y2, 4, 7)
    for t in range(4):
        (na, sa), (nb, sb_), (nc, sc) = a.tree(t), b.tree(t), c.tree(t)
        assert na.tobytes() == nb.tobytes() == nc.tobytes(), f"tree {t}"
        assert sa.tobytes() == sb_.tobytes() == sc.tobytes()
    N, F = X.shape
    counts = oracle.bag(True, 1.0, 0, 4, SEED_REG, [0, N], N)
    subs = [oracle.subspace(1.0, F, SEED_REG + i) for i in range(4)]
    assert_forest_equal(b, oracle_forest(X, y2, counts, subs, 7, 32, False))


def test_fp64_engine_near_the_row_limit(ctx, monkeypatch):
    """fp64 labels up to the engine's explicit limit of 2^30 rows (ADVICE r04 medium lifted
    the old 2^29; ADVICE r05 asked for a limit at the largest tested size): 2^30 - 4096 rows
    take the 64-bit-addressed scatter.  The fp64 engine forced on dyadic labels (SBAG_F64=1)
    must give the integer engine's tree byte for byte -- its row-order fp64 sums of dyadic
    labels are exact."""
    N, F = (1 << 30) - 4096, 2
    ds = nat.DeviceDataset.synthetic(N, F, seed=7, ctx=ctx)
    try:
        part = [round(i * N / 256) for i in range(257)]

        def fit():
            return nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                           learner_end=1, partition_offsets=part, max_depth=3, max_bins=32,
                           impurity=nat.IMPURITY_VARIANCE)

        a = fit()
        monkeypatch.setenv("SBAG_F64", "1")
        b = fit()
    finally:
        ds.free()
    (na, sa), (nb, sb_) = a.tree(0), b.tree(0)
    assert len(na) > 1
    assert na.tobytes() == nb.tobytes()
    assert sa.tobytes() == sb_.tobytes()


def test_fp64_engine_refuses_past_the_row_limit(ctx, monkeypatch):
    """Past 2^30 rows the fp64 engine refuses (SBAG_EUNSUPPORTED) before any work rather than
    run kernels at sizes no test covers; the integer engine still fits those rows."""
    N = (1 << 30) + 64
    ds = nat.DeviceDataset.synthetic(N, 1, seed=7, ctx=ctx)
    try:
        monkeypatch.setenv("SBAG_F64", "1")
        with pytest.raises(nat.SparkException, match="2\\^30"):
            nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                    learner_end=1, max_depth=1, max_bins=8, impurity=nat.IMPURITY_VARIANCE)
    finally:
        ds.free()


def test_fp64_fit_after_integer_fit_on_one_context():
    """Round 6 sizes the fp64 path's entry lists by the largest in-bag count and trims the
    N-entry lists an earlier integer fit left in the context's workspace (so the carried
    labels fit on the C4 shard).  An integer fit, then a real-label fit on the same context,
    must give the real-label fit of a fresh context byte for byte (and so must the integer
    fit run again afterwards, on lists the fp64 fit re-sized)."""
    N, F, L = 100_000, 8, 6
    part = [0, 30_000, 30_000, 64_000, N]

    def fit(c, labels):
        ds = nat.DeviceDataset.synthetic(N, F, seed=11, ctx=c)
        try:
            if labels == "real":
                ds.set_labels(ds.labels() * 1.1 + 0.3)
            return nat.fit(c, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                           learner_end=L, partition_offsets=part, max_depth=7, max_bins=32,
                           impurity=nat.IMPURITY_VARIANCE)
        finally:
            ds.free()

    shared, fresh_r, fresh_i = nat.Context(0), nat.Context(0), nat.Context(0)
    try:
        i1 = fit(shared, "int")
        r1 = fit(shared, "real")
        i2 = fit(shared, "int")
        r0 = fit(fresh_r, "real")
        i0 = fit(fresh_i, "int")
        for t in range(L):
            for a, b in ((r1, r0), (i1, i0), (i2, i0)):
                (na, sa), (nb, sb_) = a.tree(t), b.tree(t)
                assert na.tobytes() == nb.tobytes(), f"tree {t}"
                assert sa.tobytes() == sb_.tobytes(), f"tree {t} stats"
        for f in (i1, r1, i2, r0, i0):
            f.free()
    finally:
        for c in (shared, fresh_r, fresh_i):
            c.close()
