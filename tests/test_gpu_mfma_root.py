"""GPU: the root histogram as an int8 MFMA contraction (sbag_mfma.hip, k_hist_mfma).

With shared identity bins (every feature's codes are its bins, <= 32 of them, no feature
subspace) the root histogram of every replica is counts[R x N] times the one-hot bins of each
feature, plus digit planes of the labels' fixed-point image (and of its square on the exact
path).  Its sums are integers, so the trees must be byte-identical to the LDS-atomic root
(SBAG_ROOT_MFMA=0: k_hist_rl) and to the oracle's restatement of
RandomForest.findBestSplits (ml/ensemble/ensembleParams.scala:113-115)."""
import numpy as np
import pytest

import oracle
from parity_utils import assert_forest_equal, oracle_forest

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu

SEED = oracle.DEFAULT_SEED_REGRESSOR


@pytest.fixture(scope="module")
def ctx():
    return sb.default_context(0)


def _data(N, F, label, seed):
    rng = np.random.default_rng(seed)
    levels = rng.choice([2, 5, 17, 32], size=F)
    X = np.stack([rng.integers(0, levels[f], size=N) for f in range(F)], axis=1).astype(np.float64)
    base = X[:, 0] * 3.0 - X[:, min(1, F - 1)] + rng.integers(-8, 9, size=N)
    if label == "dyadic":  # k' < 2^8: 2 digit planes
        y = base / 4.0
    elif label == "wide":  # k' < 2^16: 3 digit planes
        y = base + rng.integers(-2**14, 2**14, size=N)
    else:  # fp64 labels: the screened engine's approximate image, no squares plane
        y = base * 1.1 + 0.3
    return X, y


def _fit(ctx, X, y, L, depth, monkeypatch, mfma):
    monkeypatch.setenv("SBAG_ROOT_MFMA", "1" if mfma else "0")
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    try:
        f = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED, learner_begin=0,
                    learner_end=L, partition_offsets=None, max_depth=depth, max_bins=32,
                    impurity=nat.IMPURITY_VARIANCE)
    finally:
        ds.free()
    return f


@pytest.mark.parametrize("digits", ["auto", "7"])
@pytest.mark.parametrize("label", ["dyadic", "f64", "wide"])
@pytest.mark.parametrize("N,F,L", [(135_184, 13, 3), (70_000, 9, 40), (200_016, 21, 70)])
def test_mfma_root_equals_lds_root(ctx, monkeypatch, label, N, F, L, digits):
    """Trees byte-identical with the MFMA root and with k_hist_rl's: row counts across
    65536-row slices and ragged 256-row chunks, 8-feature groups with idle waves, one to
    three 32-replica tiles and replica groups split over launches -- with the label image's
    digit planes as the host picks them (balanced int8 base-256 digits of k - midpoint
    whenever they need fewer planes: every case here) and forced to unsigned 7-bit digits
    (SBAG_MFMA_DIGITS=7)."""
    if digits == "7":
        monkeypatch.setenv("SBAG_MFMA_DIGITS", "7")
    X, y = _data(N, F, label, N + F)
    a = _fit(ctx, X, y, L, 6, monkeypatch, True)
    b = _fit(ctx, X, y, L, 6, monkeypatch, False)
    ta, tb = a.timing(), b.timing()
    assert ta["root_ms"] > 0.0 and ta["root_mfma_ops"] > 0.0, ta
    assert tb["root_ms"] == 0.0
    for t in range(L):
        (na, sa), (nb, sb_) = a.tree(t), b.tree(t)
        assert na.tobytes() == nb.tobytes(), f"tree {t}"
        assert sa.tobytes() == sb_.tobytes(), f"tree {t} stats"


@pytest.mark.parametrize("label", ["dyadic", "f64"])
def test_mfma_root_against_oracle(ctx, monkeypatch, label):
    """The MFMA-rooted forest against the oracle, every field bit-exact."""
    N, F, L = 40_000, 7, 4
    X, y = _data(N, F, label, 7)
    forest = _fit(ctx, X, y, L, 7, monkeypatch, True)
    assert forest.timing()["root_ms"] > 0.0
    counts = oracle.bag(True, 1.0, 0, L, SEED, [0, N], N)
    subs = [oracle.subspace(1.0, F, SEED + i) for i in range(L)]
    orf = oracle_forest(X, y, counts, subs, 7, 32, False)
    assert_forest_equal(forest, orf)
