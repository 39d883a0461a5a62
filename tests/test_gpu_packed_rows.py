"""GPU: per-replica packed rows for the histograms (sbag_host.cpp, k_pack_rows).

With identity bins (the codes are the bins) and feature subspaces, every level's histogram
gathers each entry's row; packed rows hold only the replica's F_r features (in subspace
order), so the gather pulls roundup(F_r) bytes instead of the whole code row.  The packed
bytes are the same bins, so the trees must be byte-identical with and without them
(SBAG_PACK_ROWS=0 / 1), and bit-exact against the oracle's restatement of
HasSubBag.scala:90-106 (mkSubspace) + RandomForest.findBestSplits."""
import numpy as np
import pytest

import oracle
from parity_utils import assert_forest_equal, oracle_forest

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu

SEED = oracle.DEFAULT_SEED_CLASSIFIER


@pytest.fixture(scope="module")
def ctx():
    return sb.default_context(0)


def _data(N, F, classes, seed):
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 32, size=(N, F)).astype(np.float64)
    code = (X[:, 0] * 3 + X[:, min(3, F - 1)] + rng.integers(0, 4, N)).astype(np.int64)
    y = (code % classes).astype(np.float64) if classes else X[:, 1] * 0.25 - X[:, 2] / 8.0
    return X, y


def _fit(ctx, X, y, L, depth, ratio, gini, monkeypatch, pack):
    monkeypatch.setenv("SBAG_PACK_ROWS", "1" if pack else "0")
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    try:
        return nat.fit(ctx, ds, replacement=False, sample_ratio=ratio, seed=SEED, learner_begin=0,
                       learner_end=L, partition_offsets=None, max_depth=depth, max_bins=32,
                       impurity=nat.IMPURITY_GINI if gini else nat.IMPURITY_VARIANCE)
    finally:
        ds.free()


@pytest.mark.parametrize("classes", [0, 5, 64])
@pytest.mark.parametrize("N,F,L,ratio", [(60_001, 37, 6, 0.5), (30_000, 100, 3, 0.3)])
def test_packed_rows_equal_code_rows(ctx, monkeypatch, classes, N, F, L, ratio):
    X, y = _data(N, F, classes, N + F + classes)
    a = _fit(ctx, X, y, L, 7, ratio, classes > 0, monkeypatch, True)
    b = _fit(ctx, X, y, L, 7, ratio, classes > 0, monkeypatch, False)
    for t in range(L):
        (na, sa), (nb, sb_) = a.tree(t), b.tree(t)
        assert na.tobytes() == nb.tobytes(), f"tree {t}"
        assert sa.tobytes() == sb_.tobytes(), f"tree {t} stats"


def test_packed_rows_against_oracle(ctx, monkeypatch):
    N, F, L, C = 20_000, 21, 4, 7
    X, y = _data(N, F, C, 3)
    forest = _fit(ctx, X, y, L, 6, 0.6, True, monkeypatch, True)
    counts = oracle.bag(False, 0.6, 0, L, SEED, [0, N], N)
    subs = [oracle.subspace(0.6, F, SEED + i) for i in range(L)]
    orf = oracle_forest(X, y, counts, subs, 6, 32, True)
    assert_forest_equal(forest, orf)
