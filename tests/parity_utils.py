"""Shared helpers for the parity tests: run the product (HIP via the C ABI) and
the oracle (CPU restatement) on the same inputs and compare node by node."""
import numpy as np

import oracle

FIELDS = ("id", "left", "right", "feature", "threshold", "prediction", "impurity", "gain")


def oracle_forest(X, y, counts, subspaces, depth, bins, classification, min_inst=1, min_gain=0.0,
                  part=None, dt_seed=None):
    return oracle.fit(X, y, counts, subspaces, max_depth=depth, max_bins=bins,
                      min_instances_per_node=min_inst, min_info_gain=min_gain,
                      classification=classification, part=part, dt_seed=dt_seed)


def assert_tree_equal(native, t, orf, to, rel_tol_pred=0.0):
    """Native tree t against oracle tree to: structure, splits, thresholds, impurities,
    gains, stats bit-exact; regression predictions within rel_tol_pred (0 = bit-exact)."""
    nn, ns = native.tree(t)
    on, os_ = orf.tree(to)
    assert list(native.subspace(t)) == list(orf.subspaces[to]), f"tree {t}: subspace"
    assert len(nn) == len(on), f"tree {t}: {len(nn)} nodes vs oracle {len(on)}"
    for f in FIELDS:
        a, b = nn[f], on[f]
        if f == "prediction" and rel_tol_pred > 0:
            np.testing.assert_allclose(a, b, rtol=rel_tol_pred, atol=0, err_msg=f"tree {t} {f}")
        else:
            same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
            assert same.all(), f"tree {t} field {f}: {a[~same][:5]} vs {b[~same][:5]}"
    assert ns.shape == os_.shape, f"tree {t}: stats shape {ns.shape} vs {os_.shape}"
    assert (ns == os_).all(), f"tree {t}: stats differ"


def assert_forest_equal(native, orf, rel_tol_pred=0.0):
    """Every tree of the native forest against the oracle's, in learner order."""
    L = len(native)
    assert L == orf.nodes.shape[0]
    for t in range(L):
        assert_tree_equal(native, t, orf, t, rel_tol_pred)


def fuzz_case(seed):
    """One randomized parity case of scripts/fuzz_parity.py: (X, y, classification,
    non-dyadic labels, partition offsets, fit params, feature kind)."""
    rng = np.random.default_rng(seed)
    N = int(np.exp(rng.uniform(np.log(2000), np.log(150_000))))
    F = int(rng.choice([1, 3, 12, 40, 64, 65, 100, 140]))
    cls = bool(rng.integers(0, 2))
    kind = rng.choice(["mixed", "u8"])
    sign_rng = np.random.default_rng(seed + 7919)  # (apart, so a seed's other draws stay put)
    if kind == "u8":  # 32-level integer columns: identity codes, the bench's layout
        X = rng.integers(0, 32, size=(N, F)).astype(np.float64)
    else:
        X = np.empty((N, F))
        for f in range(F):
            levels = int(rng.choice([2, 3, 7, 31, 200, 5000]))
            X[:, f] = np.round(rng.normal(size=N) * levels) / 8.0
            X[rng.random(N) < 0.1, f] = 0.0
            if sign_rng.random() < 0.2:  # one sign, no 0.0: a short split-finding sample implies one
                X[:, f] = (np.abs(X[:, f]) + 0.125) * sign_rng.choice([-1.0, 1.0])
    f64 = False
    if cls:
        C = int(rng.choice([2, 3, 5, 9, 17, 33, 64, 80]))
        code = np.floor(np.abs(X[:, 0]) * 3 + np.abs(X[:, min(1, F - 1)])).astype(np.int64)
        y = ((code + rng.integers(0, 4, N)) % C).astype(np.float64)
    else:
        f64 = bool(rng.random() < 0.35)
        y = rng.integers(-400, 400, size=N) / 16.0 + X[:, 0] * 0.25
        if f64:
            y = y * 1.1 + 0.3
    if f64:  # (round 6: fp64 labels over several partitions too -- Spark's per-partition sums;
        # drawn from a stream of their own, so every other draw of a seed stays put)
        prng = np.random.default_rng(seed + 4099)
        P = int(prng.integers(1, 7))
        cuts = np.sort(prng.integers(0, N + 1, size=P - 1))
    else:
        P = int(rng.integers(1, 7))
        cuts = np.sort(rng.integers(0, N + 1, size=P - 1))
    part = [0] + [int(c) for c in cuts] + [N]
    p = dict(L=int(rng.integers(1, 13)), replacement=bool(rng.integers(0, 2)),
             ratio=float(rng.choice([1.0, 0.9, 0.63, 0.5])), depth=int(rng.integers(0, 15)),
             bins=int(rng.choice([2, 5, 16, 32, 32, 64])), min_inst=int(rng.choice([1, 1, 3, 20])),
             min_gain=float(rng.choice([0.0, 0.0, 0.001, 0.05])))
    if not p["replacement"] and p["ratio"] == 1.0:
        p["ratio"] = 0.7
    return X, y, cls, f64, part, p, kind


def fuzz_case_big(seed):
    """--big: 1-3M rows and 16-32 learners, so the fit splits its learner range into two
    halves on two streams and the histograms run at shard-like sizes."""
    rng = np.random.default_rng(seed)
    N = int(rng.integers(1 << 20, 3_000_000))
    F = int(rng.choice([8, 20, 40, 100]))
    cls = bool(rng.integers(0, 2))
    kind = rng.choice(["mixed", "u8"])
    if kind == "u8":
        X = rng.integers(0, 32, size=(N, F)).astype(np.float64)
    else:
        X = np.round(rng.normal(size=(N, F)) * rng.choice([3, 31, 500], size=F)) / 8.0
    f64 = False
    if cls:
        C = int(rng.choice([2, 5, 17, 64]))
        code = np.floor(np.abs(X[:, 0]) * 3 + np.abs(X[:, min(1, F - 1)])).astype(np.int64)
        y = ((code + rng.integers(0, 4, N)) % C).astype(np.float64)
    else:
        f64 = bool(rng.random() < 0.3)
        y = rng.integers(-400, 400, size=N) / 16.0 + X[:, 0] * 0.25
        if f64:
            y = y * 1.1 + 0.3
    if f64:  # (round 6: fp64 labels over several partitions too -- Spark's per-partition sums;
        # drawn from a stream of their own, so every other draw of a seed stays put)
        prng = np.random.default_rng(seed + 4099)
        P = int(prng.integers(1, 9))
        cuts = np.sort(prng.integers(0, N + 1, size=P - 1))
    else:
        P = int(rng.integers(1, 9))
        cuts = np.sort(rng.integers(0, N + 1, size=P - 1))
    part = [0] + [int(c) for c in cuts] + [N]
    p = dict(L=int(rng.choice([16, 24, 32])), replacement=bool(rng.integers(0, 2)),
             ratio=float(rng.choice([1.0, 0.8, 0.5])), depth=int(rng.integers(3, 12)),
             bins=int(rng.choice([16, 32, 64])), min_inst=int(rng.choice([1, 5])),
             min_gain=float(rng.choice([0.0, 0.001])))
    if not p["replacement"] and p["ratio"] == 1.0:
        p["ratio"] = 0.7
    return X, y, cls, f64, part, p, kind
