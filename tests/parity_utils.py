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
