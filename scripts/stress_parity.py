"""Repeat GPU parity cases in one process to catch nondeterminism (debug aid).
usage: python scripts/stress_parity.py [reps]"""
import os
import sys

sys.path.insert(0, "/root/repo")
sys.path.insert(0, "/root/repo/oracle")
sys.path.insert(0, "/root/repo/tests")
import numpy as np

import sbag_loader

sb = sbag_loader.load()
nat = sb._native
import oracle  # noqa: E402
import parity_utils  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
seed = oracle.DEFAULT_SEED_REGRESSOR
F = 5
ctx = sb.default_context(0)
cases = {}
for n_rows, P in [(30000, 3), (16000, 2), (40000, 1)]:
    rng = np.random.default_rng(n_rows + P)
    X = np.round(rng.normal(size=(n_rows, F)), 2)
    X[rng.random((n_rows, F)) < 0.15] = 0.0
    y = (rng.integers(-256, 256, n_rows) / 16).astype(np.float64)
    part = [int(round(i * n_rows / P)) for i in range(P + 1)]
    counts = oracle.bag(True, 1.0, 0, 3, seed, part, n_rows)
    subs = [oracle.subspace(1.0, F, seed + i) for i in range(3)]
    orf = oracle.fit(X, y, counts, subs, max_depth=6, max_bins=32, part=part)
    cases[(n_rows, P)] = (X, y, part, orf)
fails = 0
for rep in range(reps):
    for key, (X, y, part, orf) in cases.items():
        ds = nat.DeviceDataset.from_numpy(X, y, ctx)
        forest = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=seed, learner_begin=0,
                         learner_end=3, partition_offsets=part, max_depth=6, max_bins=32)
        try:
            parity_utils.assert_forest_equal(forest, orf)
        except AssertionError as e:
            fails += 1
            print(rep, key, "FAIL", str(e)[:300], flush=True)
        forest.free()
        ds.free()
print("reps", reps, "fails", fails, flush=True)
