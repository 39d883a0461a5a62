#!/usr/bin/env python3
"""GBMRegressor.fit on synthetic rows with the booster calls timed apart from the
Python-side work (residuals, BLAS.dot model, predictions) and each booster fit's device
breakdown.  usage: python scripts/gbm_probe.py [rows] [features] [boosters] [depth]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import sbag_loader  # noqa: E402

sb = sbag_loader.load()
nat = sb._native
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
F = int(sys.argv[2]) if len(sys.argv) > 2 else 20
L = int(sys.argv[3]) if len(sys.argv) > 3 else 10
depth = int(sys.argv[4]) if len(sys.argv) > 4 else 5
rng = np.random.default_rng(7)
X = rng.integers(0, 32, size=(n, F)).astype(np.float64)
y = X[:, 0] * 0.37 - X[:, 1] * 1.3 + rng.standard_normal(n)
ctx = nat.default_context(0)
ds = nat.DeviceDataset.from_numpy(X, y, ctx)
counts = nat.sample(ctx, True, 1.0, 1234, 0, L, n, None)
sub = np.arange(F, dtype=np.int32)
res = y.copy()
fits, preds, bds = [], [], []
for m in range(L + 1):
    t0 = time.perf_counter()
    f = nat.fit_booster(ctx, ds, res, counts[m % L], sub, max_depth=depth, max_bins=32)
    t1 = time.perf_counter()
    p = nat.predict_dataset(ctx, f, ds, nat.AGG_MEAN)
    t2 = time.perf_counter()
    tm = f.timing()
    f.free()
    res = res - 0.5 * p
    if m > 0:  # the first call warms the context and workspace
        fits.append(1e3 * (t1 - t0))
        preds.append(1e3 * (t2 - t1))
        bds.append({k: round(v, 2) for k, v in tm.items() if k.endswith("_ms") and v})
print(json.dumps({"rows": n, "features": F, "depth": depth, "fit_ms": [round(v, 2) for v in fits],
                  "predict_ms": [round(v, 2) for v in preds], "breakdown_last": bds[-1]}))
ds.free()
