"""Throughput of GBMRegressor.fit on synthetic rows: every boosting
iteration is one Poisson bag + one DecisionTreeRegressor on fp64 pseudo-residuals, fitted
by the booster engine (sbag_fit_booster, Spark's row-order fp64 sums).  Prints one JSON
line per shape.  Not part of bench.py (the headline is the bagging fit).

usage: python3 scripts/bench_gbm.py [--rows N] [--features F] [--learners L] [--depth D]
       python3 scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5
(--synthetic: the rows are the device generator's codes (k_synth, as bench.py), so no host
matrix is ingested; the loop is GBMRegressor.train's for the squared loss at learning rate
0.5 -- Poisson(1) bag, booster on the residuals, prediction, residual update -- driven
through the native calls, each booster and its prediction timed.)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import sbag_loader  # noqa: E402

sb = sbag_loader.load()

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, nargs="+", default=[100_000, 1_000_000])
ap.add_argument("--features", type=int, default=20)
ap.add_argument("--learners", type=int, default=10)
ap.add_argument("--depth", type=int, default=5)
ap.add_argument("--synthetic", action="store_true")
a = ap.parse_args()


def synthetic_line(n):
    nat = sb._native
    ctx = nat.default_context(0)
    ds = nat.DeviceDataset.synthetic(n, a.features, seed=20261015, ctx=ctx)
    y = ds.labels() * 1.1 + 0.3  # real-valued labels
    counts = nat.sample(ctx, True, 1.0, 1234, 0, a.learners, n, None)
    sub = np.arange(a.features, dtype=np.int32)
    res = y.copy()
    f = nat.fit_booster(ctx, ds, res, counts[0], sub, max_depth=a.depth, max_bins=32)  # warm
    f.free()
    fit_ms, pred_ms = [], []
    t_all = time.perf_counter()
    for m in range(a.learners):
        t0 = time.perf_counter()
        f = nat.fit_booster(ctx, ds, res, counts[m], sub, max_depth=a.depth, max_bins=32)
        t1 = time.perf_counter()
        p = nat.predict_dataset(ctx, f, ds, nat.AGG_MEAN)
        t2 = time.perf_counter()
        bd = {k: round(v, 2) for k, v in f.timing().items() if k.endswith("_ms") and v}
        f.free()
        res = res - 0.5 * p
        fit_ms.append(1e3 * (t1 - t0))
        pred_ms.append(1e3 * (t2 - t1))
    dt = time.perf_counter() - t_all
    ds.free()
    print(json.dumps({"rows": n, "features": a.features, "boosters": a.learners, "depth": a.depth,
                      "data": "device synthetic codes, labels 1.1 y + 0.3", "fit_s": round(dt, 3),
                      "ms_per_booster": round(1e3 * dt / a.learners, 2),
                      "booster_fit_ms": round(sum(fit_ms) / len(fit_ms), 2),
                      "predict_ms": round(sum(pred_ms) / len(pred_ms), 2), "breakdown_last": bd,
                      "rows_x_boosters_per_s": round(n * a.learners / dt, 1)}), flush=True)


for n in a.rows:
    if a.synthetic:
        synthetic_line(n)
        continue
    rng = np.random.default_rng(7)
    X = rng.integers(0, 32, size=(n, a.features)).astype(np.float64)
    y = X[:, 0] * 0.37 - X[:, 1] * 1.3 + rng.standard_normal(n)  # real-valued labels
    est = sb.GBMRegressor().setBaseLearner(sb.DecisionTreeRegressor().setMaxDepth(a.depth))
    params = {"numBaseLearners": a.learners, "learningRate": 0.5, "loss": "squared",
              "replacement": True, "sampleRatio": 1.0, "subspaceRatio": 1.0}
    frame = sb.Frame(X, y)
    est.fit(sb.Frame(X[:1000], y[:1000]), params=params)  # warm the context and kernels
    t0 = time.perf_counter()
    model = est.fit(frame, params=params)
    dt = time.perf_counter() - t0
    print(json.dumps({"rows": n, "features": a.features, "boosters": len(model.models),
                      "depth": a.depth, "fit_s": round(dt, 3),
                      "ms_per_booster": round(1e3 * dt / max(1, len(model.models)), 2),
                      "rows_x_boosters_per_s": round(n * len(model.models) / dt, 1)}), flush=True)
