"""Throughput of GBMRegressor.fit on synthetic rows: every boosting
iteration is one Poisson bag + one DecisionTreeRegressor on fp64 pseudo-residuals, fitted
by the booster engine (sbag_fit_booster, Spark's row-order fp64 sums).  Prints one JSON
line per shape.  Not part of bench.py (the headline is the bagging fit).

usage: python3 scripts/bench_gbm.py [--rows N] [--features F] [--learners L] [--depth D]
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
a = ap.parse_args()
for n in a.rows:
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
