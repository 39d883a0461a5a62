"""A C3-sized fit on continuous features (VERDICT r03 "per-replica binning" gap): 10M x 100
rows whose features take thousands of distinct values each, so every replica's thresholds
come from its own split-finding sample (Spark's findSplits per bagged subbag) and
the engine materializes per-replica bins (splitting the learner range when they exceed the
device budget).  Same tree parameters as C3: 128 learners, depth 8, maxBins 32, P = 128,
Poisson(1) bags, dyadic labels.  Prints one JSON line.  Not part of bench.py.

usage: python3 scripts/bench_continuous.py [--rows N] [--learners L]
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
nat = sb._native

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--features", type=int, default=100)
ap.add_argument("--learners", type=int, default=128)
a = ap.parse_args()
N, F, L = a.rows, a.features, a.learners

t0 = time.perf_counter()
rng = np.random.default_rng(20261017)
blk = min(N, 1_000_000)
B = np.round(rng.standard_normal((blk, F), dtype=np.float32) * 300).astype(np.float64) / 8
X = np.empty((N, F))
for k in range(0, N, blk):  # tiles of one block, each shifted: thousands of distinct values
    n = min(blk, N - k)
    X[k:k + n] = B[:n] + (k // blk) / 16.0
y = np.round((X[:, 0] * 0.37 - X[:, 1] * 1.3 + X[:, 2] * 0.05) * 16) / 16  # dyadic
t1 = time.perf_counter()
print(f"[continuous] data {t1 - t0:.1f} s", file=sys.stderr, flush=True)
ctx = nat.default_context(0)
ds = nat.DeviceDataset.from_numpy(X, y, ctx)
del X
t2 = time.perf_counter()
print(f"[continuous] ingest {t2 - t1:.1f} s", file=sys.stderr, flush=True)
part = [round(i * N / 128) for i in range(129)]


def fit(lend):
    return nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=-1395689524, learner_begin=0,
                   learner_end=lend, partition_offsets=part, max_depth=8, max_bins=32,
                   impurity=nat.IMPURITY_VARIANCE)


fit(2).free()  # warm
t3 = time.perf_counter()
f = fit(L)
t4 = time.perf_counter()
tm = f.timing()
nodes = sum(len(f.tree(i)[0]) for i in range(L))
f.free()
ds.free()
print(json.dumps({"rows": N, "features": F, "learners": L, "depth": 8, "max_bins": 32,
                  "data": "continuous: ~2400-38000 distinct values per feature, per-replica thresholds",
                  "fit_ms": round(1e3 * (t4 - t3), 1),
                  "estimator_rows_per_s": round(L * N / (t4 - t3), 1),
                  "ingest_s": round(t2 - t1, 1), "nodes": nodes,
                  "breakdown_ms": {k: round(v, 2) for k, v in tm.items() if k.endswith("_ms")}}),
      flush=True)
