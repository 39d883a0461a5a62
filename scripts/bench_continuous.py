"""A C3-sized fit on continuous features (bench.py's `continuous_features` line, standalone):
10M x 100 rows whose features take thousands of distinct values each, so every replica's
thresholds come from its own split-finding sample (Spark's findSplits per bagged subbag,
SURVEY H8) and the engine materializes per-replica bins.  Same tree parameters as C3: 128
learners, depth 8, maxBins 32, P = 128, Poisson(1) bags, dyadic labels.  Prints one JSON line.

usage: python3 scripts/bench_continuous.py [--rows N] [--features F] [--learners L] [--steps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import sbag_loader  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--features", type=int, default=100)
ap.add_argument("--learners", type=int, default=128)
ap.add_argument("--steps", type=int, default=1)
a = ap.parse_args()
nat = sbag_loader.load()._native
ctx = nat.default_context(0)
part = [round(i * a.rows / 128) for i in range(129)]
print(json.dumps(bench.continuous_fit(nat, ctx, a.rows, a.features, a.learners, 8, 32, part,
                                      steps=a.steps)), flush=True)
