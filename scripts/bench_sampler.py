"""Time the Poisson bag sampler alone (sbag_sample) on C3's shape: 10M rows, 128
learners, P partitions of equal size.  For rocprofv3 / PMC passes over k_poisson4.

usage: python3 scripts/bench_sampler.py [--partitions P] [--reps K]
"""
import argparse
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
ap.add_argument("--learners", type=int, default=128)
ap.add_argument("--partitions", type=int, default=128)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
off = np.linspace(0, a.rows, a.partitions + 1).astype(np.int64)
ctx = nat.Context(0)
for k in range(a.reps):
    t0 = time.perf_counter()
    got = nat.sample(ctx, True, 1.0, -1395689524, 0, a.learners, a.rows, off)
    dt = time.perf_counter() - t0
    print(f"rep {k}: {dt * 1e3:.1f} ms wall incl. device->host copy, mean count "
          f"{got[0].mean():.4f}", flush=True)
ctx.close()
