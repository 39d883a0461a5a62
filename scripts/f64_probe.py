#!/usr/bin/env python3
"""One C3-shape fit on real-valued labels (the row-order fp64 path), learner halves
serialized, per-level stage times (SBAG_LEVEL_TRACE) and the fit's breakdown.
usage: SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 python scripts/f64_probe.py [rows] [learners] [features]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sbag_loader  # noqa: E402

sb = sbag_loader.load()
nat = sb._native
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
L = int(sys.argv[2]) if len(sys.argv) > 2 else 128
F = int(sys.argv[3]) if len(sys.argv) > 3 else 100
ctx = nat.Context(0)
ds = nat.DeviceDataset.synthetic(N, F, seed=20261015, ctx=ctx)
ds.set_labels(ds.labels() * 1.1 + 0.3)
part = [int(round(i * N / 128)) for i in range(129)]


def fit():
    return nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=-1395689524, learner_begin=0,
                   learner_end=L, partition_offsets=part, max_depth=8, max_bins=32,
                   impurity=nat.IMPURITY_VARIANCE)


fit().free()
t0 = time.perf_counter()
f = fit()
dt = time.perf_counter() - t0
print(json.dumps({"rows": N, "features": F, "learners": L, "fit_ms": round(1000 * dt, 1),
                  "exact_fallbacks": f.timing()["exact_fallbacks"],
                  "breakdown": {k: round(v, 2) for k, v in f.timing().items() if k.endswith("_ms")}}))
f.free()
ds.free()
ctx.close()
